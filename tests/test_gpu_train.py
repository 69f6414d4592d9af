"""T1 — one training step of each project on the HIP path vs the reference.

The models, optimisers and batch are built exactly as the reference's main()
builds them (seeds.step_models / step_batch; tests/golden/gen_golden.py ran
the reference's own train() on the same inputs).  Checked:
* the returned records (pec/mtc/epc/fdc averages): 1e-3 relative to golden;
* the per-batch printed counts (n_sel, n_pseudo): exact;
* AdamW's first step moves each weight by ~ -lr*sign(grad): the update signs
  agree with the oracle's step (run here on the CPU) on >= 97 % of each
  student's weights and >= 90 % of every tensor (grads whose sign is below fp32 noise can flip — the
  reference's own fp32 gradients are ~2 % from exact, see test_gpu_hourglass);
* teachers after the EMA update equal alpha*teacher + (1-alpha)*student
  (alpha keyed on the epoch) to fp32 rounding;
* BN running statistics: 1e-3 relative.
"""
import os

import numpy as np
import pytest
import torch

import seeds
from oracle import hourglass as OH
from oracle import render as OR
from oracle import step as OS

pytestmark = pytest.mark.gpu
GD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def _flat(x, out):
    if isinstance(x, (list, tuple)):
        for v in x:
            _flat(v, out)
    else:
        out.append(float(x))
    return out


def _factory(k, s, mode):
    from ubpl_amd.hourglass import StackedHourglass
    return StackedHourglass(k, s, mode)


def _run_ours(cfg, flat_adam):
    from ubpl_amd import train as T
    from ubpl_amd.optim import FlatAdamW
    models, emas, optims = seeds.step_models(_factory, cfg, device="cuda")
    if flat_adam:
        optims = [FlatAdamW(m, lr=cfg["lr"], weight_decay=0) for m in models]
    before = [[p.detach().clone() for p in m.parameters()] for m in models + emas]
    loader, args = seeds.step_batch(cfg, OR.kps_heatmap_torch)
    import io
    import contextlib
    buf = io.StringIO()
    with contextlib.redirect_stdout(buf):
        if cfg["project"] == "MT_UBPL":
            rec = T.train_mt_ubpl(loader, models, emas, optims, args)
        elif cfg["project"] == "DualPose_UBPL":
            rec = T.train_dualpose_ubpl(loader, models, emas, optims, args)
        elif cfg["project"] == "MT":
            rec = T.train_mt(loader, models[0], emas[0], optims[0], args)
        else:
            rec = T.train_supervised(loader, models[0], optims[0], args)
    import re
    counts = [[int(a), int(b)] for a, b in re.findall(r"\((\s*\d+)/(\s*\d+)\)", buf.getvalue())]
    return models + emas, before, rec, counts, args


def _run_oracle(cfg):
    models, emas, optims = seeds.step_models(OH.oracle_factory, cfg)
    before = [[p.detach().clone() for p in m.parameters()] for m in models + emas]
    loader, args = seeds.step_batch(cfg, OR.kps_heatmap_torch)
    if cfg["project"] == "MT_UBPL":
        OS.train_mt_ubpl(loader, models, emas, optims, args)
    elif cfg["project"] == "DualPose_UBPL":
        OS.train_dualpose_ubpl(loader, models, emas, optims, args)
    elif cfg["project"] == "MT":
        OS.train_mt(loader, models[0], emas[0], optims[0], args)
    else:
        OS.train_supervised(loader, models[0], optims[0], args)
    return models + emas, before


@pytest.mark.parametrize("case,flat_adam", [("mt_ubpl", True), ("mt_ubpl_e0", False), ("dualpose", True),
                                            ("mt", True), ("sup", False)])
def test_train_step_vs_reference(case, flat_adam):
    torch.set_num_threads(min(32, os.cpu_count() or 1))
    g = np.load(os.path.join(GD, "steps.npz"))
    cfg = seeds.step_cases()[case]
    ours, before, rec, counts, args = _run_ours(cfg, flat_adam)
    np.testing.assert_allclose(_flat(rec, []), g[case + "/records"], rtol=1e-3, atol=1e-9)
    assert np.array_equal(np.array(counts, np.int64).reshape(-1, 2), g[case + "/printed_counts"])
    ref, ref_before = _run_oracle(cfg)
    n_students = cfg["brNum"]
    for mi, (m, r, b0, rb0) in enumerate(zip(ours, ref, before, ref_before)):
        names = [n for n, _ in m.named_parameters()]
        agree_n, total_n = 0, 0
        for n, p, q, p0, q0 in zip(names, m.parameters(), r.parameters(), b0, rb0):
            assert torch.equal(p0.cpu(), q0), (mi, n)          # same seeded init
            du = (p.detach().cpu() - p0.cpu()).double()
            dr = (q.detach() - q0).double()
            if mi < n_students:
                if seeds.bn_cancelled(n) or float(dr.abs().max()) == 0.0:
                    assert float(du.abs().max()) <= 1.01 * args.lr, (mi, n)
                    continue
                same = int(((du > 0) == (dr > 0)).sum())
                agree_n, total_n = agree_n + same, total_n + du.numel()
                assert same >= 0.9 * du.numel(), (mi, n, same / du.numel())
            else:
                # teacher = alpha*teacher + (1-alpha)*student_after_step (utils/parameters.py:6-8),
                # checked on our own tensors (the students were checked against the oracle above)
                s_new = dict(ours[mi - len(ours) // 2].named_parameters())[n].detach().cpu()
                alpha = min(1 - 1 / (args.epo + 1), args.ema_decay)
                a_part, b_part = p0.cpu().double() * alpha, (1 - alpha) * s_new.double()
                err = (p.detach().cpu().double() - (a_part + b_part)).abs()
                assert bool((err <= 2.5e-7 * (a_part.abs() + b_part.abs()) + 1e-12).all()), (mi, n)
        if mi < n_students:
            assert agree_n >= 0.97 * total_n, (mi, agree_n / total_n)
        for (bn, b), (_, rb) in zip(m.named_buffers(), r.named_buffers()):
            if bn.endswith("num_batches_tracked"):
                assert int(b) == int(rb), bn
            else:
                err = float((b.cpu().double() - rb.double()).norm() / (rb.double().norm() + 1e-30))
                assert err < 1e-3, (mi, bn, err)


def test_step_graph_replay_matches_eager(monkeypatch):
    """Four MT_UBPL steps with the step graph (2 eager warm-up steps, capture,
    2 replays) leave the students, teachers and BN statistics bit-identical to
    four eager steps: the replay runs the same kernels in the same order, with
    the AdamW step count and the BN arrival counters on the device.  Networks
    on one stream: the configuration the step graph is enabled for by default."""
    monkeypatch.setenv("UBPL_MODEL_STREAMS", "0")
    _graph_vs_eager(monkeypatch)


@pytest.mark.xfail(reason="open race: captured step with per-network streams diverges from eager in ~40 % of "
                          "runs (DESIGN.md §6); the graph is off by default in that configuration",
                   strict=False)
def test_step_graph_with_model_streams_matches_eager(monkeypatch):
    monkeypatch.setenv("UBPL_MODEL_STREAMS", "1")
    _graph_vs_eager(monkeypatch)


def _graph_vs_eager(monkeypatch):
    from ubpl_amd import train as T
    from ubpl_amd.optim import FlatAdamW
    cfg = seeds.step_cases()["mt_ubpl"]

    def run(graph):
        monkeypatch.setenv("UBPL_STEP_GRAPH", "1" if graph else "0")
        models, emas, _ = seeds.step_models(_factory, cfg, device="cuda")
        optims = [FlatAdamW(m, lr=cfg["lr"], weight_decay=0) for m in models]
        loader, args = seeds.step_batch(cfg, OR.kps_heatmap_torch)
        import io
        import contextlib
        with contextlib.redirect_stdout(io.StringIO()):
            rec = T.train_mt_ubpl(list(loader) * 4, models, emas, optims, args)
        runner = T._StepGraph.get(T._mt_ubpl_core, models, emas, optims, args)
        assert (runner.graph is not None) == graph
        torch.cuda.synchronize()
        return [m.flat_params.clone() for m in models + emas], [m.flat_stats.clone() for m in models + emas], rec

    p_e, s_e, r_e = run(False)
    p_g, s_g, r_g = run(True)
    diag = {"params": [float((a - b).abs().max()) for a, b in zip(p_e, p_g)],
            "stats": [float((a - b).abs().max()) for a, b in zip(s_e, s_g)]}
    for a, b in zip(p_e, p_g):
        assert torch.equal(a, b), diag
    for a, b in zip(s_e, s_g):
        assert torch.equal(a, b), diag
    assert _flat(r_e, []) == _flat(r_g, [])

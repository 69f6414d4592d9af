"""T1 — one training step of each project on the HIP path vs the reference.

The models, optimisers and batch are built exactly as the reference's main()
builds them (seeds.step_models / step_batch; tests/golden/gen_golden.py ran
the reference's own train() on the same inputs, steps.npz).  The exact result
is the oracle's restatement run in float64 (gen_oracle64.py, steps64.npz).
Checked, per case:
* the returned records (pec/mtc/epc/fdc averages) and every student
  parameter's gradient as the optimizer sees it (norm, sum and 8 sampled
  elements) — by MAGNITUDE, with the criterion of test_gpu_hourglass.py:
  |ours - fp64| <= 3 |reference fp32 - fp64| + 1e-4 |fp64| (the reference's
  own fp32 step sits up to a few % from exact on deep train-mode BN
  gradients at B=4, SURVEY Appendix A / DESIGN §2).  A lost loss weight, a
  single instead of doubled FDL gradient (projects/MT_UBPL.py:334-336) or a
  wrong normaliser moves these by O(1);
* the per-batch printed counts (n_sel, n_pseudo): exact;
* the parameter update: AdamW's first step applied to those gradients;
* teachers after the EMA update equal alpha*teacher + (1-alpha)*student
  (alpha keyed on the epoch) to fp32 rounding;
* BN running statistics: 1e-3 relative.
"""
import os

import numpy as np
import pytest
import torch

import seeds
from oracle import render as OR

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


def _run_ours(cfg, flat_adam, monkeypatch):
    """Our train() on the case; also returns each student's gradient record as
    its optimizer step sees it."""
    from ubpl_amd import train as T
    from ubpl_amd.optim import FlatAdamW
    models, emas, optims = seeds.step_models(_factory, cfg, device="cuda")
    if flat_adam:
        optims = [FlatAdamW(m, lr=cfg["lr"], weight_decay=0) for m in models]
    before = [[p.detach().clone() for p in m.parameters()] for m in models + emas]
    loader, args = seeds.step_batch(cfg, OR.kps_heatmap_torch)
    grads, full = {}, {}

    def snap():
        torch.cuda.synchronize()
        for mi, m in enumerate(models):
            grads[mi] = seeds.grad_record([(n, p.grad) for n, p in m.named_parameters()])
            full[mi] = {n: p.grad.detach().double().cpu() for n, p in m.named_parameters() if p.grad is not None}
    orig = T._step_and_ema
    monkeypatch.setattr(T, "_step_and_ema", lambda *a, **k: (snap(), orig(*a, **k))[1])
    for o in optims:
        ostep = o.step
        o.step = lambda *a, _s=ostep, **k: (snap() if not grads else None, _s(*a, **k))[1]
    import io
    import contextlib
    import re
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
    counts = [[int(a), int(b)] for a, b in re.findall(r"\((\s*\d+)/(\s*\d+)\)", buf.getvalue())]
    return models + emas, before, rec, counts, args, grads, full


def _noise_floor(ours, ref32, ref64, scale, rtol=1e-4):
    """|ours - fp64| <= 3 |ref32 - fp64| + rtol * scale (elementwise)."""
    return np.abs(ours - ref64) <= 3 * np.abs(ref32 - ref64) + rtol * scale + 1e-12


def _grad_errors(st, sa, st64, sa64, idx):
    """Per-parameter relative errors against fp64 of a gradient record: the
    norm, the 8 sampled elements (L2) and the sum (relative to sum |g|)."""
    e = []
    for i in idx:
        m = ~np.isnan(sa64[i])
        n64 = np.sqrt(st64[i, 1])
        e.append((abs(np.sqrt(st[i, 1]) - n64) / n64,
                  np.linalg.norm(sa[i][m] - sa64[i][m]) / max(np.linalg.norm(sa64[i][m]), 1e-30),
                  abs(st[i, 0] - st64[i, 0]) / max(st64[i, 2], 1e-30)))
    return np.array(e)


def check_full_grads(case, ours, g32, g64):
    """Full tensors (B <= 8 cases, oracle run here).  The reference's own fp32
    step sits 1-3 % from fp64 on these B=4 steps (train-mode BN backward over
    4x4 planes amplifies rounding; tools/step_grad_diag.py), and that error
    varies ~10x from tensor to tensor of the same level, so a tensor's bar is
    3x the larger of its own reference error and the 90th percentile of the
    student's reference errors (+1e-4), and the student's median error may
    not exceed 3.5x the reference's (measured: 0.7-3x — MFMA block sums and
    split pieces round differently from the CPU's FMA chains, and these
    chaotic B=4 backward passes amplify any rounding ~1e4x).  A lost loss
    term or factor moves the median tensor by >= 10 %: the doubled-FDL case
    mt_ubpl_fdl moves it 11.5 %."""
    for mi, grads in ours.items():
        rows = []
        for n, gg in g64[mi].items():
            if seeds.bn_cancelled(n) or float(gg.norm()) == 0:
                continue
            rows.append((n, float((grads[n] - gg).norm() / gg.norm()), float((g32[mi][n] - gg).norm() / gg.norm())))
        eo, er = np.array([r[1] for r in rows]), np.array([r[2] for r in rows])
        assert np.median(eo) <= 3.5 * np.median(er) + 1e-5, (case, mi, np.median(eo), np.median(er))
        p90 = np.percentile(er, 90)
        bad = [r for r in rows if r[1] > 3 * max(r[2], p90) + 1e-4]
        assert not bad, (case, mi, p90, bad[:6])


def check_step_grads(case, mi, rec, names, g32, g64):
    """Our gradients vs fp64, against the reference's fp32 gradients vs fp64.
    Per-parameter errors of fp32 gradients are random (one realisation per
    tensor), so the bar is statistical over the ~450 tensors of a student:
    median and 95th percentile no worse than 2x / 3x the reference's, and no
    tensor beyond 3x its own reference error + 10x the reference's median
    error (a lost factor or term moves tensors by 10-100 %)."""
    st, sa = rec
    st32, sa32 = g32[case + "/model%d/grad_stats" % mi], g32[case + "/model%d/grad_samp" % mi]
    st64, sa64 = g64[case + "/model%d/grad_stats" % mi], g64[case + "/model%d/grad_samp" % mi]
    live = st64[:, 1] > 0
    keep = np.array([not seeds.bn_cancelled(n) for n in names])
    assert np.array_equal((st[:, 1] > 0)[keep], live[keep]), (case, mi)
    idx = [i for i in range(len(names)) if live[i] and keep[i]]
    eo, er = _grad_errors(st, sa, st64, sa64, idx), _grad_errors(st32, sa32, st64, sa64, idx)
    for c, what in enumerate(("norm", "samples", "sum")):
        mo, mr = np.median(eo[:, c]), np.median(er[:, c])
        po, pr = np.percentile(eo[:, c], 95), np.percentile(er[:, c], 95)
        assert po <= 3 * pr + 1e-4, (case, mi, what, "p95", po, pr)
        if what == "sum":
            continue            # a tensor's sum cancels: only its tail is compared
        assert mo <= 2 * mr + 1e-5, (case, mi, what, "median", mo, mr)
        # gross per-tensor errors only (the statistics of one tensor fluctuate)
        bad = np.nonzero(eo[:, c] > 3 * er[:, c] + 10 * pr + 1e-4)[0]
        assert bad.size == 0, (case, mi, what, [(names[idx[b]], eo[b, c], er[b, c]) for b in bad[:5]])


STEP_CASES = [("mt_ubpl", True), ("mt_ubpl_e0", False), ("dualpose", True), ("mt", True), ("sup", False),
              ("mt_ubpl_noep", True), ("mt_ubpl_fdl", True), ("dualpose_hg4", True), ("mt_ubpl_b32", True)]


@pytest.mark.parametrize("case,flat_adam", STEP_CASES)
def test_train_step_vs_reference(case, flat_adam, monkeypatch):
    cfg = seeds.step_cases()[case]
    _check_step(case, cfg, *_run_ours(cfg, flat_adam, monkeypatch))


def _run_captured(cfg, monkeypatch):
    """The bench's exact configuration: per-network streams, the whole step
    captured in a HIP graph and replayed.  The graph needs WARM eager steps
    before it captures, so: snapshot every piece of state a step changes
    (parameters, BN running statistics and counters of all four networks,
    AdamW moments and device step counts), run the warm-up steps, restore the
    snapshot IN PLACE (same addresses: the graph bakes them in), then run the
    golden batch once more — captured and replayed from the seeded state.
    The gradients are read after the replay from the flat gradient buffers
    (AdamW does not clear them)."""
    from ubpl_amd import train as T
    from ubpl_amd.optim import FlatAdamW
    monkeypatch.setenv("UBPL_MODEL_STREAMS", "1")
    monkeypatch.setenv("UBPL_STEP_GRAPH", "1")
    T._StepGraph.clear()
    models, emas, _ = seeds.step_models(_factory, cfg, device="cuda")
    optims = [FlatAdamW(m, lr=cfg["lr"], weight_decay=0) for m in models]
    before = [[p.detach().clone() for p in m.parameters()] for m in models + emas]
    loader, args = seeds.step_batch(cfg, OR.kps_heatmap_torch)
    state = [t for m in models + emas for t in (m.flat_params, m.flat_stats, m._nbt)]
    state += [t for o in optims for t in (o.exp_avg, o.exp_avg_sq, o._step_t)]
    snap = [t.clone() for t in state]
    import io
    import contextlib
    import re
    train, core = _train_fn(T, cfg)
    with contextlib.redirect_stdout(io.StringIO()):
        train(list(loader) * T._StepGraph.WARM, models, emas, optims, args)
    runner = T._StepGraph.get(core, models, emas, optims, args)
    assert runner.graph is None and runner.n_eager == T._StepGraph.WARM
    torch.cuda.synchronize()
    for t, v in zip(state, snap):
        t.copy_(v)
    buf = io.StringIO()
    with contextlib.redirect_stdout(buf):
        rec = train(loader, models, emas, optims, args)
    assert runner.graph is not None and runner.n_eager == T._StepGraph.WARM     # this step was the replay
    torch.cuda.synchronize()
    counts = [[int(a), int(b)] for a, b in re.findall(r"\((\s*\d+)/(\s*\d+)\)", buf.getvalue())]
    grads, full = {}, {}
    for mi, m in enumerate(models):
        grads[mi] = seeds.grad_record([(n, p.grad) for n, p in m.named_parameters()])
        full[mi] = {n: p.grad.detach().double().cpu() for n, p in m.named_parameters() if p.grad is not None}
    T._StepGraph.clear()
    return models + emas, before, rec, counts, args, grads, full


def _train_fn(T, cfg):
    if cfg["project"] == "DualPose_UBPL":
        return T.train_dualpose_ubpl, T._dualpose_core
    return T.train_mt_ubpl, T._mt_ubpl_core


def test_captured_dualpose_step_vs_reference(monkeypatch):
    """The DualPose_UBPL step replayed from its captured HIP graph on
    per-network streams against the reference's fixtures (as below)."""
    case = "dualpose"
    cfg = seeds.step_cases()[case]
    _check_step(case, cfg, *_run_captured(cfg, monkeypatch))


def test_captured_b32_step_vs_reference(monkeypatch):
    """the timed path itself — the B=32 headline step
    replayed from its captured HIP graph on per-network streams — against the
    reference's fixtures (records, printed counts, gradient records, AdamW
    step, EMA, BN statistics), with the bars of the eager B=32 case."""
    case = "mt_ubpl_b32"
    cfg = seeds.step_cases()[case]
    _check_step(case, cfg, *_run_captured(cfg, monkeypatch))


def _check_step(case, cfg, ours, before, rec, counts, args, grads, full):
    g = np.load(os.path.join(GD, "steps.npz"))
    g64 = np.load(os.path.join(GD, "steps64.npz"))
    r, r32, r64 = np.array(_flat(rec, [])), g[case + "/records"], g64[case + "/records"]
    assert _noise_floor(r, r32, r64, np.abs(r64)).all(), (r, r32, r64)
    assert np.array_equal(np.array(counts, np.int64).reshape(-1, 2), g[case + "/printed_counts"])
    n_students = cfg["brNum"]
    names = [n for n, _ in ours[0].named_parameters()]
    if cfg["B"] > 8:
        # B=32: the oracle's fp32/fp64 steps take minutes on a CPU; the fixtures hold
        # the reference's and the fp64 gradient records (norm, sum, samples per tensor)
        for mi in range(n_students):
            check_step_grads(case, mi, grads[mi], names, g, g64)
    else:
        from step_oracle import oracle_grads
        torch.set_num_threads(min(16, os.cpu_count() or 1))
        check_full_grads(case, full, oracle_grads(cfg, False), oracle_grads(cfg, True))
    for mi, (m, b0) in enumerate(zip(ours, before)):
        if mi < n_students:
            # AdamW's first step from the gradients checked above: p1 = p0 - lr g / (|g| + eps)
            # (torch.optim.AdamW, step 1, weight_decay 0; bias corrections cancel)
            for n, p, p0 in zip(names, m.parameters(), b0):
                if n not in full[mi]:
                    assert torch.equal(p.detach().cpu(), p0.cpu()), n       # never-trained skip_layer
                    continue
                gg = full[mi][n]
                want = p0.cpu().double() - args.lr * gg / (gg.abs() + 1e-8)
                err = (p.detach().cpu().double() - want).abs()
                assert bool((err <= 1e-3 * args.lr + 2.5e-7 * p0.cpu().double().abs()).all()), (mi, n)
        else:
            # teacher = alpha*teacher + (1-alpha)*student_after_step (utils/parameters.py:6-8)
            for n, p, p0 in zip(names, m.parameters(), b0):
                s_new = dict(ours[mi - n_students].named_parameters())[n].detach().cpu()
                alpha = min(1 - 1 / (args.epo + 1), args.ema_decay)
                a_part, b_part = p0.cpu().double() * alpha, (1 - alpha) * s_new.double()
                err = (p.detach().cpu().double() - (a_part + b_part)).abs()
                assert bool((err <= 2.5e-7 * (a_part.abs() + b_part.abs()) + 1e-12).all()), (mi, n)
        bst = np.array([[b.detach().double().sum().item(), (b.detach().double() ** 2).sum().item()]
                        for _, b in m.named_buffers()])
        ref = g[case + "/model%d/buf" % mi]
        assert np.array_equal(bst[2::3], ref[2::3])                          # num_batches_tracked
        nb, nr = np.sqrt(bst[:, 1]), np.sqrt(ref[:, 1])                      # per-buffer norms
        err = np.abs(nb - nr) <= 1e-3 * nr + 1e-7
        assert err.all(), (mi, np.argwhere(~err)[:4])


def test_step_graph_replay_matches_eager(monkeypatch):
    """Four MT_UBPL steps with the step graph (2 eager warm-up steps, capture,
    2 replays) leave the students, teachers and BN statistics bit-identical to
    four eager steps: the replay runs the same kernels in the same order, with
    the AdamW step count and the BN arrival counters on the device.  Networks
    on one stream: the configuration the step graph is enabled for by default."""
    monkeypatch.setenv("UBPL_MODEL_STREAMS", "0")
    _graph_vs_eager(monkeypatch)


def test_step_graph_with_model_streams_matches_eager(monkeypatch):
    """The same with one HIP stream per network (the default configuration):
    rounds 1-3 saw this diverge in ~40 % of runs — the packed-FP32 instruction
    fault of DESIGN.md §6, fixed in round 4 (csrc/Makefile NOPK)."""
    monkeypatch.setenv("UBPL_MODEL_STREAMS", "1")
    _graph_vs_eager(monkeypatch)


def test_dualpose_step_graph_matches_eager(monkeypatch):
    """Four DualPose_UBPL steps, captured and replayed on per-network streams,
    bit-identical to four eager steps."""
    monkeypatch.setenv("UBPL_MODEL_STREAMS", "1")
    _graph_vs_eager(monkeypatch, "dualpose")


def _graph_vs_eager(monkeypatch, case="mt_ubpl"):
    from ubpl_amd import train as T
    from ubpl_amd.optim import FlatAdamW
    cfg = seeds.step_cases()[case]
    train, core = _train_fn(T, cfg)

    def run(graph):
        monkeypatch.setenv("UBPL_STEP_GRAPH", "1" if graph else "0")
        models, emas, _ = seeds.step_models(_factory, cfg, device="cuda")
        optims = [FlatAdamW(m, lr=cfg["lr"], weight_decay=0) for m in models]
        loader, args = seeds.step_batch(cfg, OR.kps_heatmap_torch)
        import io
        import contextlib
        with contextlib.redirect_stdout(io.StringIO()):
            rec = train(list(loader) * 4, models, emas, optims, args)
        runner = T._StepGraph.get(core, models, emas, optims, args)
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


def _rows(obj, rows):
    """A batch restricted to some of its rows (every tensor whose first dim is the batch)."""
    if torch.is_tensor(obj):
        return obj[rows].clone() if obj.dim() and obj.shape[0] == 4 else obj
    if isinstance(obj, (list, tuple)):
        return type(obj)(_rows(v, rows) for v in obj)
    if isinstance(obj, dict):
        return {k: _rows(v, rows) for k, v in obj.items()}
    return obj


def test_step_graph_ragged_batch_and_new_epoch(monkeypatch):
    """The captured step's other paths, against the same schedule run eagerly,
    bit for bit: a batch of another shape mid-epoch (2 of the 4 rows: it runs
    eagerly, and the full-size batches after it replay the graph again), then a
    new epoch whose host constants change (learning rate halved, EMA epoch
    advanced: the runner releases its graph and captures anew)."""
    import contextlib
    import io
    from ubpl_amd import train as T
    from ubpl_amd.optim import FlatAdamW
    cfg = seeds.step_cases()["mt_ubpl"]
    monkeypatch.setenv("UBPL_MODEL_STREAMS", "1")

    def run(graph):
        monkeypatch.setenv("UBPL_STEP_GRAPH", "1" if graph else "0")
        T._StepGraph.clear()
        models, emas, _ = seeds.step_models(_factory, cfg, device="cuda")
        optims = [FlatAdamW(m, lr=cfg["lr"], weight_decay=0) for m in models]
        loader, args = seeds.step_batch(cfg, OR.kps_heatmap_torch)
        full = loader[0]
        small = _rows(full, [0, 2])                 # one unlabeled, one labeled row
        with contextlib.redirect_stdout(io.StringIO()):
            r1 = T.train_mt_ubpl([full, full, full, small, full], models, emas, optims, args)
            runner = T._StepGraph.get(T._mt_ubpl_core, models, emas, optims, args)
            first = runner.graph
            for o in optims:
                o.param_groups[0]["lr"] *= 0.5
            args.epo += 1
            r2 = T.train_mt_ubpl([full] * 4, models, emas, optims, args)
        runner = T._StepGraph.get(T._mt_ubpl_core, models, emas, optims, args)
        if graph:
            assert first is not None and runner.graph is not None and runner.graph is not first
        else:
            assert first is None and runner.graph is None
        torch.cuda.synchronize()
        out = ([m.flat_params.clone() for m in models + emas], [m.flat_stats.clone() for m in models + emas],
               _flat([r1, r2], []))
        T._StepGraph.clear()
        return out

    p_e, s_e, r_e = run(False)
    p_g, s_g, r_g = run(True)
    for a, b in zip(p_e, p_g):
        assert torch.equal(a, b), float((a - b).abs().max())
    for a, b in zip(s_e, s_g):
        assert torch.equal(a, b), float((a - b).abs().max())
    assert r_e == r_g

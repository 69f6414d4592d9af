"""Repeatability of the multi-stream path (the race of rounds 1-3).

Root cause found in round 4 (tools/fwd_race.py, tools/gpu_r04_race*.sh): a
packed-FP32 VALU instruction — the hourglass upsample-add's v_pk_add_f32 with
op_sel — returned wrong results for one 16-lane pass (its src1 high half
dropped: out = up instead of up + low for 16 consecutive float4 z-components)
when other kernels' matrix work ran beside it from concurrent queues.  With the
library built without packed-FP32 instructions (csrc/Makefile NOPK; the built
code objects are checked on the CPU by test_cpu_host.py::
test_device_code_has_no_packed_fp32_instructions) and no PyTorch elementwise
kernel running beside the networks' backward (train._backward_all), these
configurations repeat bit for bit.  Before the fix, the first case differed in
every repeat (3 of 3, 4 of 4, 5 of 5 on four boxes) and the second in 1 of 11
(3 of 3 with the 1x1 split-load kernel at launch bounds (256, 1)).
"""
import contextlib
import io

import pytest
import torch

import seeds
from oracle import render as OR

pytestmark = pytest.mark.gpu


def _forwards(models, imgs, streams):
    main = torch.cuda.current_stream()
    outs = []
    for s in streams:
        s.wait_stream(main)
    for m, s in zip(models, streams):
        with torch.cuda.stream(s), torch.no_grad():
            for x in imgs:
                outs.append(m(x)[0].clone())
    for s in streams:
        main.wait_stream(s)
    torch.cuda.synchronize()
    return outs


@pytest.mark.parametrize("precision", ["2xfp16", "6xbf16"])
def test_network_forwards_on_four_streams_repeat_bit_for_bit(precision):
    """Four train-mode HG2 forwards (B=32, 256x256, two views each), one HIP
    stream per network as the training step runs them, repeated on the same
    weights and inputs: every repeat equals the first."""
    from ubpl_amd.hourglass import StackedHourglass
    torch.manual_seed(1388)
    models = [StackedHourglass(16, 2, "AvgPool") for _ in range(4)]
    for m in models:
        m.set_conv_precision(precision)
    g = torch.Generator().manual_seed(7)
    imgs = [(torch.rand(32, 3, 256, 256, generator=g) - 0.49).cuda() for _ in range(2)]
    streams = [torch.cuda.Stream() for _ in models]
    ref = _forwards(models, imgs, streams)
    for r in range(4):
        cur = _forwards(models, imgs, streams)
        bad = [i for i, (a, b) in enumerate(zip(ref, cur)) if not torch.equal(a, b)]
        assert not bad, (precision, r, bad)


def _step(case):
    from ubpl_amd import train as T
    from ubpl_amd.hourglass import StackedHourglass
    from ubpl_amd.optim import FlatAdamW
    cfg = seeds.step_cases()[case]
    models, emas, _ = seeds.step_models(lambda k, s, m: StackedHourglass(k, s, m), cfg, device="cuda")
    optims = [FlatAdamW(m, lr=cfg["lr"], weight_decay=0) for m in models]
    loader, args = seeds.step_batch(cfg, OR.kps_heatmap_torch)
    grads = {}
    orig = T._step_and_ema

    def snap(*a, **k):
        torch.cuda.synchronize()
        grads["g"] = [m.flat_grads.clone() for m in models]
        return orig(*a, **k)
    T._step_and_ema = snap
    try:
        with contextlib.redirect_stdout(io.StringIO()):
            rec = T.train_mt_ubpl(loader, models, emas, optims, args)
    finally:
        T._step_and_ema = orig
    torch.cuda.synchronize()
    return (grads["g"] + [m.flat_params.clone() for m in models + emas]
            + [m.flat_stats.clone() for m in models + emas]), rec


def test_headline_step_on_network_streams_repeats_bit_for_bit(monkeypatch):
    """The B=32 headline MT_UBPL step (eager, one stream per network, the
    second-view backward on the teacher's stream) from freshly seeded models:
    gradients, updated parameters, teachers and BatchNorm statistics equal the
    first run bit for bit, and so do the printed records."""
    monkeypatch.setenv("UBPL_MODEL_STREAMS", "1")
    monkeypatch.setenv("UBPL_STEP_GRAPH", "0")
    ref, rref = _step("mt_ubpl_b32")
    for r in range(3):
        cur, rcur = _step("mt_ubpl_b32")
        bad = [i for i, (a, b) in enumerate(zip(ref, cur)) if not torch.equal(a, b)]
        assert not bad, (r, bad)
        assert rcur == rref


@pytest.mark.parametrize("case", ["mt_ubpl", "dualpose"])
def test_network_phases_enqueue_no_torch_arithmetic(case, monkeypatch):
    """the invariant the fix rests on, checked — between the fork
    of the network streams and their join (the forwards; the backwards) no
    PyTorch arithmetic op is enqueued (train._PhaseCheck over one eager step
    of each multi-network project; join() raises on a violation)."""
    from ubpl_amd import train as T
    from ubpl_amd.hourglass import StackedHourglass
    from ubpl_amd.optim import FlatAdamW
    monkeypatch.setenv("UBPL_MODEL_STREAMS", "1")
    monkeypatch.setenv("UBPL_STEP_GRAPH", "0")
    monkeypatch.setattr(T, "_STREAM_CHECK", True)
    cfg = seeds.step_cases()[case]
    models, emas, _ = seeds.step_models(lambda k, s, m: StackedHourglass(k, s, m), cfg, device="cuda")
    optims = [FlatAdamW(m, lr=cfg["lr"], weight_decay=0) for m in models]
    loader, args = seeds.step_batch(cfg, OR.kps_heatmap_torch)
    train = T.train_dualpose_ubpl if cfg["project"] == "DualPose_UBPL" else T.train_mt_ubpl
    with contextlib.redirect_stdout(io.StringIO()):
        train(loader, models, emas, optims, args)
    torch.cuda.synchronize()

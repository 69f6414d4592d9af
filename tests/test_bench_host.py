"""bench.py's host-side accounting (no GPU): the per-sample conv FLOP it prices the step
with (266.7 GF per training sample = 16 forward-equivalents of 16.67 GF at
HG2 256^2, K=16) and the step-level fraction's peaks per precision."""
import os
import sys

import pytest

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


@pytest.fixture(scope="module")
def bench():
    import bench as b
    return b


def test_forward_flops_matches_survey(bench):
    f = bench.forward_flops(2, 16, 256)
    assert abs(f / 1e9 - 16.67) < 0.01
    assert abs(16 * f / 1e9 - 266.7) < 0.1
    f3 = bench.forward_flops(2, 16, 256, ks=3)
    f1 = bench.forward_flops(2, 16, 256, ks=1)
    f7 = bench.forward_flops(2, 16, 256, ks=7)
    assert f3 + f1 + f7 == f                     # every conv counted once, by kernel size
    assert 0.55 < f3 / f < 0.65                  # the 3x3 convs: ~60 % of the conv FLOP
    assert bench.forward_flops(2, 16, 256) == f  # the kernel-size filter does not leak


def test_step_record_peaks(bench):
    cfg = bench.CONFIGS["mt_ubpl"]
    r6 = bench.step_record(cfg, 32, 100.0, "6xbf16")
    r2 = bench.step_record(cfg, 32, 100.0, "2xfp16")
    rb = bench.step_record(cfg, 32, 100.0, "bf16")
    assert r6["flop_per_step"] == r2["flop_per_step"] == 32 * 16 * bench.forward_flops(2, 16, 256)
    assert r6["peak_tflops_fwd"] == pytest.approx(2500 / 6, rel=1e-3)
    assert r2["peak_tflops_fwd"] == pytest.approx(2500 / 3, rel=1e-3)
    # 6xbf16: everything at the 6-product peak; 2xfp16 halves the forwards' and 3x3 gradients' part
    t6 = r6["flop_per_step"] / (2500e12 / 6)
    assert r6["step_frac"] == pytest.approx(t6 / 0.1, rel=1e-3)
    assert r6["step_frac"] / 2 < r2["step_frac"] < r6["step_frac"]
    assert rb["step_frac"] < r2["step_frac"]
    dp = bench.step_record(bench.CONFIGS["dualpose_hg4"], 16, 100.0, "2xfp16")
    assert dp["flop_per_step"] == 16 * 8 * bench.forward_flops(4, 17, 256)   # one view per network

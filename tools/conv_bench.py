"""Per-shape conv timing for the 2-stack hourglass step (GPU).

For every distinct conv shape of StackedHourglass(16, 2) at batch B, times the
forward (with its BN prologue when the network has one), the data gradient and
the weight gradient through the C-ABI, and prints ms/call, TFLOP/s and the
per-step contribution (calls per step x ms).  A student step = fwd + dgrad +
wgrad; the teacher forward adds one fwd per conv (MT_UBPL, 2 views: 8
forwards and 4 backwards per step in bench.py's workload).

    python tools/conv_bench.py [B] [reps]
"""
import os
import sys
from collections import Counter

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "ubpl-poseestimation_amd"))
from ubpl_amd import kernels as Kn  # noqa: E402


def shapes(nstack=2, k=16):
    """(Cin, Cout, KS, stride, H_in, pro) -> count per network forward."""
    c = Counter()

    def res(cin, cout, h):
        half = cout // 2
        c[(cin, half, 1, 1, h, True)] += 1
        c[(half, half, 3, 1, h, True)] += 1
        c[(half, cout, 1, 1, h, True)] += 1
        if cin != cout:
            c[(cin, cout, 1, 1, h, False)] += 1

    c[(3, 64, 7, 2, 256, False)] += 1
    res(64, 128, 128)
    res(128, 128, 64)
    res(128, 256, 64)
    for _ in range(nstack):
        res(256, 256, 64)                     # up1 of the top level
        for h in (32, 16, 8):
            for _ in range(3):
                res(256, 256, h)
        for _ in range(3):
            res(256, 256, 4)
        res(256, 256, 64)                     # features residual
        c[(256, 256, 1, 1, 64, False)] += 1   # features conv
        c[(256, k, 1, 1, 64, False)] += 1     # preds
    for _ in range(nstack - 1):
        c[(256, 256, 1, 1, 64, False)] += 1   # merge_features
        c[(k, 256, 1, 1, 64, False)] += 1     # merge_preds
    return c


def timeit(fn, reps):
    fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(reps):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / reps


def main():
    B = int(sys.argv[1]) if len(sys.argv) > 1 else 32
    reps = int(sys.argv[2]) if len(sys.argv) > 2 else 20
    dev = torch.device("cuda", 0)
    g = torch.Generator(device=dev).manual_seed(0)
    rows = []
    tot = {"fwd": 0.0, "dgrad": 0.0, "wgrad": 0.0}
    for (cin, cout, ks, st, h, pro), cnt in sorted(shapes().items(), key=lambda t: -t[0][4]):
        x = torch.randn(B, cin, h, h, device=dev, generator=g)
        w = torch.randn(cout, cin, ks, ks, device=dev, generator=g) * 0.05
        b = torch.randn(cout, device=dev, generator=g)
        ps = torch.rand(cin, device=dev, generator=g) + 0.5 if pro else None
        ph = torch.randn(cin, device=dev, generator=g) if pro else None
        wt = Kn.conv_weight_tapmajor(w) if ks > 1 else None
        y = Kn.conv2d_forward(x, w, b, st, ps, ph, w_tap=wt)
        ho = y.shape[-1]
        fl = 2.0 * B * cout * cin * ks * ks * ho * ho
        tf = timeit(lambda: Kn.conv2d_forward(x, w, b, st, ps, ph, out=y, w_tap=wt), reps)
        dw = torch.zeros_like(w)
        db = torch.zeros_like(b)
        tw = timeit(lambda: Kn.conv2d_wgrad(y, x, ks, st, dw, db, ps, ph, accumulate=False), reps)
        td = float("nan")
        if st == 1:
            wd = Kn.conv_weight_flip(w)
            dx = torch.empty_like(x)
            td = timeit(lambda: Kn.conv2d_dgrad(y, None, out=dx, wt=wd), reps)
        # per MT_UBPL step (2 views): 8 forwards (2 students + 2 teachers), 4 backwards
        step = {"fwd": 8 * cnt * tf, "dgrad": 4 * cnt * (0 if td != td else td), "wgrad": 4 * cnt * tw}
        for kx in tot:
            tot[kx] += step[kx]
        rows.append((cin, cout, ks, st, h, pro, cnt, tf, fl / tf / 1e9, td, fl / td / 1e9 if td == td else 0.0, tw,
                     fl / tw / 1e9, sum(step.values())))
    print("%5s %5s %2s %2s %4s %3s %3s | %8s %6s | %8s %6s | %8s %6s | %8s" % (
        "Cin", "Cout", "KS", "s", "H", "pro", "n", "fwd ms", "TF", "dgr ms", "TF", "wgr ms", "TF", "step ms"))
    for r in rows:
        print("%5d %5d %2d %2d %4d %3d %3d | %8.3f %6.1f | %8.3f %6.1f | %8.3f %6.1f | %8.2f" % r)
    print("per-step totals (ms): fwd %.1f  dgrad %.1f  wgrad %.1f  all %.1f" % (
        tot["fwd"], tot["dgrad"], tot["wgrad"], sum(tot.values())))


if __name__ == "__main__":
    main()

"""1x1 conv variants at the 64x64 level (B=32): with / without the fused BN
prologue, residual add (separate or aliasing the output), and the data
gradient, on the exact-f32 MFMA kernel — to see what the in-step launches pay.

    python tools/conv1x1_bench.py [B] [reps]
"""
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "ubpl-poseestimation_amd"))
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from ubpl_amd import kernels as Kn  # noqa: E402
from conv_bench import timeit  # noqa: E402


def main():
    B = int(sys.argv[1]) if len(sys.argv) > 1 else 32
    reps = int(sys.argv[2]) if len(sys.argv) > 2 else 20
    dev = torch.device("cuda", 0)
    g = torch.Generator(device=dev).manual_seed(0)
    H = int(sys.argv[3]) if len(sys.argv) > 3 else 64
    for cin, cout in ((256, 128), (128, 256), (256, 256), (128, 128), (64, 128), (128, 64)):
        x = torch.randn(B, cin, H, H, device=dev, generator=g)
        w = torch.randn(cout, cin, 1, 1, device=dev, generator=g) * 0.05
        b = torch.randn(cout, device=dev, generator=g)
        ps = torch.rand(cin, device=dev, generator=g) + 0.5
        ph = torch.randn(cin, device=dev, generator=g)
        res = torch.randn(B, cout, H, H, device=dev, generator=g)
        y = torch.empty(B, cout, H, H, device=dev)
        fl = 2.0 * B * cout * cin * H * H
        mb = lambda *ts: sum(t.numel() * 4 for t in ts) / 1e6
        cases = [
            ("plain", lambda: Kn.conv2d_forward(x, w, b, 1, out=y), mb(x, y)),
            ("pro", lambda: Kn.conv2d_forward(x, w, b, 1, ps, ph, out=y), mb(x, y)),
            ("pro+res", lambda: Kn.conv2d_forward(x, w, b, 1, ps, ph, res=res, out=y), mb(x, y, res)),
            ("pro+res=out", lambda: Kn.conv2d_forward(x, w, b, 1, ps, ph, res=res, out=res), mb(x, res, res)),
        ]
        wk = Kn.conv_weight_flip(w)       # [Cin][1][Cout] = k-major
        cases += [
            ("dma plain", lambda: Kn.conv1x1_forward_kmajor(x, wk, b, out=y), mb(x, y)),
            ("dma pro", lambda: Kn.conv1x1_forward_kmajor(x, wk, b, ps, ph, out=y), mb(x, y)),
            ("dma pro+res", lambda: Kn.conv1x1_forward_kmajor(x, wk, b, ps, ph, res=res, out=y), mb(x, y, res)),
        ]
        ws = Kn.conv_weight_split(w, 0, 3)
        cases += [
            ("sol plain", lambda: Kn.conv1x1_forward_split_load(x, ws, b, out=y), mb(x, y)),
            ("sol pro", lambda: Kn.conv1x1_forward_split_load(x, ws, b, ps, ph, out=y), mb(x, y)),
            ("sol pro+res", lambda: Kn.conv1x1_forward_split_load(x, ws, b, ps, ph, res=res, out=y), mb(x, y, res)),
        ]
        ysl = Kn.conv1x1_forward_split_load(x, ws, b, ps, ph, res=res)
        yd = Kn.conv1x1_forward_kmajor(x, wk, b, ps, ph, res=res)
        print("sol vs f32 rel %.2e" % float((ysl - yd).norm() / yd.norm()))
        yr = Kn.conv2d_forward(x, w, b, 1, ps, ph, res=res)
        print("dma vs f32 kernel rel %.2e" % float((yd - yr).norm() / yr.norm()))
        for name, fn, mbytes in cases:
            t = timeit(fn, reps)
            print("1x1 %3d->%3d %-12s %7.3f ms %6.1f TF %6.2f TB/s" % (cin, cout, name, t, fl / t / 1e9,
                                                                     mbytes / t / 1e3))
        dy = torch.randn(B, cout, H, H, device=dev, generator=g)
        wd = Kn.conv_weight_flip(w)
        dx = torch.empty_like(x)
        t = timeit(lambda: Kn.conv2d_dgrad(dy, None, out=dx, wt=wd), reps)
        print("1x1 %3d->%3d %-12s %7.3f ms %6.1f TF %6.2f TB/s" % (cin, cout, "dgrad", t, fl / t / 1e9,
                                                                 mb(dy, dx) / t / 1e3))
        t = timeit(lambda: Kn.conv1x1_forward_kmajor(dy, w, None, out=dx), reps)
        print("1x1 %3d->%3d %-12s %7.3f ms %6.1f TF %6.2f TB/s" % (cin, cout, "dma dgrad", t, fl / t / 1e9,
                                                                 mb(dy, dx) / t / 1e3))
        wsd = Kn.conv_weight_split(w, 1, 3)
        t = timeit(lambda: Kn.conv1x1_forward_split_load(dy, wsd, None, out=dx), reps)
        print("1x1 %3d->%3d %-12s %7.3f ms %6.1f TF %6.2f TB/s" % (cin, cout, "sol dgrad", t, fl / t / 1e9,
                                                                 mb(dy, dx) / t / 1e3))
        dw, db = torch.zeros_like(w), torch.zeros_like(b)
        t = timeit(lambda: Kn.conv2d_wgrad(dy, x, 1, 1, dw, db, ps, ph, accumulate=False), reps)
        print("1x1 %3d->%3d %-12s %7.3f ms %6.1f TF %6.2f TB/s" % (cin, cout, "wgrad", t, fl / t / 1e9,
                                                                 mb(dy, x) / t / 1e3))


if __name__ == "__main__":
    main()

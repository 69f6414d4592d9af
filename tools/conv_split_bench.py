"""Forward-conv timing, exact-f32 MFMA (conv.hip) vs split-bf16 (conv_split.hip,
2 and 3 pieces), for every conv shape of the 2-stack hourglass at batch B.

    python tools/conv_split_bench.py [B] [reps]
"""
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "ubpl-poseestimation_amd"))
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from ubpl_amd import kernels as Kn  # noqa: E402
from conv_bench import shapes, timeit  # noqa: E402


def main():
    B = int(sys.argv[1]) if len(sys.argv) > 1 else 32
    reps = int(sys.argv[2]) if len(sys.argv) > 2 else 20
    dev = torch.device("cuda", 0)
    g = torch.Generator(device=dev).manual_seed(0)
    tot = {"f32": 0.0, "s2": 0.0, "s3": 0.0, "psa": 0.0, "sa": 0.0}
    print("%5s %5s %2s %4s %3s %3s | %8s %6s | %8s %6s | %8s %6s" % (
        "Cin", "Cout", "KS", "H", "pro", "n", "f32 ms", "TF", "s2 ms", "TF", "s3 ms", "TF"))
    for (cin, cout, ks, st, h, pro), cnt in sorted(shapes().items(), key=lambda t: -t[0][4]):
        if st != 1 or cin % 16:
            continue
        x = torch.randn(B, cin, h, h, device=dev, generator=g)
        w = torch.randn(cout, cin, ks, ks, device=dev, generator=g) * 0.05
        b = torch.randn(cout, device=dev, generator=g)
        ps = torch.rand(cin, device=dev, generator=g) + 0.5 if pro else None
        ph = torch.randn(cin, device=dev, generator=g) if pro else None
        wt = Kn.conv_weight_tapmajor(w) if ks > 1 else None
        y = Kn.conv2d_forward(x, w, b, st, ps, ph, w_tap=wt)
        fl = 2.0 * B * cout * cin * ks * ks * h * h
        t = {"f32": timeit(lambda: Kn.conv2d_forward(x, w, b, st, ps, ph, out=y, w_tap=wt), reps)}
        for npc in (2, 3):
            ws = Kn.conv_weight_split(w, 0, npc)
            ys = Kn.conv2d_forward_split(x, ws, b, ps, ph)
            err = float((ys - y).norm() / y.norm())
            t["s%d" % npc] = timeit(lambda: Kn.conv2d_forward_split(x, ws, b, ps, ph, out=ys), reps)
            t["e%d" % npc] = err
        ws3 = Kn.conv_weight_split(w, 0, 3)
        pad = (ks - 1) // 2
        xs = Kn.split_activation(x, 3, pad, ps, ph)
        yp = Kn.conv2d_forward_psa(xs, ws3, b)
        t["ep"] = float((yp - y).norm() / y.norm())
        t["psa"] = timeit(lambda: Kn.conv2d_forward_psa(xs, ws3, b, out=yp), reps)
        t["sa"] = timeit(lambda: Kn.split_activation(x, 3, pad, ps, ph, out=xs.buf), reps)
        for kx in tot:
            tot[kx] += 12 * cnt * t[kx]      # 8 forwards + 4 data gradients per MT_UBPL step
        print("%5d %5d %2d %4d %3d %3d | %8.3f %6.1f | %8.3f %6.1f | %8.3f %6.1f | psa %.3f %6.1f + split %.3f | rel %.1e %.1e %.1e" % (
            cin, cout, ks, h, pro, cnt, t["f32"], fl / t["f32"] / 1e9, t["s2"], fl / t["s2"] / 1e9, t["s3"],
            fl / t["s3"] / 1e9, t["psa"], fl / t["psa"] / 1e9, t["sa"], t["e2"], t["e3"], t["ep"]))
    print("per-step fwd+dgrad-shaped totals (ms): f32 %.1f  s2 %.1f  s3 %.1f  psa %.1f + split %.1f" % (
        tot["f32"], tot["s2"], tot["s3"], tot["psa"], tot["sa"]))


if __name__ == "__main__":
    main()

"""conv_psa_kernel timing at the roofline shape(s) (3x3 on the split path, pre-split
operands resident), HIP events around back-to-back launches; prints the time per
launch, the f32-equivalent TFLOP/s, the fraction of the split peak and a checksum
(compare PSA variants for bit-identity: run once per UBPL_PSA_* setting).

    python tools/psa_bench.py [B] [reps] [pieces: 3 (6xbf16, default) | 1 (bf16)]
"""
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "ubpl-poseestimation_amd"))
from ubpl_amd import kernels as Kn  # noqa: E402

PEAK = 2500.0 / 6


def main():
    B = int(sys.argv[1]) if len(sys.argv) > 1 else 32
    reps = int(sys.argv[2]) if len(sys.argv) > 2 else 50
    npieces = int(sys.argv[3]) if len(sys.argv) > 3 else 3
    peak = PEAK if npieces == 3 else 2500.0
    dev = torch.device("cuda", 0)
    g = torch.Generator(device=dev).manual_seed(0)
    shapes = ((128, 128, 64), (64, 64, 128), (128, 128, 32), (256, 256, 64))
    if os.environ.get("PSA_BENCH_96"):
        shapes = ((128, 128, 96), (256, 256, 96))     # the HG8 384x384 top-level planes
    for cin, cout, h in shapes:
        x = torch.randn(B, cin, h, h, device=dev, generator=g)
        w = torch.randn(cout, cin, 3, 3, device=dev, generator=g) * 0.05
        b = torch.randn(cout, device=dev, generator=g)
        ws = Kn.conv_weight_split(w, 0, npieces)
        xs = Kn.split_activation(x, npieces, 1)
        y = Kn.conv2d_forward_psa(xs, ws, b)
        torch.cuda.synchronize()
        for _ in range(3):
            Kn.conv2d_forward_psa(xs, ws, b, out=y)
        torch.cuda.synchronize()
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        torch.cuda._sleep(20_000_000)
        s.record()
        for _ in range(reps):
            Kn.conv2d_forward_psa(xs, ws, b, out=y)
        e.record()
        torch.cuda.synchronize()
        ms = s.elapsed_time(e) / reps
        fl = 2.0 * B * cout * cin * 9 * h * h
        ref = Kn.conv2d_forward(x, w, b, 1, w_tap=Kn.conv_weight_tapmajor(w))
        err = float((y - ref).norm() / ref.norm())
        print("%4d->%4d %3dx%-3d B=%d: %8.1f us  %6.1f TF  frac %.3f  checksum %.10e  rel-vs-f32 %.2e" % (
            cin, cout, h, h, B, ms * 1e3, fl / ms / 1e9, fl / ms / 1e9 / peak, float(y.double().sum()), err),
            flush=True)


if __name__ == "__main__":
    main()

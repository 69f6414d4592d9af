"""3x3 weight gradient per hourglass level (B=32): exact-f32 kernel vs the
split path over PSA operands (wgrad3_psa), and the 1x1 weight gradients.

    python tools/wgrad_bench.py [B] [reps]
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
    for C, H in ((128, 64), (128, 32), (128, 16), (64, 128)):
        x = torch.randn(B, C, H, H, device=dev, generator=g)
        dy = torch.randn(B, C, H, H, device=dev, generator=g)
        ps = torch.rand(C, device=dev, generator=g) + 0.5
        ph = torch.randn(C, device=dev, generator=g)
        dw, db = torch.zeros(C, C, 3, 3, device=dev), torch.zeros(C, device=dev)
        fl = 2.0 * B * C * C * 9 * H * H
        t32 = timeit(lambda: Kn.conv2d_wgrad(dy, x, 3, 1, dw, db, ps, ph, accumulate=False), reps)
        line = "3x3 wgrad C=%3d H=%3d  f32 %7.3f ms %6.1f TF" % (C, H, t32, fl / t32 / 1e9)
        xs = Kn.split_activation(x, 3, 1, ps, ph)
        ys = Kn.split_activation(dy, 3, 1)
        if Kn.wgrad3_psa_ok(ys, xs):
            tp = timeit(lambda: Kn.conv2d_wgrad3_psa(ys, xs, dw, db, accumulate=False), reps)
            line += " | psa %7.3f ms %6.1f TF (splits %d)" % (tp, fl / tp / 1e9, _lib_splits(B, C, H))
        print(line, flush=True)
    for cin, cout, H in ((256, 128, 64), (128, 256, 64), (256, 256, 64), (256, 128, 32), (128, 256, 32),
                         (256, 256, 16)):
        x = torch.randn(B, cin, H, H, device=dev, generator=g)
        dy = torch.randn(B, cout, H, H, device=dev, generator=g)
        ps = torch.rand(cin, device=dev, generator=g) + 0.5
        ph = torch.randn(cin, device=dev, generator=g)
        dw, db = torch.zeros(cout, cin, 1, 1, device=dev), torch.zeros(cout, device=dev)
        fl = 2.0 * B * cin * cout * H * H
        t32 = timeit(lambda: Kn.conv2d_wgrad(dy, x, 1, 1, dw, db, ps, ph, accumulate=False), reps)
        ts = timeit(lambda: Kn.conv2d_wgrad1x1_split_load(dy, x, dw, db, ps, ph, accumulate=False), reps)
        print("1x1 wgrad %3d->%3d H=%3d  f32 %7.3f ms %6.1f TF | split-load %7.3f ms %6.1f TF" % (
            cin, cout, H, t32, fl / t32 / 1e9, ts, fl / ts / 1e9), flush=True)


def _lib_splits(B, C, H):
    from ubpl_amd import _lib
    return int(_lib.lib().ubpl_wgrad3_psa_workspace(B, C, C, H, H)) // (C * (9 * C + 1))


if __name__ == "__main__":
    main()

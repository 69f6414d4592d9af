"""BatchNorm backward pieces at the hourglass planes (B=32): statistics
partials pass, finalize (via part_ready), apply, and the whole backward.

    python tools/bn_bench.py [B] [reps]
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
    reps = int(sys.argv[2]) if len(sys.argv) > 2 else 50
    dev = torch.device("cuda", 0)
    g = torch.Generator(device=dev).manual_seed(0)
    for C, H in ((128, 128), (128, 64), (256, 64), (128, 32), (256, 16), (128, 16), (256, 8), (256, 4)):
        x = torch.randn(B, C, H, H, device=dev, generator=g)
        dz = torch.randn(B, C, H, H, device=dev, generator=g)
        gamma = torch.rand(C, device=dev, generator=g) + 0.5
        mean, istd = torch.randn(C, device=dev, generator=g) * 0.1, torch.rand(C, device=dev, generator=g) + 0.5
        sc, sh = gamma * istd, torch.randn(C, device=dev, generator=g)
        coef = torch.empty(3 * C, device=dev)
        dg, db = torch.zeros(C, device=dev), torch.zeros(C, device=dev)
        out = torch.empty_like(dz)
        part = Kn.bn_bwd_partials(dz, x, sc, sh, mean, 1)
        scratch = Kn.bn_part(B, C, dev)
        beta = torch.zeros(C, device=dev)
        rm, rv = torch.zeros(C, device=dev), torch.ones(C, device=dev)
        m_o, i_o, s_o, h_o = (torch.empty(C, device=dev) for _ in range(4))
        t_fwd = timeit(lambda: Kn.bn_forward_stats(x, gamma, beta, 1e-5, 0.1, rm, rv, scratch, m_o, i_o, s_o, h_o),
                       reps)
        t_part = timeit(lambda: Kn.bn_bwd_partials(dz, x, sc, sh, mean, 1), reps)
        t_ready = timeit(lambda: Kn.bn_backward(dz, x, gamma, mean, istd, sc, sh, 1, scratch, coef, dg, db, out=out,
                                                part=part), reps)
        t_all = timeit(lambda: Kn.bn_backward(dz, x, gamma, mean, istd, sc, sh, 1, scratch, coef, dg, db, out=out),
                       reps)
        mb = 3 * x.numel() * 4 / 1e6
        print("C=%3d H=%3d  fwd stats %7.1f us | bwd partials %7.1f us | finalize+apply %7.1f us | bwd all %7.1f us"
              " (apply %.0f MB)" % (C, H, t_fwd * 1e3, t_part * 1e3, t_ready * 1e3, t_all * 1e3, mb), flush=True)


if __name__ == "__main__":
    main()

"""Workload for rocprofv3 --pmc passes: the split-path 3x3 kernels at the 64x64
level (B=32, 128 channels) — conv_psa_kernel forward and wgrad3_psa_kernel —
REPS launches each.

    rocprofv3 --pmc SQ_WAVE_CYCLES ... -- python tools/pmc_psa.py
"""
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "ubpl-poseestimation_amd"))
from ubpl_amd import kernels as Kn  # noqa: E402

REPS = int(os.environ.get("REPS", "10"))


def main():
    dev = torch.device("cuda", 0)
    g = torch.Generator(device=dev).manual_seed(0)
    B, C, H = 32, 128, 64
    x = torch.randn(B, C, H, H, device=dev, generator=g)
    dy = torch.randn(B, C, H, H, device=dev, generator=g)
    w = torch.randn(C, C, 3, 3, device=dev, generator=g) * 0.03
    b = torch.randn(C, device=dev, generator=g)
    ps = torch.rand(C, device=dev, generator=g) + 0.5
    ph = torch.randn(C, device=dev, generator=g)
    xs = Kn.split_activation(x, 3, 1, ps, ph)
    ys = Kn.split_activation(dy, 3, 1)
    ws = Kn.conv_weight_split(w, 0, 3)
    y = Kn.conv2d_forward_psa(xs, ws, b)
    dw, db = torch.zeros_like(w), torch.zeros_like(b)
    torch.cuda.synchronize()
    for _ in range(REPS):
        Kn.conv2d_forward_psa(xs, ws, b, out=y)
    for _ in range(REPS):
        Kn.conv2d_wgrad3_psa(ys, xs, dw, db, accumulate=False)
    torch.cuda.synchronize()
    print("pmc workload done: %d launches each" % REPS)


if __name__ == "__main__":
    main()

"""Workload for rocprofv3 --pmc passes: the bench's dominant kernel (3x3 conv
forward with the fused BN+ReLU prologue, Residual conv2 at the 64x64 level:
B=32, 128->128) and the same layer's weight gradient, REPS launches each.

    rocprofv3 --pmc FETCH_SIZE -d gpurun_out/pmc -o fetch --output-format csv -- python tools/pmc_conv.py
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
    w = torch.randn(C, C, 3, 3, device=dev, generator=g) * 0.03
    b = torch.randn(C, device=dev, generator=g)
    ps = torch.rand(C, device=dev, generator=g) + 0.5
    ph = torch.randn(C, device=dev, generator=g)
    wt = Kn.conv_weight_tapmajor(w)
    y = Kn.conv2d_forward(x, w, b, 1, ps, ph, w_tap=wt)
    dw, db = torch.zeros_like(w), torch.zeros_like(b)
    torch.cuda.synchronize()
    for _ in range(REPS):
        Kn.conv2d_forward(x, w, b, 1, ps, ph, out=y, w_tap=wt)
    for _ in range(REPS):
        Kn.conv2d_wgrad(y, x, 3, 1, dw, db, ps, ph, accumulate=False)
    torch.cuda.synchronize()
    print("pmc workload done: %d launches each" % REPS)


if __name__ == "__main__":
    main()

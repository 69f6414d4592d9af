"""Workload for rocprofv3 --pmc passes: the 1x1 conv kernels at the 64x64 level
(B=32) — the f32 LDS-DMA kernel (conv1x1_dma_kernel) and the 6xbf16
split-on-load kernel (conv1x1_sol_kernel), 256->128 with the BN prologue and
128->256 with prologue + residual, REPS launches each.

    rocprofv3 --pmc SQ_WAVE_CYCLES ... -- python tools/pmc_1x1.py
"""
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "ubpl-poseestimation_amd"))
from ubpl_amd import kernels as Kn  # noqa: E402

REPS = int(os.environ.get("REPS", "5"))


def main():
    dev = torch.device("cuda", 0)
    g = torch.Generator(device=dev).manual_seed(0)
    B, H = 32, 64
    shapes = ((256, 128, False), (128, 256, True))
    if os.environ.get("SHAPE"):
        shapes = (shapes[int(os.environ["SHAPE"])],)
    only_sol = os.environ.get("ONLY_SOL") == "1"
    for cin, cout, resid in shapes:
        x = torch.randn(B, cin, H, H, device=dev, generator=g)
        w = torch.randn(cout, cin, 1, 1, device=dev, generator=g) * 0.05
        b = torch.randn(cout, device=dev, generator=g)
        ps = torch.rand(cin, device=dev, generator=g) + 0.5
        ph = torch.randn(cin, device=dev, generator=g)
        res = torch.randn(B, cout, H, H, device=dev, generator=g) if resid else None
        y = torch.empty(B, cout, H, H, device=dev)
        wk = Kn.conv_weight_flip(w)
        ws = Kn.conv_weight_split(w, 0, 3)
        torch.cuda.synchronize()
        for _ in range(0 if only_sol else REPS):
            Kn.conv1x1_forward_kmajor(x, wk, b, ps, ph, res=res, out=y)
        for _ in range(REPS):
            Kn.conv1x1_forward_split_load(x, ws, b, ps, ph, res=res, out=y)
        torch.cuda.synchronize()
    print("pmc workload done: %d launches each" % REPS)


if __name__ == "__main__":
    main()

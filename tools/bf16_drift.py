"""GPU-box: how far the "bf16" conv precision (one bf16 piece per operand,
f32 accumulation) drifts from the fp32-equivalent 6xbf16 path through a
stacked hourglass: relative L2 of each stack's heatmaps, train-mode forward,
same seeded init and inputs; also each conv precision against a copy of the
network whose weights were rounded to bf16 first (separates weight rounding
from activation rounding).

    python tools/bf16_drift.py [B] [res] [stacks...]
"""
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "ubpl-poseestimation_amd"))
from ubpl_amd.hourglass import StackedHourglass  # noqa: E402


def rel(a, b):
    return float((a.double() - b.double()).norm() / b.double().norm())


def main():
    B = int(sys.argv[1]) if len(sys.argv) > 1 else 4
    R = int(sys.argv[2]) if len(sys.argv) > 2 else 256
    stacks = [int(s) for s in sys.argv[3:]] or [2, 8]
    dev = torch.device("cuda")
    gen = torch.Generator().manual_seed(11)
    x = (torch.rand(B, 3, R, R, generator=gen) - 0.45).to(dev)
    for S in stacks:
        outs = {}
        for prec in ("6xbf16", "bf16", "f32"):
            torch.manual_seed(2024)
            m = StackedHourglass(16, S, "AvgPool")
            m.set_conv_precision(prec)
            m.train()
            with torch.no_grad():
                outs[prec] = m(x)[0]
        torch.manual_seed(2024)
        mr = StackedHourglass(16, S, "AvgPool")
        mr.set_conv_precision("6xbf16")
        with torch.no_grad():
            for p in mr.parameters():
                p.copy_(p.to(torch.bfloat16).float())
            mr.train()
            outs["wbf16"] = mr(x)[0]
        for k in ("f32", "bf16", "wbf16"):
            print("S=%d B=%d R=%d %-6s vs 6xbf16: %s" % (
                S, B, R, k, " ".join("%.2e" % rel(outs[k][:, s], outs["6xbf16"][:, s]) for s in range(S))),
                flush=True)


if __name__ == "__main__":
    main()

"""Workload for a rocprofv3 kernel trace of single network passes (B=32, one
stream, nothing overlapping): REPS teacher forwards, then REPS student
forward+backward passes.

    rocprofv3 --kernel-trace -d gpurun_out/pp -o pp --output-format csv -- python tools/pass_profile.py
"""
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "ubpl-poseestimation_amd"))
import bench  # noqa: E402

REPS = int(os.environ.get("REPS", "3"))


def main():
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    from ubpl_amd import _lib
    from ubpl_amd.hourglass import StackedHourglass
    _lib.load()
    torch.manual_seed(1388)
    m = StackedHourglass(16, 2, "AvgPool")
    e = StackedHourglass(16, 2, "AvgPool")
    imgs = bench.make_batches(1, 32, 16, dev, 1388)[0][0][0].to(dev).float().contiguous()
    with torch.no_grad():
        e(imgs)
    o, f = m(imgs)
    (o.square().mean() + f.square().mean()).backward()
    torch.cuda.synchronize()
    torch.cuda.nvtx.range_push("fwd") if hasattr(torch.cuda, "nvtx") else None
    for _ in range(REPS):
        with torch.no_grad():
            e(imgs)
    torch.cuda.synchronize()
    for _ in range(REPS):
        o, f = m(imgs)
        (o.square().mean() + f.square().mean()).backward()
    torch.cuda.synchronize()
    print("pass profile workload done")


if __name__ == "__main__":
    main()

#!/bin/bash
# GPU box: out-of-bounds guard probe of every launch of one HG2 forward + backward at B=32 (the batch
# at which the split-load 1x1 kernel and the 64-channel split weight gradients run; round 2 probed B=4).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 500 python tools/guard_probe.py 32 2 AvgPool 256 > gpurun_out/guard_b32.log 2>&1; echo "guard rc=$?"
grep -v "Warn\|amdgpu.ids" gpurun_out/guard_b32.log | tail -25

#!/bin/bash
# GPU box: the B=32 step on ONE stream with the allocator's free memory poisoned differently per run:
# a difference means some kernel reads memory it did not write.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
DET_POISON=1 UBPL_MODEL_STREAMS=0 timeout -k 10 240 python tools/det_step.py mt_ubpl_b32 3 > gpurun_out/det_poison_one.log 2>&1 || { tail -5 gpurun_out/det_poison_one.log; exit 1; }
grep -v "Warn\|amdgpu.ids" gpurun_out/det_poison_one.log | head -30

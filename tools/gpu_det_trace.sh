#!/bin/bash
# GPU box: first differing op (per stream) between repeats of the B=32 eager step, with only the ops
# named in OPS (default the 1x1 split-load convs) checksummed (inputs before, outputs after).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
DET_OPS=${OPS:-conv1x1_forward_split_load} timeout -k 10 300 python tools/det_trace.py mt_ubpl_b32 ${REPS:-3} > gpurun_out/det_trace_sol.log 2>&1 || { tail -20 gpurun_out/det_trace_sol.log; exit 1; }
grep -v "Warn\|amdgpu.ids" gpurun_out/det_trace_sol.log | tail -60

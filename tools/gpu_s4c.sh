#!/bin/bash
# GPU box: eager-step nondeterminism — per-op trace of the 1x1 split-load convs (inputs and outputs
# checksummed), then the step's repeat check with the split-load 1x1 kernel off (UBPL_NO_SOL=1).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
DET_OPS=${OPS:-conv1x1_forward_split_load} timeout -k 10 300 python tools/det_trace.py mt_ubpl_b32 ${REPS:-5} > gpurun_out/det_trace_sol.log 2>&1 || { tail -20 gpurun_out/det_trace_sol.log; exit 1; }
grep -v "Warn\|amdgpu.ids" gpurun_out/det_trace_sol.log | grep -E "run|det_trace|ops per" | head -40
UBPL_NO_SOL=1 timeout -k 10 240 python tools/det_step.py mt_ubpl_b32 ${REPS2:-6} > gpurun_out/det_nosol.log 2>&1 || { tail -5 gpurun_out/det_nosol.log; exit 1; }
grep -E "vs 0:|repeats differ" gpurun_out/det_nosol.log

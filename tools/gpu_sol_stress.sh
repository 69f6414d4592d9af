#!/bin/bash
# GPU box: conv1x1_sol_kernel outputs under four concurrent streams vs run alone (tools/sol_stress.py).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for cfg in "30 32 64" "40 32 32"; do
  timeout -k 10 150 python tools/sol_stress.py $cfg > gpurun_out/sol_stress.log 2>&1 || { tail -5 gpurun_out/sol_stress.log; exit 1; }
  grep -v "Warn\|amdgpu.ids" gpurun_out/sol_stress.log | tail -6
done

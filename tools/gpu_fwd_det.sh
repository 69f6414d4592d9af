#!/bin/bash
# GPU box: are the B=32 autograd forwards of four networks on four streams bit-repeatable?
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 200 python tools/graph_fwd_probe.py ${REPS:-6} 32 2 0 eager+locate > gpurun_out/fwd_eager_locate.log 2>&1 || { tail -5 gpurun_out/fwd_eager_locate.log; exit 1; }
grep -v "Warn\|amdgpu.ids\|detach\|ds = " gpurun_out/fwd_eager_locate.log | tail -20

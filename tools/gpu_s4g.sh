#!/bin/bash
# GPU box: first differing op of the B=32 eager step on abvar/lb1 with the 1x1 split-load convs,
# pools, upsample-adds and BatchNorm passes checksummed (inputs before, outputs after).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
UBPL_LIB_DIR=$PWD/abvar/lb1 DET_OPS=${OPS:-conv1x1_forward_split_load,maxpool2x2,upsample2x_add,bn_forward_stats,bn_apply} timeout -k 10 300 python tools/det_trace.py mt_ubpl_b32 3 > gpurun_out/det_trace_lb1_g.log 2>&1 || { tail -20 gpurun_out/det_trace_lb1_g.log; exit 1; }
grep -v "Warn\|amdgpu.ids" gpurun_out/det_trace_lb1_g.log | grep -v "^\s*$" | tail -60

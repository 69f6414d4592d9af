#!/bin/bash
# GPU box: first differing op between repeats of the B=32 eager step on the 1x1 split-load kernel
# built with launch bounds 1 (abvar/lb1: differs in 11 of 11 repeats) — every op's outputs
# checksummed in-stream (DET_OPS unset), then the same restricted to the 1x1 convs' inputs+outputs.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
UBPL_LIB_DIR=$PWD/abvar/lb1 timeout -k 10 300 python tools/det_trace.py mt_ubpl_b32 3 > gpurun_out/det_trace_lb1_all.log 2>&1 || { tail -20 gpurun_out/det_trace_lb1_all.log; exit 1; }
grep -v "Warn\|amdgpu.ids" gpurun_out/det_trace_lb1_all.log | grep -v "^\s*$" | tail -40
UBPL_LIB_DIR=$PWD/abvar/lb1 DET_OPS=conv1x1_forward_split_load timeout -k 10 300 python tools/det_trace.py mt_ubpl_b32 3 > gpurun_out/det_trace_lb1_sol.log 2>&1 || { tail -20 gpurun_out/det_trace_lb1_sol.log; exit 1; }
grep -v "Warn\|amdgpu.ids" gpurun_out/det_trace_lb1_sol.log | grep -v "^\s*$" | tail -30

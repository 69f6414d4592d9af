#!/bin/bash
# GPU box: bit-repeatability of the B=32 step: in-tree build with per-network streams, the same on one
# stream, and the abvar/nolds build (1x1 prologue coefficients by scalar loads) with streams.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 240 python tools/det_step.py mt_ubpl_b32 ${REPS:-4} > gpurun_out/det_streams.log 2>&1 || { tail -5 gpurun_out/det_streams.log; exit 1; }
[ -n "$ONLY_STREAMS" ] && { cat gpurun_out/det_streams.log | grep -v Warn; exit 0; }
tail -${REPS:-4} gpurun_out/det_streams.log
UBPL_MODEL_STREAMS=0 timeout -k 10 240 python tools/det_step.py mt_ubpl_b32 ${REPS:-4} > gpurun_out/det_onestream.log 2>&1 || { tail -5 gpurun_out/det_onestream.log; exit 1; }
tail -${REPS:-4} gpurun_out/det_onestream.log
UBPL_LIB_DIR=$PWD/abvar/nolds timeout -k 10 240 python tools/det_step.py mt_ubpl_b32 ${REPS:-4} > gpurun_out/det_nolds.log 2>&1 || { tail -5 gpurun_out/det_nolds.log; exit 1; }
echo "== nolds"; tail -${REPS:-4} gpurun_out/det_nolds.log

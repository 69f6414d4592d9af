#!/bin/bash
# GPU box: repeat check of the B=32 eager step on abvar/lb1pp0 (no scratch in any default-path split
# kernel: 1x1 split-load with launch bounds 1, PSA kernel without the ping-pong drains) vs abvar/lb1.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
i=0
for v in lb1pp0 lb1; do
  UBPL_LIB_DIR=$PWD/abvar/$v timeout -k 10 200 python tools/det_step.py mt_ubpl_b32 ${REPS:-6} > gpurun_out/det_s4i_$i.log 2>&1 || { echo "[$v] failed"; tail -3 gpurun_out/det_s4i_$i.log; exit 1; }
  echo "[$v] $(tail -1 gpurun_out/det_s4i_$i.log)"
  grep "first differing BN" gpurun_out/det_s4i_$i.log | head -2
  i=$((i+1))
done

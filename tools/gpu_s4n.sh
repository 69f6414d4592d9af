#!/bin/bash
# GPU box: the always-differing abvar/lb1 build vs the same with the 1x1 split-load kernel's output
# stores non-temporal (abvar/lb1nt): does the race follow that kernel's cached stores?
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
i=0
for v in lb1nt lb1; do
  UBPL_LIB_DIR=$PWD/abvar/$v timeout -k 10 200 python tools/det_step.py mt_ubpl_b32 ${REPS:-6} > gpurun_out/det_s4n_$i.log 2>&1 || { echo "[$v] failed"; tail -3 gpurun_out/det_s4n_$i.log; exit 1; }
  echo "[$v] $(tail -1 gpurun_out/det_s4n_$i.log)"
  grep "first differing BN" gpurun_out/det_s4n_$i.log | head -2
  i=$((i+1))
done

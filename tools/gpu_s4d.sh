#!/bin/bash
# GPU box: eager-step repeat check (B=32 headline case), REPS repeats per setting: default, the
# split-load 1x1 kernel off, and the 1x1 split-load kernel built with launch bounds 1 (no spills).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
i=0
for e in "-" "UBPL_NO_SOL=1" "UBPL_LIB_DIR=$PWD/abvar/lb1" "-"; do
  v=""; [ "$e" != "-" ] && v="$e"
  env $v timeout -k 10 200 python tools/det_step.py mt_ubpl_b32 ${REPS:-12} > gpurun_out/det_s4d_$i.log 2>&1 || { echo "[$e] failed"; tail -3 gpurun_out/det_s4d_$i.log; exit 1; }
  echo "[$e] $(tail -1 gpurun_out/det_s4d_$i.log)"
  grep "first differing BN" gpurun_out/det_s4d_$i.log | head -3
  i=$((i+1))
done

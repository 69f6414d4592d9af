#!/bin/bash
# GPU box: which streams race — the always-differing abvar/lb1 build with the teachers on their
# students' streams, with the second-view backward on the student's own stream, and with every
# network on one side stream.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
i=0
for e in ${SETTINGS:-"UBPL_TEACHER_STREAMS=0" "UBPL_SPLIT_BWD=0" "UBPL_ONE_SIDE=1"}; do
  UBPL_LIB_DIR=$PWD/abvar/lb1 env $e timeout -k 10 200 python tools/det_step.py mt_ubpl_b32 ${REPS:-6} > gpurun_out/det_s4j_$i.log 2>&1 || { echo "[$e] failed"; tail -3 gpurun_out/det_s4j_$i.log; exit 1; }
  echo "[lb1 $e] $(tail -1 gpurun_out/det_s4j_$i.log)"
  grep "first differing BN" gpurun_out/det_s4j_$i.log | head -2
  i=$((i+1))
done

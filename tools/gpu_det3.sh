#!/bin/bash
# GPU box: bisect the B=32 step's run-to-run differences over the stream / precision knobs.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
i=0
for e in "-" "UBPL_TEACHER_STREAMS=0" "UBPL_SPLIT_BWD=0" "UBPL_TEACHER_STREAMS=0 UBPL_SPLIT_BWD=0" "UBPL_ONE_SIDE=1" "UBPL_CONV_PRECISION=f32" "UBPL_NO_SOL=1"; do
  v=""; [ "$e" != "-" ] && v="$e"
  env $v timeout -k 10 200 python tools/det_step.py mt_ubpl_b32 ${REPS:-4} > gpurun_out/det3_$i.log 2>&1 || { echo "[$e] failed"; tail -3 gpurun_out/det3_$i.log; exit 1; }
  echo "[$e] $(tail -1 gpurun_out/det3_$i.log)  $(grep 'run 1 vs 0' gpurun_out/det3_$i.log)"
  grep "first differing BN" gpurun_out/det3_$i.log | head -2
  i=$((i+1))
done

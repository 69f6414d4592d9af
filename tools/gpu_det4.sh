#!/bin/bash
# GPU box: is the B=32 step's nondeterminism the 1x1 split-load kernel's register spills (scratch)?
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
i=0
for e in "UBPL_SOL_BM=64" "UBPL_LIB_DIR=$PWD/abvar/lb1" "-" "UBPL_SOL_BM=64 UBPL_SOL_NS=3"; do
  v=""; [ "$e" != "-" ] && v="$e"
  env $v timeout -k 10 200 python tools/det_step.py mt_ubpl_b32 ${REPS:-4} > gpurun_out/det4_$i.log 2>&1 || { echo "[$e] failed"; tail -3 gpurun_out/det4_$i.log; exit 1; }
  echo "[$e] $(tail -1 gpurun_out/det4_$i.log)  $(grep 'run 1 vs 0' gpurun_out/det4_$i.log)"
  i=$((i+1))
done

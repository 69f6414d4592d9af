#!/bin/bash
# GPU box: does the B=32 step's run-to-run drift depend on the HIP runtime's queue / kernarg setup?
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
i=0
for e in "-" "GPU_MAX_HW_QUEUES=8" "GPU_MAX_HW_QUEUES=2" "HIP_FORCE_DEV_KERNARG=1" "HIP_FORCE_DEV_KERNARG=0"; do
  v=""; [ "$e" != "-" ] && v="$e"
  env $v timeout -k 10 200 python tools/det_step.py mt_ubpl_b32 ${REPS:-4} > gpurun_out/det5_$i.log 2>&1 || { echo "[$e] failed"; tail -3 gpurun_out/det5_$i.log; exit 1; }
  echo "[$e] $(tail -1 gpurun_out/det5_$i.log)"
  i=$((i+1))
done

#!/bin/bash
# GPU box: the always-differing abvar/lb1 build with the upsample-add out of place (UBPL_UPADD_OOP=1)
# and with the caching allocator's blocks never reused inside the step (PYTORCH_NO_HIP_MEMORY_CACHING=1).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
i=0
for e in "UBPL_UPADD_OOP=1" "PYTORCH_NO_HIP_MEMORY_CACHING=1"; do
  UBPL_LIB_DIR=$PWD/abvar/lb1 env $e timeout -k 10 200 python tools/det_step.py mt_ubpl_b32 ${REPS:-6} > gpurun_out/det_s4k_$i.log 2>&1 || { echo "[$e] failed"; tail -3 gpurun_out/det_s4k_$i.log; exit 1; }
  echo "[lb1 $e] $(tail -1 gpurun_out/det_s4k_$i.log)"
  grep "first differing BN" gpurun_out/det_s4k_$i.log | head -2
  i=$((i+1))
done

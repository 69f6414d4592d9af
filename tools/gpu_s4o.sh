#!/bin/bash
# GPU box: the always-differing abvar/lb1 build with every queue of the process confined to a CU
# subset (HSA_CU_MASK): if the race needs the eight XCDs' separate L2s, one XCD's CUs should not show it.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
i=0
for m in "0:0-31" "0:0-127"; do
  HSA_CU_MASK=$m UBPL_LIB_DIR=$PWD/abvar/lb1 timeout -k 10 300 python tools/det_step.py mt_ubpl_b32 ${REPS:-5} > gpurun_out/det_s4o_$i.log 2>&1 || { echo "[$m] failed"; tail -3 gpurun_out/det_s4o_$i.log; exit 1; }
  echo "[HSA_CU_MASK=$m] $(tail -1 gpurun_out/det_s4o_$i.log)"
  grep "first differing BN" gpurun_out/det_s4o_$i.log | head -1
  i=$((i+1))
done

#!/bin/bash
# GPU box: the always-differing abvar/lb1 build on ONE stream (UBPL_MODEL_STREAMS=0) and with every
# kernel serialised by the runtime (AMD_SERIALIZE_KERNEL=3): is the race across streams or between
# consecutive kernels of one stream?
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
i=0
for e in "UBPL_MODEL_STREAMS=0" "AMD_SERIALIZE_KERNEL=3" "UBPL_MODEL_STREAMS=0 AMD_SERIALIZE_KERNEL=3"; do
  UBPL_LIB_DIR=$PWD/abvar/lb1 env $e timeout -k 10 200 python tools/det_step.py mt_ubpl_b32 ${REPS:-6} > gpurun_out/det_s4h_$i.log 2>&1 || { echo "[$e] failed"; tail -3 gpurun_out/det_s4h_$i.log; exit 1; }
  echo "[lb1 $e] $(tail -1 gpurun_out/det_s4h_$i.log)"
  grep "first differing BN" gpurun_out/det_s4h_$i.log | head -2
  i=$((i+1))
done

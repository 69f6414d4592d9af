#!/bin/bash
# GPU box (round 4, race item 1): the always-differing abvar/lb1 build (1x1 split-load kernel at launch
# bounds (256, 1)) under runtime settings and a BN hand-off variant, one det_step each:
#   lb1          baseline (expected: every repeat differs)
#   lb1 + HIP_FORCE_DEV_KERNARG=0           kernel arguments in host memory instead of device memory
#   lb1 + DEBUG_CLR_KERNARG_HDP_FLUSH_WA=1  the runtime's kernarg write-visibility workaround
#   lb1acq       BN last-arriver ticket with agent-scope acq_rel (bn.hip UBPL_BN_ACQREL)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
run() {   # name, lib variant, env...
  local n=$1 v=$2; shift 2
  env UBPL_LIB_DIR=$PWD/abvar/$v "$@" timeout -k 10 240 python tools/det_step.py mt_ubpl_b32 ${REPS:-4} \
      > gpurun_out/r04_race_$n.log 2>&1 || { echo "[$n] failed rc=$?"; tail -3 gpurun_out/r04_race_$n.log; exit 1; }
  echo "[$n] $(tail -1 gpurun_out/r04_race_$n.log)"
  grep "first differing BN" gpurun_out/r04_race_$n.log | head -1
}
run lb1 lb1
run kernarg_host lb1 HIP_FORCE_DEV_KERNARG=0
run kernarg_hdp lb1 DEBUG_CLR_KERNARG_HDP_FLUSH_WA=1
run acqrel lb1acq

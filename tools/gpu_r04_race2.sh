#!/bin/bash
# GPU box (round 4, race item 1, second pass): does a forwards-only run reproduce the
# always-differing abvar/lb1 build's divergence, and which kernel families / options matter.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
fwd() {   # name, lib variant, args, env...
  local n=$1 v=$2 a=$3; shift 3
  env UBPL_LIB_DIR=$PWD/abvar/$v "$@" timeout -k 10 200 python tools/fwd_race.py $a \
      > gpurun_out/r04_fwd_$n.log 2>&1 || { echo "[$n] failed rc=$?"; tail -3 gpurun_out/r04_fwd_$n.log; exit 1; }
  echo "[fwd $n] $(tail -1 gpurun_out/r04_fwd_$n.log)"
}
det() {   # name, lib variant, env...
  local n=$1 v=$2; shift 2
  env UBPL_LIB_DIR=$v "$@" timeout -k 10 240 python tools/det_step.py mt_ubpl_b32 ${REPS:-4} \
      > gpurun_out/r04_det_$n.log 2>&1 || { echo "[$n] failed rc=$?"; tail -3 gpurun_out/r04_det_$n.log; exit 1; }
  echo "[det $n] $(tail -1 gpurun_out/r04_det_$n.log)"
}
fwd lb1 lb1 "4 4 2"
fwd lb1_grad lb1 "4 4 2" FWD_GRAD=1
fwd lb1_2nets lb1 "4 2 2"
fwd lb1_onestream lb1 "4 4 2" FWD_STREAMS=0
det lb1_3xbf16 $PWD/abvar/lb1 UBPL_CONV_PRECISION=3xbf16
det lb1_bf16 $PWD/abvar/lb1 UBPL_CONV_PRECISION=bf16
det lb1_f32 $PWD/abvar/lb1 UBPL_CONV_PRECISION=f32
det lb1tepi0 $PWD/abvar/lb1tepi0
det lb1coef0 $PWD/abvar/lb1coef0
REPS=7 det default $PWD/ubpl-poseestimation_amd/ubpl_amd

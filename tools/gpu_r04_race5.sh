#!/bin/bash
# GPU box (round 4, race item 1, fifth pass): is the hourglass's low3 (the residual's output,
# split-K conv + reduce) already wrong before the upsample-add, and does split-K matter.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
fwd() {   # name, args, env...
  local n=$1 a=$2; shift 2
  env UBPL_CONV_PRECISION=3xbf16 "$@" timeout -k 10 200 python tools/fwd_race.py $a \
      > gpurun_out/r04_fwd5_$n.log 2>&1 || { echo "[$n] failed rc=$?"; tail -3 gpurun_out/r04_fwd5_$n.log; exit 1; }
  echo "[fwd $n] $(tail -1 gpurun_out/r04_fwd5_$n.log)"
}
fwd low3clone "5 4 2" FWD_LOCATE=1 UBPL_SAVE_LOW3=clone
fwd nosplitk "5 4 2" UBPL_NO_SPLITK=1
fwd nosplitk_locate "5 4 2" UBPL_NO_SPLITK=1 FWD_LOCATE=1
UBPL_LIB_DIR=$PWD/abvar/lb1 UBPL_NO_SPLITK=1 timeout -k 10 240 python tools/det_step.py mt_ubpl_b32 4 > gpurun_out/r04_det5_lb1_nosplitk.log 2>&1 || exit 1
echo "[det lb1 nosplitk] $(tail -1 gpurun_out/r04_det5_lb1_nosplitk.log)"
grep "first differing" gpurun_out/r04_fwd5_low3clone.log | head -12
grep "first differing" gpurun_out/r04_fwd5_nosplitk_locate.log | head -12

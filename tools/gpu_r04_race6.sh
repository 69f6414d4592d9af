#!/bin/bash
# GPU box (round 4, race item 1, sixth pass): the upsample-add's output is wrong while both of its
# operands are right; with an agent-scope acquire fence (L2 invalidate) at the start of every
# upsample-add workgroup (abvar/upfence, abvar/lb1upfence), does the divergence go away?
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
fwd() {   # name, lib, args, env...
  local n=$1 v=$2 a=$3; shift 3
  env UBPL_LIB_DIR=$PWD/abvar/$v UBPL_CONV_PRECISION=3xbf16 "$@" timeout -k 10 200 python tools/fwd_race.py $a \
      > gpurun_out/r04_fwd6_$n.log 2>&1 || { echo "[$n] failed rc=$?"; tail -3 gpurun_out/r04_fwd6_$n.log; exit 1; }
  echo "[fwd $n] $(tail -1 gpurun_out/r04_fwd6_$n.log)"
}
fwd upfence upfence "6 4 2"
fwd upfence_locate upfence "5 4 2" FWD_LOCATE=1
UBPL_LIB_DIR=$PWD/abvar/lb1upfence timeout -k 10 240 python tools/det_step.py mt_ubpl_b32 4 > gpurun_out/r04_det6_lb1upfence.log 2>&1 || exit 1
echo "[det lb1upfence] $(tail -1 gpurun_out/r04_det6_lb1upfence.log)"
grep "first differing" gpurun_out/r04_fwd6_upfence_locate.log | head -12
grep "first differing BN" gpurun_out/r04_det6_lb1upfence.log | head -4

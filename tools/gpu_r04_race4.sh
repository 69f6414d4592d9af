#!/bin/bash
# GPU box (round 4, race item 1, fourth pass): locate the first differing saved activation in the
# 100 % reproducer (3xbf16 forwards on 4 streams, default build) and vary the HW queue count.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
fwd() {   # name, args, env...
  local n=$1 a=$2; shift 2
  env UBPL_CONV_PRECISION=3xbf16 "$@" timeout -k 10 200 python tools/fwd_race.py $a \
      > gpurun_out/r04_fwd4_$n.log 2>&1 || { echo "[$n] failed rc=$?"; tail -3 gpurun_out/r04_fwd4_$n.log; exit 1; }
  echo "[fwd $n] $(tail -1 gpurun_out/r04_fwd4_$n.log)"
}
fwd locate "5 4 2" FWD_LOCATE=1
fwd locate_oop "5 4 2" FWD_LOCATE=1 UBPL_UPADD_OOP=1
fwd nets2 "5 2 2"
fwd nets2v1 "5 2 1"
fwd q8 "5 4 2" GPU_MAX_HW_QUEUES=8
fwd q1 "5 4 2" GPU_MAX_HW_QUEUES=1
fwd q2 "5 4 2" GPU_MAX_HW_QUEUES=2
grep "first differing" gpurun_out/r04_fwd4_locate.log | head -20
grep "first differing" gpurun_out/r04_fwd4_locate_oop.log | head -20

#!/bin/bash
# GPU box (round 4, race item 1, third pass): forwards only on the DEFAULT build; the 3xbf16
# precision (register-staged split kernel only: no LDS-DMA, no PSA / split-load kernels) and the
# default 6xbf16, with memory reuse and the per-forward weight re-layouts switched off in turn.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
fwd() {   # name, args, env...
  local n=$1 a=$2; shift 2
  env "$@" timeout -k 10 200 python tools/fwd_race.py $a \
      > gpurun_out/r04_fwd3_$n.log 2>&1 || { echo "[$n] failed rc=$?"; tail -3 gpurun_out/r04_fwd3_$n.log; exit 1; }
  echo "[fwd $n] $(tail -1 gpurun_out/r04_fwd3_$n.log)"
}
fwd 3x "5 4 2" UBPL_CONV_PRECISION=3xbf16
fwd 3x_keep1 "5 4 2" UBPL_CONV_PRECISION=3xbf16 FWD_KEEPALL=1
fwd 3x_keep2 "5 4 2" UBPL_CONV_PRECISION=3xbf16 FWD_KEEPALL=2
fwd 3x_once "5 4 2" UBPL_CONV_PRECISION=3xbf16 UBPL_RELAYOUT_ONCE=1
fwd 3x_nocache "5 4 2" UBPL_CONV_PRECISION=3xbf16 PYTORCH_NO_HIP_MEMORY_CACHING=1
fwd 6x "5 4 2"
fwd 6x_keep2 "5 4 2" FWD_KEEPALL=2
fwd 6x_once "5 4 2" UBPL_RELAYOUT_ONCE=1
fwd f32 "5 4 2" UBPL_CONV_PRECISION=f32

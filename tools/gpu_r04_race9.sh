#!/bin/bash
# GPU box (round 4, race item 1, ninth pass): the upsample-add's wrong elements are exactly the
# low halves of its second v_pk_add_f32 (op_sel:[0,1]) for one 16-lane pass: builds without
# packed-FP32 instructions (abvar/nopk, abvar/lb1nopk: -target-feature -packed-fp32-ops).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
env UBPL_LIB_DIR=$PWD/abvar/nopk UBPL_CONV_PRECISION=3xbf16 timeout -k 10 200 python tools/fwd_race.py 6 4 2 \
    > gpurun_out/r04_fwd9_nopk.log 2>&1 || { tail -3 gpurun_out/r04_fwd9_nopk.log; exit 1; }
echo "[fwd 3xbf16 nopk] $(tail -1 gpurun_out/r04_fwd9_nopk.log)"
env UBPL_CONV_PRECISION=3xbf16 timeout -k 10 200 python tools/fwd_race.py 4 4 2 \
    > gpurun_out/r04_fwd9_base.log 2>&1 || { tail -3 gpurun_out/r04_fwd9_base.log; exit 1; }
echo "[fwd 3xbf16 default] $(tail -1 gpurun_out/r04_fwd9_base.log)"
UBPL_LIB_DIR=$PWD/abvar/lb1nopk timeout -k 10 240 python tools/det_step.py mt_ubpl_b32 5 > gpurun_out/r04_det9_lb1nopk.log 2>&1 || exit 1
echo "[det lb1nopk] $(tail -1 gpurun_out/r04_det9_lb1nopk.log)"
UBPL_LIB_DIR=$PWD/abvar/nopk timeout -k 10 240 python tools/det_step.py mt_ubpl_b32 8 > gpurun_out/r04_det9_nopk.log 2>&1 || exit 1
echo "[det nopk] $(tail -1 gpurun_out/r04_det9_nopk.log)"

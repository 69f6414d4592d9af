#!/bin/bash
# GPU box (round 4, race item 1, eighth pass): what the upsample-add's wrong output elements hold.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
env UBPL_CONV_PRECISION=3xbf16 FWD_LOCATE=1 UBPL_SAVE_LOW3=add timeout -k 10 200 python tools/fwd_race.py 5 4 2 \
    > gpurun_out/r04_fwd8_add.log 2>&1 || { tail -3 gpurun_out/r04_fwd8_add.log; exit 1; }
tail -1 gpurun_out/r04_fwd8_add.log
grep "wrong" gpurun_out/r04_fwd8_add.log | head -30
env UBPL_CONV_PRECISION=3xbf16 FWD_LOCATE=1 UBPL_SAVE_LOW3=add UBPL_UPADD_OOP=1 timeout -k 10 200 python tools/fwd_race.py 5 4 2 \
    > gpurun_out/r04_fwd8_add_oop.log 2>&1 || { tail -3 gpurun_out/r04_fwd8_add_oop.log; exit 1; }
tail -1 gpurun_out/r04_fwd8_add_oop.log
grep "differing" gpurun_out/r04_fwd8_add_oop.log | head -10

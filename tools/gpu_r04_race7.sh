#!/bin/bash
# GPU box (round 4, race item 1, seventh pass): clones of the upsample-add's operands right before
# it and of its result right after it: is the result wrong when written, or overwritten later?
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
env UBPL_CONV_PRECISION=3xbf16 FWD_LOCATE=1 UBPL_SAVE_LOW3=add FWD_SHOW=4 timeout -k 10 200 python tools/fwd_race.py 5 4 2 \
    > gpurun_out/r04_fwd7_add.log 2>&1 || { tail -3 gpurun_out/r04_fwd7_add.log; exit 1; }
tail -1 gpurun_out/r04_fwd7_add.log
grep "differing" gpurun_out/r04_fwd7_add.log | head -40

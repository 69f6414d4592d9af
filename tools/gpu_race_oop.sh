#!/bin/bash
# GPU box: graph-race locate pass with the upsample-add out of place (up1 saved), per VERDICT r2 item 7
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
UBPL_UPADD_OOP=1 timeout -k 10 300 python tools/graph_fwd_probe.py ${REPS:-80} 4 2 0 locate > gpurun_out/race_oop.log 2>&1
rc=$?; tail -25 gpurun_out/race_oop.log; exit $rc

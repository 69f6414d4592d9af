#!/bin/bash
# tests (+smoke) then bench (+optional rocprof); stops after a crash/timeout (rc >= 124).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
bash tools/gpu_check.sh
rc=$?
if [ $rc -ge 124 ]; then echo "check rc=$rc: stopping"; exit $rc; fi
bash tools/gpu_bench.sh

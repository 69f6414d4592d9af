#!/bin/bash
# GPU-box check: smoke, then the -m gpu suite.  Each GPU step has its own time
# limit; a crash / timeout / abort (rc >= 124) stops the script before the next
# GPU step (an ordinary assertion failure, rc 1, does not).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export PYTHONDONTWRITEBYTECODE=1
mkdir -p gpurun_out
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1
rc=$?; echo "smoke rc=$rc" >> gpurun_out/smoke.log; tail -3 gpurun_out/smoke.log
if [ $rc -ge 124 ]; then exit $rc; fi
timeout -k 10 ${GPU_TEST_TIMEOUT:-900} python -u -m pytest ${GPU_TESTS:-tests} -m gpu -q --timeout 300 --timeout-method thread -p no:cacheprovider -rf > gpurun_out/gpu_tests.log 2>&1
rc=$?; echo "tests rc=$rc" >> gpurun_out/gpu_tests.log; tail -25 gpurun_out/gpu_tests.log
exit $rc

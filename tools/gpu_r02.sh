#!/bin/bash
# GPU box: the given test files (default: the whole -m gpu suite), then optionally the bench.
# Every GPU step has its own time limit; the script stops at the first failure.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export PYTHONDONTWRITEBYTECODE=1
mkdir -p gpurun_out
TESTS=${TESTS:-tests}
timeout -k 10 ${TEST_TIMEOUT:-900} python -u -m pytest $TESTS -m gpu -x -v --timeout 120 --timeout-method thread \
    ${PYTEST_ARGS} > gpurun_out/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "passed|failed|error" gpurun_out/pytest.log | tail -3
if [ $rc -ne 0 ]; then grep -E "^(FAILED|ERROR)|Error|assert" gpurun_out/pytest.log | head -20; exit $rc; fi
if [ -n "$BENCH" ]; then
  timeout -k 10 600 python bench.py --steps ${STEPS:-10} --warmup ${WARM:-3} ${BENCH_ARGS} > gpurun_out/bench.json 2> gpurun_out/bench.err
  rc=$?; echo "bench rc=$rc"; cat gpurun_out/bench.json; tail -3 gpurun_out/bench.err
fi
exit $rc

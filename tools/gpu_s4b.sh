#!/bin/bash
# GPU box: split-kernel parity tests first, then the bf16-vs-6xbf16 loss-curve test on the in-tree build
# and on abvar/old (printing both curves), then the rest of the suite.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export PYTHONDONTWRITEBYTECODE=1
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_split.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_split.log 2>&1
rc=$?; tail -3 gpurun_out/pytest_split.log; [ $rc -ne 0 ] && { grep -E "^(FAILED|ERROR)|Error|assert" gpurun_out/pytest_split.log | head -20; exit $rc; }
for v in new old; do
  e=""; [ $v = old ] && e="UBPL_LIB_DIR=$PWD/abvar/old"
  env $e timeout -k 10 400 python -u -m pytest "tests/test_gpu_hourglass.py::test_bf16_precision_trains_like_fp32" -m gpu -q -s --timeout 300 --timeout-method thread > gpurun_out/pytest_bf16_$v.log 2>&1
  echo "== $v rc=$?"; grep -E "6xbf16|bf16  |passed|failed" gpurun_out/pytest_bf16_$v.log | cut -c1-220
done

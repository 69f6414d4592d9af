#!/bin/bash
# GPU box (round 4): 128-pixel conv1x1_sol_kernel tiles (UBPL_SOL_BN=128, three workgroups per CU):
# the split tests on that setting, the 1x1 microbench A/B, the headline bench A/B.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
UBPL_SOL_BN=128 timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_split.py \
    > gpurun_out/r04_sol_t.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -2 gpurun_out/r04_sol_t.log; [ $rc -ne 0 ] && exit $rc
for v in 256 128; do
  echo "== sol bn=$v"; UBPL_SOL_BN=$v timeout -k 10 200 python tools/conv1x1_bench.py 32 20 2>&1 | grep " sol " || exit 1
done
for v in 128 256 128 256; do
  UBPL_SOL_BN=$v timeout -k 10 300 python bench.py --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/r04_sol_b$v.json 2>/dev/null || { echo "bench $v failed"; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/r04_sol_b$v.json'));print('head sol bn $v:', d['value'], 'img/s')"
done

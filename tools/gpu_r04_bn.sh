#!/bin/bash
# GPU box (round 4): small-plane BatchNorm statistics with their loads issued together (bn.hip):
# kernel / split / hourglass / train tests, the BN microbench and the headline bench, each A/B
# against the previous bn.hip (abvar/OLDBN).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
[ -n "$SKIP_TESTS" ] || timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_kernels.py \
    tests/test_gpu_split.py tests/test_gpu_hourglass.py tests/test_gpu_train.py > gpurun_out/r04_bn_t.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -2 gpurun_out/r04_bn_t.log; [ $rc -ne 0 ] && exit $rc
for v in intree OLDBN; do
  d=""; [ $v != intree ] && d="UBPL_LIB_DIR=$PWD/abvar/$v"
  echo "== bn $v"; env $d timeout -k 10 200 python tools/bn_bench.py 32 50 || exit 1
done
for v in intree OLDBN; do
  d=""; [ $v != intree ] && d="UBPL_LIB_DIR=$PWD/abvar/$v"
  env $d timeout -k 10 300 python bench.py --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/r04_bn_$v.json 2>/dev/null || { echo "bench $v failed"; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/r04_bn_$v.json'));print('head $v:', d['value'], 'img/s')"
done

#!/bin/bash
# GPU box (round 4): a 4-stage A ring in the one-buffer halo kernel where the LDS allows (the
# 64-row tiles; abvar/NA4) vs 3 stages: bit-identity, PSA microbench, headline bench.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
UBPL_LIB_DIR=$PWD/abvar/NA4 timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_split.py -k halo \
    > gpurun_out/r04_na4_t.log 2>&1
rc=$?; echo "halo tests (NA4) rc=$rc"; tail -1 gpurun_out/r04_na4_t.log; [ $rc -ne 0 ] && exit $rc
for v in intree NA4 intree NA4; do
  d=""; [ $v != intree ] && d="UBPL_LIB_DIR=$PWD/abvar/$v"
  echo "== $v"; env $d timeout -k 10 120 python tools/psa_bench.py 32 50 3 || exit 1
done
for v in intree NA4; do
  d=""; [ $v != intree ] && d="UBPL_LIB_DIR=$PWD/abvar/$v"
  env $d timeout -k 10 300 python bench.py --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/r04_na4_$v.json 2>/dev/null || { echo "bench $v failed"; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/r04_na4_$v.json'));print('head $v:', d['value'], 'img/s')"
done

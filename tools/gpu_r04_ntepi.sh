#!/bin/bash
# GPU box (round 4): conv epilogue stores non-temporal (abvar/NTEPI) vs default: PSA / 1x1
# microbench and the headline bench, same box.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for v in intree NTEPI; do
  d=""; [ $v != intree ] && d="UBPL_LIB_DIR=$PWD/abvar/$v"
  echo "== $v"; env $d timeout -k 10 120 python tools/psa_bench.py 32 50 3 || exit 1
  env $d timeout -k 10 200 python tools/conv1x1_bench.py 32 20 2>&1 | grep " sol " | head -8 || exit 1
done
for v in intree NTEPI intree NTEPI; do
  d=""; [ $v != intree ] && d="UBPL_LIB_DIR=$PWD/abvar/$v"
  env $d timeout -k 10 300 python bench.py --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/r04_ntepi_$v.json 2>/dev/null || { echo "bench $v failed"; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/r04_ntepi_$v.json'));print('head $v:', d['value'], 'img/s; roofline', d['roofline']['avg_launch_us'])"
done

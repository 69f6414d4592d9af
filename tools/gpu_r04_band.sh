#!/bin/bash
# GPU box (round 4): banded halo refill in the one-buffer halo kernel (rows refilled as they fall
# out of use): bit-identity tests, then the PSA microbench A/B against the whole-halo reload
# (abvar/NOBAND, UBPL_PSAH_BAND=0) and the headline bench.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_split.py -k halo \
    > gpurun_out/r04_band_t.log 2>&1
rc=$?; echo "halo tests rc=$rc"; tail -2 gpurun_out/r04_band_t.log; [ $rc -ne 0 ] && exit $rc
for v in intree NOBAND intree NOBAND; do
  d=""; [ $v != intree ] && d="UBPL_LIB_DIR=$PWD/abvar/$v"
  echo "== $v"; env $d timeout -k 10 120 python tools/psa_bench.py 32 50 3 || exit 1
done
for v in intree NOBAND intree; do
  d=""; [ $v != intree ] && d="UBPL_LIB_DIR=$PWD/abvar/$v"
  env $d timeout -k 10 300 python bench.py --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/r04_band_$v.json 2>/dev/null || { echo "bench $v failed"; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/r04_band_$v.json'));print('head $v:', d['value'], 'img/s; roofline', d['roofline']['avg_launch_us'], d['roofline']['frac'])"
done

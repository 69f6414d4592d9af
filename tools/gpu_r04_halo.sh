#!/bin/bash
# GPU box (round 4): conv_psah_kernel (3x3 input halo staged once per channel group):
# bit-identity vs conv_psa_kernel + f64 bar, microbench A/B (UBPL_PSA_HALO=0/1), timing-only
# diagnostics of conv_psa_kernel (abvar/NODMA, abvar/NOREAD), then the split / hourglass / train
# tests and the headline bench A/B.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_split.py -k halo \
    > gpurun_out/r04_halo_t1.log 2>&1
rc=$?; echo "halo tests rc=$rc"; tail -3 gpurun_out/r04_halo_t1.log; [ $rc -ne 0 ] && exit $rc
for v in "0 1" "1 1" "1 2"; do
  set -- $v
  echo "== halo=$1 teams=$2"; UBPL_PSA_HALO=$1 UBPL_PSA_TEAMS=$2 timeout -k 10 120 python tools/psa_bench.py 32 50 || exit 1
done
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_split.py \
    tests/test_gpu_hourglass.py tests/test_gpu_race.py tests/test_gpu_train.py > gpurun_out/r04_halo_t2.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 gpurun_out/r04_halo_t2.log; [ $rc -ne 0 ] && exit $rc
for v in 1 0 1; do
  UBPL_PSA_HALO=$v timeout -k 10 300 python bench.py --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/r04_halo_b$v.json 2>/dev/null || { echo "bench halo$v failed"; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/r04_halo_b$v.json'));print('head halo $v:', d['value'], 'img/s; roofline', d['roofline']['avg_launch_us'], 'us frac', d['roofline']['frac'])"
done

#!/bin/bash
# GPU box (round 4): wave-uniform wave ids (spill-free halo kernels), unguarded full-tile
# epilogues, the default halo policy: kernel / hourglass / race / train tests, the PSA and 1x1
# microbenches, then the headline bench A/B against UBPL_PSA_HALO=0.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_split.py \
    tests/test_gpu_hourglass.py tests/test_gpu_race.py tests/test_gpu_train.py > gpurun_out/r04_halo6_t.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 gpurun_out/r04_halo6_t.log; [ $rc -ne 0 ] && exit $rc
for v in 0 d 3 1; do
  e="UBPL_X=1"; [ $v != d ] && e="UBPL_PSA_HALO=$v"
  echo "== psa halo=$v"; env $e timeout -k 10 120 python tools/psa_bench.py 32 50 3 || exit 1
done
echo "== conv1x1"; timeout -k 10 200 python tools/conv1x1_bench.py 32 20 2>&1 | grep " sol " || exit 1
for v in d 0 d 0; do
  e="UBPL_X=1"; [ $v = 0 ] && e="UBPL_PSA_HALO=0"
  env $e timeout -k 10 300 python bench.py --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/r04_halo6_b$v.json 2>/dev/null || { echo "bench $v failed"; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/r04_halo6_b$v.json'));print('head halo $v:', d['value'], 'img/s; roofline', d['roofline']['avg_launch_us'])"
done

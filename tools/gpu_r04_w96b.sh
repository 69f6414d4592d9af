#!/bin/bash
# GPU box (round 4): the one-piece (bf16) halo kernel on the 96-wide planes: bit-identity tests,
# the 96x96 bf16 microbench A/B and the configs[4] bf16 bench A/B (HG8 384x384).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_split.py -k halo \
    > gpurun_out/r04_w96b_t.log 2>&1
rc=$?; echo "halo tests rc=$rc"; tail -2 gpurun_out/r04_w96b_t.log; [ $rc -ne 0 ] && exit $rc
for v in 0 d; do
  e="UBPL_X=1"; [ $v != d ] && e="UBPL_PSA_HALO=$v"
  echo "== 96 bf16 halo=$v"; env $e PSA_BENCH_96=1 timeout -k 10 120 python tools/psa_bench.py 16 30 1 || exit 1
done
for v in d 0; do
  e="UBPL_X=1"; [ $v != d ] && e="UBPL_PSA_HALO=$v"
  env $e timeout -k 10 400 python bench.py --config mt_ubpl_hg8_384_bf16 --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/r04_w96b_c5$v.json 2>/dev/null || { echo "bench $v failed"; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/r04_w96b_c5$v.json'));print('hg8 384 bf16 halo $v:', d['value'], 'img/s; roofline', d['roofline']['avg_launch_us'], d['roofline']['frac'])"
done

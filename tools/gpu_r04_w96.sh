#!/bin/bash
# GPU box (round 4): the halo kernel on the 96-wide planes (192-pixel tiles): bit-identity tests,
# the 96x96 microbench A/B, the HG8 384x384 bench A/B (configs[4], 6xbf16).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_split.py -k halo \
    > gpurun_out/r04_w96_t.log 2>&1
rc=$?; echo "halo tests rc=$rc"; tail -2 gpurun_out/r04_w96_t.log; [ $rc -ne 0 ] && exit $rc
for v in 0 d; do
  e="UBPL_X=1"; [ $v != d ] && e="UBPL_PSA_HALO=$v"
  echo "== 96 halo=$v"; env $e PSA_BENCH_96=1 timeout -k 10 120 python tools/psa_bench.py 16 30 3 || exit 1
done
for v in d 0; do
  e="UBPL_X=1"; [ $v != d ] && e="UBPL_PSA_HALO=$v"
  env $e timeout -k 10 400 python bench.py --config mt_ubpl_hg8_384 --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/r04_w96_c4$v.json 2>/dev/null || { echo "bench $v failed"; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/r04_w96_c4$v.json'));print('hg8 384 halo $v:', d['value'], 'img/s; roofline', d['roofline']['avg_launch_us'], d['roofline']['frac'])"
done

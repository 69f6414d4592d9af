#!/bin/bash
# GPU box (round 4): (1) the split-path kernel tests (bf16 PSA now at KSUB=2); (2) the bf16 headline
# line at UBPL_PSA_KSUB1 = 1..4; (3) the headline with GPU_MAX_HW_QUEUES=8 vs default (graph replay).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_split.py \
    "tests/test_gpu_config5.py::test_headline_bf16_step_trains_like_6xbf16" > gpurun_out/r04_ab1_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -2 gpurun_out/r04_ab1_tests.log; [ $rc -ne 0 ] && exit $rc
for k in 1 2 3 4 2 1; do
  UBPL_PSA_KSUB1=$k timeout -k 10 300 python bench.py --config mt_ubpl_hg2_256_bf16 --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/r04_ab1_hb_$k.json 2>/dev/null || { echo "bench ksub $k failed"; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/r04_ab1_hb_$k.json'));print('hb ksub $k:', d['value'], 'img/s; roofline', d['roofline']['avg_launch_us'], 'us frac', d['roofline']['frac'])"
done
for q in 8 default 8 default; do
  e="UBPL_X=1"; [ $q = 8 ] && e="GPU_MAX_HW_QUEUES=8"
  env $e timeout -k 10 300 python bench.py --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/r04_ab1_q$q.json 2>/dev/null || { echo "bench q$q failed"; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/r04_ab1_q$q.json'));print('head queues $q:', d['value'], 'img/s')"
done

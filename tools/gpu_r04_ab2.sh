#!/bin/bash
# GPU box (round 4): the warp-specialized conv_psa_kernel (UBPL_PSA_WS, default on): kernel and step
# tests, then a same-box bench A/B against the 256-thread kernel (UBPL_PSA_WS=0).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_split.py \
    tests/test_gpu_hourglass.py tests/test_gpu_race.py tests/test_gpu_train.py \
    > gpurun_out/r04_ab2_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 gpurun_out/r04_ab2_tests.log; [ $rc -ne 0 ] && exit $rc
for w in 1 0 1 0; do
  UBPL_PSA_WS=$w timeout -k 10 300 python bench.py --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/r04_ab2_ws$w.json 2>/dev/null || { echo "bench ws$w failed"; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/r04_ab2_ws$w.json'));print('head ws $w:', d['value'], 'img/s; roofline', d['roofline']['avg_launch_us'], 'us frac', d['roofline']['frac'])"
done

#!/bin/bash
# GPU box (round 4): the halo kernel as the 6xbf16 default (one halo buffer, two workgroups per CU):
# kernel / hourglass / race / train tests, the headline bench A/B against UBPL_PSA_HALO=0, then
# rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes over the bench command for roofline.traffic.
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_split.py \
    tests/test_gpu_hourglass.py tests/test_gpu_race.py tests/test_gpu_train.py > gpurun_out/r04_halo7_t.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -2 gpurun_out/r04_halo7_t.log; [ $rc -ne 0 ] && exit $rc
for v in d 0 d; do
  e="UBPL_X=1"; [ $v = 0 ] && e="UBPL_PSA_HALO=0"
  env $e timeout -k 10 300 python bench.py --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/r04_halo7_b$v.json 2>/dev/null || { echo "bench $v failed"; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/r04_halo7_b$v.json'));print('head halo $v:', d['value'], 'img/s; roofline', d['roofline']['avg_launch_us'], d['roofline']['frac'])"
done
OUT=gpurun_out/pmc_r04h; mkdir -p $OUT
for c in FETCH_SIZE WRITE_SIZE; do
  n=$(echo $c | cut -d_ -f1 | tr A-Z a-z)
  UBPL_STEP_GRAPH=0 timeout -k 10 600 rocprofv3 --pmc $c -d $OUT -o $n --output-format csv -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline > $OUT/$n.log 2>&1
  rc=$?; echo "pmc $n rc=$rc"; [ $rc -ne 0 ] && exit $rc
done
python3 tools/pmc_roofline.py $OUT gpurun_out/pmc_roofline_psah.json "profiles/r04: rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes over bench.py --steps 2 --warmup 1 (eager step; tools/gpu_r04_halo7.sh), round-4 halo kernel" psah
rm -f $OUT/*.csv

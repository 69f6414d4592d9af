#!/bin/bash
# GPU box (round 4, final code): the whole -m gpu suite, the headline bench with its CPU baseline,
# the bf16 line, PMC FETCH_SIZE / WRITE_SIZE passes for roofline.traffic, and a rocprofv3
# kernel trace of the headline bench.
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 600 --timeout-method thread > gpurun_out/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -1 gpurun_out/pytest.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 400 python bench.py > gpurun_out/bench_head.json 2> gpurun_out/bench_head.err || { echo "bench failed"; exit 1; }
python -c "import json;d=json.load(open('gpurun_out/bench_head.json'));print('head', d['value'], d['roofline']['avg_launch_us'], d['roofline']['frac'], d['cpu_baseline']['value'])"
timeout -k 10 300 python bench.py --config mt_ubpl_hg2_256_bf16 --no-cpu-baseline > gpurun_out/bench_hb.json 2>/dev/null || { echo "bench hb failed"; exit 1; }
python -c "import json;d=json.load(open('gpurun_out/bench_hb.json'));print('hb', d['value'])"
OUT=gpurun_out/pmc_r04f; mkdir -p $OUT
for c in FETCH_SIZE WRITE_SIZE; do
  n=$(echo $c | cut -d_ -f1 | tr A-Z a-z)
  UBPL_STEP_GRAPH=0 timeout -k 10 600 rocprofv3 --pmc $c -d $OUT -o $n --output-format csv -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline > $OUT/$n.log 2>&1
  rc=$?; echo "pmc $n rc=$rc"; [ $rc -ne 0 ] && exit $rc
done
python3 tools/pmc_roofline.py $OUT gpurun_out/pmc_roofline_psah.json "profiles/r04: rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes over bench.py --steps 2 --warmup 1 (eager step; tools/gpu_r04_final.sh), round-4 final code (halo kernel, non-temporal epilogue stores)" psah > /dev/null
rm -f $OUT/*.csv
mkdir -p gpurun_out/prof_head
timeout -k 10 500 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_head -o run --output-format csv -- python3 bench.py --steps 3 --warmup 2 --no-cpu-baseline > gpurun_out/prof_head.json 2> gpurun_out/prof_head.err
echo "prof rc=$?"

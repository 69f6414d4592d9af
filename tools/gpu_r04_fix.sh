#!/bin/bash
# GPU box (round 4): the race fix (no packed-FP32 instructions, two-phase backward) — the new
# repeatability tests, the graph-with-streams test as a real test, and a same-box bench A/B
# against the pre-fix build (abvar/pk: packed-FP32 instructions allowed).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_race.py \
    > gpurun_out/r04_fix_race_tests.log 2>&1; echo "race tests rc=$?"; grep -E "PASS|FAIL|Error|passed|failed" gpurun_out/r04_fix_race_tests.log | tail -8
timeout -k 10 400 python -u -m pytest -x -v --runxfail --timeout 300 --timeout-method thread \
    "tests/test_gpu_train.py::test_step_graph_with_model_streams_matches_eager" \
    > gpurun_out/r04_fix_graph_streams.log 2>&1; echo "graph+streams rc=$?"; grep -E "passed|failed" gpurun_out/r04_fix_graph_streams.log | tail -2
for v in new old new old; do
  if [ $v = old ]; then e="UBPL_LIB_DIR=$PWD/abvar/pk"; else e="UBPL_X=1"; fi
  env $e timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/r04_fix_bench_$v.json 2>/dev/null || { echo "bench $v failed"; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/r04_fix_bench_$v.json'));print('bench $v:', d['value'], 'img/s, roofline', d['roofline']['avg_launch_us'], 'us')"
done

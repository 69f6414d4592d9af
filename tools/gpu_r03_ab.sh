#!/bin/bash
# GPU box, round 3: same-box A/B/C of library variants (in-tree = new, abvar/old, abvar/pp) on the
# conv microbenchmarks, then the -m gpu suite on the in-tree build, then the bench per variant and
# the config-5 bf16 bench.  Every GPU step has its own time limit; the script stops at the first failure.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export PYTHONDONTWRITEBYTECODE=1
mkdir -p gpurun_out
R=$PWD
VARIANTS=${VARIANTS:-"new old solpp"}
libdir() { if [ "$1" = new ]; then echo ""; else echo "UBPL_LIB_DIR=$R/abvar/$1"; fi; }
if [ -z "$SKIP_MB" ]; then
for v in $VARIANTS; do
  for mb in "psa_bench.py 32 50" "conv1x1_bench.py 32 20" "wgrad_bench.py 32 20"; do
    n=$(echo $mb | cut -d. -f1)
    env $(libdir $v) timeout -k 10 180 python tools/$mb > gpurun_out/mb_${n}_$v.log 2>&1 || { echo "mb $n $v failed"; tail -5 gpurun_out/mb_${n}_$v.log; exit 1; }
  done
  echo "== $v"; grep -E "B=" gpurun_out/mb_psa_bench_$v.log | cut -c1-100
done
fi
if [ -z "$SKIP_TESTS" ]; then
  timeout -k 10 900 python -u -m pytest ${TESTS:-tests} -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/pytest.log 2>&1
  rc=$?; echo "pytest rc=$rc"; grep -E "passed|failed|error" gpurun_out/pytest.log | tail -3
  if [ $rc -ne 0 ]; then grep -E "^(FAILED|ERROR)|Error|assert" gpurun_out/pytest.log | head -20; exit $rc; fi
fi
for v in $VARIANTS; do
  env $(libdir $v) timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/bench_$v.json 2> gpurun_out/bench_$v.err || { echo "bench $v failed"; tail -5 gpurun_out/bench_$v.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/bench_$v.json'));print('bench $v:', d['value'], 'img/s', d['ms_per_step'], 'ms; roofline', d['roofline']['avg_launch_us'], 'us frac', d['roofline']['frac'])"
done
if [ -n "$CONFIG5" ]; then
  timeout -k 10 400 python bench.py --config mt_ubpl_hg8_384_bf16 --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/bench_c5.json 2> gpurun_out/bench_c5.err || { tail -5 gpurun_out/bench_c5.err; exit 1; }
  cat gpurun_out/bench_c5.json
fi
if [ -n "$PROF_C5" ]; then
  export TMPDIR=/tmp
  mkdir -p gpurun_out/prof_c5
  timeout -k 10 500 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_c5 -o run --output-format csv -- python3 bench.py --config mt_ubpl_hg8_384_bf16 --steps 3 --warmup 2 --no-cpu-baseline > gpurun_out/prof_c5.json 2> gpurun_out/prof_c5.err
  rc=$?; echo "prof c5 rc=$rc"; cat gpurun_out/prof_c5.json; find gpurun_out/prof_c5 -name "*.csv" | head
fi
if [ -n "$PROF_HEAD" ]; then
  export TMPDIR=/tmp
  mkdir -p gpurun_out/prof_head
  timeout -k 10 500 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_head -o run --output-format csv -- python3 bench.py --steps 5 --warmup 3 --no-cpu-baseline > gpurun_out/prof_head.json 2> gpurun_out/prof_head.err
  rc=$?; echo "prof head rc=$rc"; cat gpurun_out/prof_head.json; find gpurun_out/prof_head -name "*.csv" | head
fi

#!/bin/bash
# GPU box, round 3 session 4: same-box A/B of library variants (in-tree = new, abvar/<v>) on the PSA
# microbenchmark, then (unless SKIP_TESTS) the -m gpu suite on the in-tree build, then the bench per
# variant.  Each GPU step has its own time limit; the script stops at the first failure.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export PYTHONDONTWRITEBYTECODE=1
mkdir -p gpurun_out
R=$PWD
VARIANTS=${VARIANTS:-"new"}
libdir() { if [ "$1" = new ]; then echo ""; else echo "UBPL_LIB_DIR=$R/abvar/$1"; fi; }
if [ -z "$SKIP_MB" ]; then
  for r in 1 2; do
    for v in $VARIANTS; do
      env $(libdir $v) timeout -k 10 180 python tools/${MB:-psa_bench.py 32 50} > gpurun_out/mb_$v.log 2>&1 || { echo "mb $v failed"; tail -5 gpurun_out/mb_$v.log; exit 1; }
      echo "== $v r$r"; grep -E "B=" gpurun_out/mb_$v.log | cut -c1-150
      if [ -n "$MB2" ]; then
        env $(libdir $v) timeout -k 10 180 python tools/$MB2 > gpurun_out/mb2_$v.log 2>&1 || { echo "mb2 $v failed"; tail -5 gpurun_out/mb2_$v.log; exit 1; }
        grep -E "${MB2_GREP:-.}" gpurun_out/mb2_$v.log | cut -c1-150
      fi
    done
  done
fi
if [ -z "$SKIP_TESTS" ]; then
  timeout -k 10 900 python -u -m pytest ${TESTS:-tests} -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/pytest.log 2>&1
  rc=$?; echo "pytest rc=$rc"; grep -E "passed|failed|error" gpurun_out/pytest.log | tail -3
  if [ $rc -ne 0 ]; then grep -E "^(FAILED|ERROR)|Error|assert" gpurun_out/pytest.log | head -20; exit $rc; fi
fi
if [ -z "$SKIP_BENCH" ]; then
  for r in 1 2; do
    for v in $VARIANTS; do
      env $(libdir $v) timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/bench_$v.json 2> gpurun_out/bench_$v.err || { echo "bench $v failed"; tail -5 gpurun_out/bench_$v.err; exit 1; }
      python -c "import json;d=json.load(open('gpurun_out/bench_$v.json'));print('bench $v r$r:', d['value'], 'img/s', d['ms_per_step'], 'ms; roofline', d['roofline']['avg_launch_us'], 'us frac', d['roofline']['frac'])"
    done
  done
fi

#!/bin/bash
# GPU box, round 4: the -m gpu suite (TESTS, default all; SKIP_TESTS=1 skips it), then the benches
# named in BENCHES ("head" = headline, "eager" = headline with UBPL_STEP_GRAPH=0, "hb" = headline
# shape on the bf16 precision, "c5" = config 5 bf16, "c4" = config 4 6xbf16, "c3" = DualPose HG4)
# and the rocprofv3 kernel traces named in PROFS.  Each GPU step has its own time limit; stops at
# the first failure.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export PYTHONDONTWRITEBYTECODE=1
mkdir -p gpurun_out
cfg() { case $1 in head|eager) echo mt_ubpl;; hb) echo mt_ubpl_hg2_256_bf16;; c5) echo mt_ubpl_hg8_384_bf16;; c4) echo mt_ubpl_hg8_384;; c3) echo dualpose_hg4;; esac; }
if [ -z "$SKIP_TESTS" ]; then
  timeout -k 10 1100 python -u -m pytest ${TESTS:-tests} -m gpu -x -v --timeout 600 --timeout-method thread > gpurun_out/pytest.log 2>&1
  rc=$?; echo "pytest rc=$rc"; grep -E "passed|failed|error" gpurun_out/pytest.log | tail -3
  if [ $rc -ne 0 ]; then grep -E "^(FAILED|ERROR)|Error|assert" gpurun_out/pytest.log | head -20; exit $rc; fi
fi
for b in $BENCHES; do
  e="UBPL_X=1"; [ $b = eager ] && e="UBPL_STEP_GRAPH=0"
  env $e timeout -k 10 400 python bench.py --config $(cfg $b) --steps ${STEPS:-20} --warmup 3 ${CPU:---no-cpu-baseline} > gpurun_out/bench_$b.json 2> gpurun_out/bench_$b.err || { echo "bench $b failed"; tail -5 gpurun_out/bench_$b.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/bench_$b.json'));r=d['roofline'] or {};print('bench $b:', d['value'], 'img/s', d['ms_per_step'], 'ms; roofline', r.get('avg_launch_us'), 'us frac', r.get('frac'))"
done
export TMPDIR=/tmp
for p in $PROFS; do
  mkdir -p gpurun_out/prof_$p
  timeout -k 10 500 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_$p -o run --output-format csv -- python3 bench.py --config $(cfg $p) --steps 3 --warmup 2 --no-cpu-baseline > gpurun_out/prof_$p.json 2> gpurun_out/prof_$p.err
  rc=$?; echo "prof $p rc=$rc"; [ $rc -ne 0 ] && exit $rc
done
exit 0

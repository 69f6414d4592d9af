#!/bin/bash
# GPU-box: bench line + rocprofv3 kernel-trace stats of the same command.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export PYTHONDONTWRITEBYTECODE=1
mkdir -p gpurun_out
STEPS=${STEPS:-10}; WARM=${WARM:-3}
timeout -k 10 ${BENCH_TIMEOUT:-600} python bench.py --steps $STEPS --warmup $WARM > gpurun_out/bench.json 2> gpurun_out/bench.err
rc=$?; echo "bench rc=$rc"; cat gpurun_out/bench.json; tail -5 gpurun_out/bench.err
if [ $rc -ne 0 ]; then exit $rc; fi
if [ -n "$PROFILE" ]; then
  cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
  timeout -k 10 ${PROF_TIMEOUT:-600} rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run --output-format csv -- python3 bench.py --steps $STEPS --warmup $WARM --no-cpu-baseline > gpurun_out/prof_bench.json 2> gpurun_out/prof.err
  rc=$?; echo "prof rc=$rc"; cat gpurun_out/prof_bench.json; ls -R gpurun_out/prof | head -20
fi
exit $rc

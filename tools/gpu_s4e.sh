#!/bin/bash
# GPU box, round 3 session 4 final: bench, rocprofv3 kernel trace + stats of the bench command,
# then the eager-step repeat statistics (tools/gpu_s4d.sh).
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$ROOT"; mkdir -p gpurun_out/prof
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/s4_bench.json 2> gpurun_out/s4_bench.err || { tail -5 gpurun_out/s4_bench.err; exit 1; }
cat gpurun_out/s4_bench.json
export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run --output-format csv -- python3 bench.py --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/prof_bench.json 2> gpurun_out/prof.err
rc=$?; echo "prof rc=$rc"; [ $rc -ne 0 ] && { tail -5 gpurun_out/prof.err; exit $rc; }
find gpurun_out/prof -name "*.csv" | head
bash tools/gpu_s4d.sh

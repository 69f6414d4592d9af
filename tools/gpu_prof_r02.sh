# GPU box: rocprofv3 kernel trace + stats of the bench command (round 2 profile)
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd /tmp && export TMPDIR=/tmp && cd "$ROOT"
mkdir -p gpurun_out/prof
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run --output-format csv -- python3 bench.py --steps ${STEPS:-10} --warmup ${WARM:-3} --no-cpu-baseline > gpurun_out/prof_bench.json 2> gpurun_out/prof.err
rc=$?; echo "prof rc=$rc"; cat gpurun_out/prof_bench.json; find gpurun_out/prof -name "*.csv" | head; exit $rc

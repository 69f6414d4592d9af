#!/bin/bash
# GPU box: same-box A/B of environment variants (ENVS = "A;B;C", each a space-separated env list,
# "-" = none): the microbenchmark MB (default the 1x1 bench) and the bench step, interleaved, R rounds.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export PYTHONDONTWRITEBYTECODE=1
mkdir -p gpurun_out
IFS=';' read -ra VS <<< "${ENVS:--}"
for r in $(seq 1 ${R:-1}); do
  i=0
  for v in "${VS[@]}"; do
    e=""; [ "$v" != "-" ] && e="$v"
    env $e timeout -k 10 180 python ${MB:-tools/conv1x1_bench.py 32 20} > gpurun_out/envab_mb_$i.log 2>&1 || { echo "mb [$v] failed"; tail -5 gpurun_out/envab_mb_$i.log; exit 1; }
    echo "== [$v] r$r"; grep -E "${MB_GREP:-sol}" gpurun_out/envab_mb_$i.log | head -${MB_LINES:-12}
    if [ -z "$NO_BENCH" ]; then
      env $e timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/envab_bench_$i.json 2> gpurun_out/envab_bench_$i.err || { echo "bench [$v] failed"; tail -5 gpurun_out/envab_bench_$i.err; exit 1; }
      python -c "import json;d=json.load(open('gpurun_out/envab_bench_$i.json'));print('bench [$v]:', d['value'], 'img/s', d['ms_per_step'], 'ms')"
    fi
    i=$((i+1))
  done
done

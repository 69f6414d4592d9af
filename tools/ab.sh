#!/bin/bash
# A/B the bench on one box: ab.sh "ENV=a" "ENV=b" [rounds]; prints value per run.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
A="$1"; B="$2"; R=${3:-2}
for i in $(seq 1 $R); do
  for e in "$A" "$B"; do
    env $e timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/ab.json 2> gpurun_out/ab.err || exit $?
    python -c "import json,sys; d=json.load(open('gpurun_out/ab.json')); print('$e', d['value'], d['ms_per_step'])"
  done
done

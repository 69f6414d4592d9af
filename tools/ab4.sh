#!/bin/bash
# bench under several env settings on one box: ab4.sh "ENV1" "ENV2" ... (one run each, twice around)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for i in 1 2; do
  for e in "$@"; do
    env $e timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/ab.json 2> gpurun_out/ab.err || exit $?
    python -c "import json,sys; d=json.load(open('gpurun_out/ab.json')); print('$e', d['value'], d['ms_per_step'])"
  done
done

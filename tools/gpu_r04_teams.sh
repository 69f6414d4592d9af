#!/bin/bash
# GPU box (round 4): headline bench A/B — the 128-row 6xbf16 halo launches on the two-team
# double-buffered variant (UBPL_PSA_HALO=4) vs the one-buffer default.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for v in 4 d 4 d; do
  e="UBPL_X=1"; [ $v != d ] && e="UBPL_PSA_HALO=$v"
  env $e timeout -k 10 300 python bench.py --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/r04_teams_$v.json 2>/dev/null || { echo "bench $v failed"; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/r04_teams_$v.json'));print('head halo $v:', d['value'], 'img/s; roofline', d['roofline']['avg_launch_us'])"
done

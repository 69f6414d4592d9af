#!/bin/bash
# GPU box (round 4): the halo kernel on the one-piece (bf16) path — microbench A/B and the bf16
# headline line with UBPL_PSA_HALO=0/1.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for v in "0 1" "1 1" "1 2"; do
  set -- $v
  echo "== bf16 halo=$1 teams=$2"; UBPL_PSA_HALO=$1 UBPL_PSA_TEAMS=$2 timeout -k 10 120 python tools/psa_bench.py 32 50 1 || exit 1
done
for v in 1 0 1 0; do
  UBPL_PSA_HALO=$v timeout -k 10 300 python bench.py --config mt_ubpl_hg2_256_bf16 --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/r04_halo3_hb$v.json 2>/dev/null || { echo "bench halo$v failed"; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/r04_halo3_hb$v.json'));print('bf16 head halo $v:', d['value'], 'img/s; roofline', d['roofline']['avg_launch_us'], 'us frac', d['roofline']['frac'])"
done

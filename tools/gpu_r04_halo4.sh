#!/bin/bash
# GPU box (round 4): halo kernel with exact-size halo images and a 3-stage A ring in the two-team
# variant: bit-identity tests, then the 6xbf16 and bf16 microbench A/B.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_split.py -k halo \
    > gpurun_out/r04_halo4_t1.log 2>&1
rc=$?; echo "halo tests rc=$rc"; tail -3 gpurun_out/r04_halo4_t1.log; [ $rc -ne 0 ] && exit $rc
for np in 3 1; do
for v in "0 1" "1 2" "1 1"; do
  set -- $v
  echo "== np=$np halo=$1 teams=$2"; UBPL_PSA_HALO=$1 UBPL_PSA_TEAMS=$2 timeout -k 10 120 python tools/psa_bench.py 32 50 $np || exit 1
done
done

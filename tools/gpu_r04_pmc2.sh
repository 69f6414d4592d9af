#!/bin/bash
# GPU box (round 4, final code): rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes over the bench
# command for roofline.traffic (the roofline kernel's name now carries its tile-width argument).
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/pmc_r04g; mkdir -p $OUT
for c in FETCH_SIZE WRITE_SIZE; do
  n=$(echo $c | cut -d_ -f1 | tr A-Z a-z)
  UBPL_STEP_GRAPH=0 timeout -k 10 600 rocprofv3 --pmc $c -d $OUT -o $n --output-format csv -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline > $OUT/$n.log 2>&1
  rc=$?; echo "pmc $n rc=$rc"; [ $rc -ne 0 ] && exit $rc
done
python3 tools/pmc_roofline.py $OUT gpurun_out/pmc_roofline_psah.json "profiles/r04: rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes over bench.py --steps 2 --warmup 1 (eager step; tools/gpu_r04_pmc2.sh), round-4 final code" psah
rm -f $OUT/*.csv

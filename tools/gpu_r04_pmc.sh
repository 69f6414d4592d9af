#!/bin/bash
# GPU box (round 4): rocprofv3 --pmc passes over the bench command (eager step, UBPL_STEP_GRAPH=0:
# the same kernels and launches as the captured step), one counter group per pass and process:
# FETCH_SIZE, WRITE_SIZE (roofline.traffic), and the SQ group (MFMA busy, VALU / LDS issue, waits).
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/pmc_r04; mkdir -p $OUT
bpass() {
  local name=$1; shift
  UBPL_STEP_GRAPH=0 timeout -k 10 600 rocprofv3 --pmc "$@" -d $OUT -o $name --output-format csv -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline > $OUT/$name.log 2>&1
  local rc=$?; echo "pmc bench $name rc=$rc"; return $rc
}
bpass fetch FETCH_SIZE && bpass write WRITE_SIZE && \
bpass sq SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT GRBM_GUI_ACTIVE
rc=$?
# summaries only: the per-dispatch CSVs exceed what gpurun copies back
python3 tools/pmc_roofline.py $OUT gpurun_out/r04_pmc_roofline_psa.json "profiles/r04: rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes over bench.py --steps 2 --warmup 1 (eager step; tools/gpu_r04_pmc.sh), round-4 code" psa > /dev/null
PMC_BY_GRID=1 python3 tools/pmc_summary.py $OUT gpurun_out/r04_pmc_conv_by_grid.json > /dev/null
rm -f $OUT/*.csv
exit $rc

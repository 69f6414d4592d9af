#!/bin/bash
# GPU box (round 4): what the one-buffer halo kernel's per-group halo reload costs — timing-only
# build without it (abvar/NORELOAD, stale halo) vs the in-tree build, and the PMC wait fractions.
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for v in intree NORELOAD intree NORELOAD; do
  d=""; [ $v != intree ] && d="UBPL_LIB_DIR=$PWD/abvar/$v"
  echo "== $v"; env $d timeout -k 10 120 python tools/psa_bench.py 32 50 3 || exit 1
done
OUT=gpurun_out/pmc_psah; mkdir -p $OUT
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT GRBM_GUI_ACTIVE -d $OUT -o sq --output-format csv -- python3 tools/psa_bench.py 32 20 > $OUT/log 2>&1
echo "pmc rc=$?"
PMC_BY_GRID=1 python3 tools/pmc_summary.py $OUT gpurun_out/r04_pmc_psah.json > /dev/null
rm -f $OUT/*.csv

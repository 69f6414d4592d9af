#!/bin/bash
# GPU box (round 4): SQ counters of conv_psa_kernel vs conv_psah_kernel (two teams) on
# tools/psa_bench.py (6xbf16, B=32): one pass per kernel choice, per-grid summaries only.
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/pmc_psa; mkdir -p $OUT
for v in "0 1 old" "1 2 halo2"; do
  set -- $v
  d=$OUT/$3; mkdir -p $d
  UBPL_PSA_HALO=$1 UBPL_PSA_TEAMS=$2 timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT GRBM_GUI_ACTIVE -d $d -o sq --output-format csv -- python3 tools/psa_bench.py 32 20 > $d/log 2>&1
  echo "pmc $3 rc=$?"
  PMC_BY_GRID=1 python3 tools/pmc_summary.py $d gpurun_out/r04_pmc_psa_$3.json > /dev/null
  rm -f $d/*.csv
done

#!/bin/bash
# Separate rocprofv3 --pmc passes (kernel trace only, no sys/runtime tracing)
# over tools/pmc_conv.py; each pass its own process.  Stops on the first failure.
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd /tmp && export TMPDIR=/tmp && cd "$ROOT"
OUT=${PMC_OUT:-gpurun_out/pmc}
mkdir -p $OUT
timeout -k 10 120 rocprofv3 -L > $OUT/counters_list.txt 2>&1 || true
pass() {
  local name=$1; shift
  timeout -k 10 300 rocprofv3 --pmc "$@" -d $OUT -o $name --output-format csv -- python3 ${WORKLOAD:-tools/pmc_conv.py} > $OUT/$name.log 2>&1
  local rc=$?
  echo "pmc $name rc=$rc"
  return $rc
}
if [ "$1" = "bench" ]; then
  # the same command as the bench line (short), counters per dispatch
  OUT=gpurun_out/pmc_bench; mkdir -p $OUT
  bpass() {
    local name=$1; shift
    timeout -k 10 600 rocprofv3 --pmc "$@" -d $OUT -o $name --output-format csv -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline > $OUT/$name.log 2>&1
    local rc=$?; echo "pmc bench $name rc=$rc"; return $rc
  }
  bpass fetch FETCH_SIZE && bpass write WRITE_SIZE
  exit $?
fi
pass sq SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT GRBM_GUI_ACTIVE && \
pass fetch FETCH_SIZE GRBM_GUI_ACTIVE && \
pass write WRITE_SIZE GRBM_GUI_ACTIVE

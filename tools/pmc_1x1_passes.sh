# GPU box: rocprofv3 --pmc passes over tools/pmc_1x1.py (conv1x1_sol_kernel, 64x64 B=32, SHAPE 0: 256->128 + BN
# prologue, the Residual conv1; SHAPE 1: 128->256 + prologue + residual, conv3), one counter set per run.
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd /tmp && export TMPDIR=/tmp && cd "$ROOT"
export ONLY_SOL=1 REPS=${REPS:-10}
for SHAPE in ${SHAPES:-0 1}; do
export SHAPE
OUT=${PMC_OUT:-gpurun_out/pmc_1x1}/s$SHAPE
mkdir -p $OUT
pass() {
  local name=$1; shift
  timeout -s KILL 90 rocprofv3 --pmc "$@" -d $OUT -o $name --output-format csv -- python3 tools/pmc_1x1.py > $OUT/$name.log 2>&1
  local rc=$?; echo "pmc s$SHAPE $name rc=$rc"; return $rc
}
pass sq SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT && \
pass sq2 SQ_WAVE_CYCLES SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_MISC SQ_BUSY_CYCLES GRBM_GUI_ACTIVE && \
pass fetch FETCH_SIZE && \
pass write WRITE_SIZE || exit 1
done

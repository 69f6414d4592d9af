# GPU box: rocprofv3 --pmc passes over tools/pmc_psa.py (conv_psa_kernel + wgrad3_psa_kernel at 64x64, B=32)
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd /tmp && export TMPDIR=/tmp && cd "$ROOT"
OUT=${PMC_OUT:-gpurun_out/pmc_psa}
mkdir -p $OUT
pass() {
  local name=$1; shift
  timeout -s KILL 90 rocprofv3 --pmc "$@" -d $OUT -o $name --output-format csv -- python3 tools/pmc_psa.py > $OUT/$name.log 2>&1
  local rc=$?; echo "pmc $name rc=$rc"; return $rc
}
pass sq SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT && \
pass sq2 SQ_WAVE_CYCLES SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_MISC SQ_BUSY_CYCLES GRBM_GUI_ACTIVE

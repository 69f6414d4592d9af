cd $GRAFT_REPO_ROOT
export PYTHONDONTWRITEBYTECODE=1
set -o pipefail
for mode in "default" "UBPL_MODEL_STREAMS=0" "UBPL_SPLIT_BWD=0" "UBPL_CONV_PRECISION=f32" "UBPL_MODEL_STREAMS=0 UBPL_CONV_PRECISION=f32"; do
  if [ "$mode" = default ]; then envs=""; else envs="$mode"; fi
  env $envs MODE="$mode" timeout -k 10 120 python tools/step_grad_diag.py mt_ubpl || exit 1
done

# GPU box: tools/step_grad_diag.py over execution modes (CASE, MODES env)
cd $GRAFT_REPO_ROOT
export PYTHONDONTWRITEBYTECODE=1
for mode in ${MODES:-default}; do
  if [ "$mode" = default ]; then envs=""; else envs="${mode//,/ }"; fi
  env $envs MODE="$mode" timeout -k 10 300 python tools/step_grad_diag.py ${CASE:-mt_ubpl} || exit 1
done

# GPU box: graph-vs-eager divergence counts of the captured MT_UBPL step per stream layout / env (MODES)
cd $GRAFT_REPO_ROOT
export PYTHONDONTWRITEBYTECODE=1 PROBE_STEPS=${PROBE_STEPS:-3}
REPS=${REPS:-8}
for mode in ${MODES:-base}; do
  if [ "$mode" = base ]; then envs=""; else envs="${mode//,/ }"; fi
  echo "== $mode"
  env $envs timeout -k 10 240 python tools/graph_race_probe.py $REPS graph 2>&1 | grep -v amdgpu.ids | tail -2 || exit 1
done

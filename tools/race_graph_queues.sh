mkdir -p gpurun_out
for cfg in "base" "DEBUG_HIP_FORCE_GRAPH_QUEUES=1" "DEBUG_HIP_GRAPH_BATCH_SIZE=1" "DEBUG_HIP_FORCE_GRAPH_QUEUES=4"; do
  if [ "$cfg" = base ]; then e=""; else e="$cfg"; fi
  echo "== $cfg"
  env $e timeout -k 10 150 python -u tools/graph_fwd_probe.py 100 4 2 > gpurun_out/race_$(echo $cfg | tr '=' '_').log 2>&1 || { echo "rc=$?"; tail -5 gpurun_out/race_$(echo $cfg | tr '=' '_').log; exit 1; }
  tail -1 gpurun_out/race_$(echo $cfg | tr '=' '_').log
done

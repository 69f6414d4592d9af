# GPU box: captured-step speed (UBPL_STEP_GRAPH=1, per-network streams) under HIP's graph-queue knob
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for q in ${QS:-default 1 2}; do
  if [ "$q" = default ]; then e=""; else e="DEBUG_HIP_FORCE_GRAPH_QUEUES=$q"; fi
  env $e UBPL_STEP_GRAPH=1 timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/gq_$q.json 2> gpurun_out/gq_$q.err || { echo "bench q=$q failed"; tail -3 gpurun_out/gq_$q.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/gq_$q.json'));print('graph queues $q:', d['value'], 'img/s', d['ms_per_step'], 'ms')"
done
timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/gq_eager.json 2>/dev/null && python -c "import json;d=json.load(open('gpurun_out/gq_eager.json'));print('eager:', d['value'], 'img/s')"

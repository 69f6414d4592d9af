# GPU box: same-box A/B of a kernel change — the in-tree libraries (new) against another build of them
# in $OLD (default build/ab_old, via UBPL_LIB_DIR): the PSA microbenchmark and the eager bench step, interleaved.
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
OLD=${OLD:-$GRAFT_REPO_ROOT/build/ab_old}
for r in 1 2; do
  for v in new old; do
    if [ $v = old ]; then e="UBPL_LIB_DIR=$OLD"; else e=""; fi
    env $e timeout -k 10 200 ${MB:-python tools/psa_bench.py 32 50} > gpurun_out/ab_mb_$v.log 2>&1 || { tail -3 gpurun_out/ab_mb_$v.log; exit 1; }
    echo "== microbench $v r$r"; grep -E "${MB_GREP:-B=}" gpurun_out/ab_mb_$v.log | head -${MB_LINES:-4} | cut -c1-90
  done
done
for r in 1 2; do
  for v in new old; do
    if [ $v = old ]; then e="UBPL_LIB_DIR=$OLD"; else e=""; fi
    env $e timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/ab_bench_$v.json 2>/dev/null || exit 1
    python -c "import json;d=json.load(open('gpurun_out/ab_bench_$v.json'));print('bench $v r$r:', d['value'], 'img/s, roofline', d['roofline']['avg_launch_us'], 'us')"
  done
done

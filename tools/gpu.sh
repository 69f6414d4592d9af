#!/bin/bash
# The one GPU-box launcher (round 5; replaces the ~75 one-off tools/gpu_*.sh of rounds 1-4, which
# stay in git history).  Every step runs under its own time limit; the script stops at the first
# failure, and after a crash / abort / time limit it starts nothing more on the GPU.
#
#   tools/gpu.sh STEP [STEP ...]      with the steps, in the order given:
#     smoke                 __graft_entry__.smoke()
#     tests                 pytest -m gpu over $TESTS (default: tests), -k "$K" when set
#     bench:<cfg>[:ENV=V,...]  python bench.py --config <cfg> (head = mt_ubpl, hb = mt_ubpl_hg2_256_bf16,
#                           c3 = dualpose_hg4, c4 = mt_ubpl_hg8_384, c5 = mt_ubpl_hg8_384_bf16);
#                           $STEPS timed steps (20), $WARM warm-up (3), the CPU baseline only with CPU=1
#     prof:<cfg>[:ENV=V,...]   rocprofv3 --kernel-trace --stats of a 3-step bench run, then
#                           tools/prof_summary.py over its timed window -> gpurun_out/prof_<cfg>.txt
#                           (labelled with the profiled/benched ms ratio when bench:<cfg> ran first)
#     pmc:bench             FETCH_SIZE / WRITE_SIZE passes over the bench (eager step) ->
#                           gpurun_out/pmc_roofline_$PMC_KIND.json (tools/pmc_roofline.py; psah2 default)
#     pmc:<script.py>       SQ instruction / wait counters (one pass) + FETCH / WRITE (one pass each)
#                           over a microbenchmark script -> gpurun_out/pmc_<name>/
#     ab:<ENV=a>|<ENV=b>[|...]  the bench under each setting, $AB_ROUNDS rounds (2), interleaved
#     run:<cmd with + for spaces>  any command (a microbenchmark), e.g. run:python+tools/psa_bench.py+32+20
#
# e.g. gpurun --timeout 1200 -- 'bash tools/gpu.sh tests bench:head prof:head'
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd /tmp && export TMPDIR=/tmp && cd "$ROOT" || exit 1
export PYTHONDONTWRITEBYTECODE=1
mkdir -p gpurun_out

cfg() { case $1 in head|eager) echo mt_ubpl;; hb) echo mt_ubpl_hg2_256_bf16;; c3) echo dualpose_hg4;;
                   c4) echo mt_ubpl_hg8_384;; c5) echo mt_ubpl_hg8_384_bf16;; *) echo $1;; esac; }
envs() { [ -n "$1" ] && echo "${1//,/ }"; }
stop() { echo "[$1] rc=$2: stopping"; exit $2; }

nrun=0
for step in "$@"; do
  kind=${step%%:*}; arg=${step#*:}; [ "$arg" = "$step" ] && arg=""
  name=${arg%%:*}; extra=${arg#*:}; [ "$extra" = "$arg" ] && extra=""
  case $kind in
    smoke)
      timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1
      rc=$?; tail -2 gpurun_out/smoke.log; [ $rc -ne 0 ] && stop smoke $rc ;;
    tests)
      timeout -k 10 ${TEST_TIMEOUT:-1100} python -u -m pytest ${TESTS:-tests} -m gpu -x -v ${K:+-k "$K"} \
          --timeout 600 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest.log 2>&1
      rc=$?; grep -E "passed|failed|error" gpurun_out/pytest.log | tail -2
      if [ $rc -ne 0 ]; then grep -E "^(FAILED|ERROR)|Error|assert" gpurun_out/pytest.log | head -20; stop tests $rc; fi ;;
    bench)
      c=$(cfg $name); [ $name = eager ] && extra="UBPL_STEP_GRAPH=0${extra:+,$extra}"
      tag=$name${extra:+_$(echo $extra | tr ',=/' '___')}
      env $(envs "$extra") timeout -k 10 ${BENCH_TIMEOUT:-500} python bench.py --config $c --steps ${STEPS:-20} \
          --warmup ${WARM:-3} $([ "$CPU" = 1 ] || echo --no-cpu-baseline) > gpurun_out/bench_$tag.json 2> gpurun_out/bench_$tag.err
      rc=$?; [ $rc -ne 0 ] && { tail -5 gpurun_out/bench_$tag.err; stop bench $rc; }
      python -c "import json;d=json.load(open('gpurun_out/bench_$tag.json'));r=d['roofline'] or {};print('bench $tag:', d['value'], 'img/s', d['ms_per_step'], 'ms; roofline', r.get('avg_launch_us'), 'us frac', r.get('frac'), '; cpu', (d['cpu_baseline'] or {}).get('value'))" ;;
    prof)
      c=$(cfg $name); tag=$name${extra:+_$(echo $extra | tr ',=/' '___')}
      rm -rf gpurun_out/prof_$tag; mkdir -p gpurun_out/prof_$tag
      env $(envs "$extra") timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_$tag -o run \
          --output-format csv -- python3 bench.py --config $c --steps 3 --warmup 2 --no-cpu-baseline \
          > gpurun_out/prof_$tag.json 2> gpurun_out/prof_$tag.err
      rc=$?; [ $rc -ne 0 ] && { tail -5 gpurun_out/prof_$tag.err; stop prof $rc; }
      tr=$(find gpurun_out/prof_$tag -name "*kernel_trace.csv" | head -1)
      python tools/prof_summary.py "$tr" 3 30 gpurun_out/bench_$tag.json > gpurun_out/prof_$tag.txt && head -12 gpurun_out/prof_$tag.txt
      python tools/trace_roofline.py "$tr" > gpurun_out/prof_${tag}_roofline.json 2>/dev/null || true
      find gpurun_out/prof_$tag -name "*kernel_trace.csv" -size +20M -delete ;;
    pmc)
      if [ "$name" = bench ]; then
        OUT=gpurun_out/pmc_bench; mkdir -p $OUT
        for c in FETCH_SIZE WRITE_SIZE; do
          n=$(echo $c | cut -d_ -f1 | tr A-Z a-z)
          UBPL_STEP_GRAPH=0 timeout -k 10 600 rocprofv3 --pmc $c -d $OUT -o $n --output-format csv -- \
              python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline > $OUT/$n.log 2>&1
          rc=$?; echo "pmc $n rc=$rc"; [ $rc -ne 0 ] && stop pmc $rc
        done
        python3 tools/pmc_roofline.py $OUT gpurun_out/pmc_roofline_${PMC_KIND:-psah2}.json \
            "rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes over bench.py --steps 2 --warmup 1 (eager step; tools/gpu.sh pmc:bench)" ${PMC_KIND:-psah2}
        rm -f $OUT/*.csv
      else
        # pmc:<script.py>[:ENV=V,...]: the script's environment (the program after -- stays python3)
        OUT=gpurun_out/pmc_$(basename $name .py)${extra:+_$(echo $extra | tr ',=/' '___')}; mkdir -p $OUT
        pass() {
          local n=$1; shift
          env $(envs "$extra") timeout -s KILL 120 rocprofv3 --pmc "$@" -d $OUT -o $n --output-format csv -- python3 $name > $OUT/$n.log 2>&1
          local rc=$?; echo "pmc $n rc=$rc"; [ $rc -ne 0 ] && stop pmc $rc
        }
        pass sq SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT
        pass sq2 SQ_WAVE_CYCLES SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_MISC SQ_BUSY_CYCLES SQ_VALU_MFMA_COEXEC_CYCLES GRBM_GUI_ACTIVE
        pass fetch FETCH_SIZE GRBM_GUI_ACTIVE
        pass write WRITE_SIZE GRBM_GUI_ACTIVE
        rm -f $OUT/*.csv.gz 2>/dev/null; true
      fi ;;
    ab)
      IFS='|' read -ra settings <<< "$arg"
      for r in $(seq 1 ${AB_ROUNDS:-2}); do
        for e in "${settings[@]}"; do
          env $(envs "$e") timeout -k 10 400 python bench.py --steps ${STEPS:-10} --warmup 3 --no-cpu-baseline \
              > gpurun_out/ab.json 2> gpurun_out/ab.err || { rc=$?; tail -3 gpurun_out/ab.err; stop ab $rc; }
          python -c "import json; d=json.load(open('gpurun_out/ab.json')); print('ab [$e] r$r', d['value'], d['ms_per_step'], (d['roofline'] or {}).get('avg_launch_us'))"
        done
      done ;;
    run)
      cmd=${arg//+/ }; nrun=$((nrun + 1))
      timeout -k 10 ${RUN_TIMEOUT:-300} $cmd > gpurun_out/run$nrun.log 2>&1
      rc=$?; echo "== run$nrun: $cmd"; grep -E "${RUN_GREP:-.}" gpurun_out/run$nrun.log | tail -${RUN_LINES:-30}
      [ $rc -ne 0 ] && stop run $rc ;;
    *) echo "unknown step $step"; exit 2 ;;
  esac
done
exit 0

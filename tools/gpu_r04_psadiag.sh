#!/bin/bash
# GPU box (round 4): what bounds conv_psa_kernel — timing-only builds with no LDS-DMA at all
# (abvar/NODMA: the compute loop on a ring filled once), with no compute (abvar/NOCOMP: the DMA
# ring, waits and barriers only), with no LDS fragment reads (abvar/NOREAD: register-made
# fragments, the DMA ring kept), beside the in-tree build, 256-thread and warp-specialized variants.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for r in 1 2; do
for v in intree NODMA NOREAD; do
  for ws in 0 1; do
    d=""; [ $v != intree ] && d="UBPL_LIB_DIR=$PWD/abvar/$v"
    echo "== $v ws=$ws r$r"
    env $d UBPL_PSA_WS=$ws timeout -k 10 120 python tools/psa_bench.py 32 50 || { echo "psa_bench $v failed"; exit 1; }
  done
done
done

#!/bin/bash
# GPU box: CSAN over ONE eager step of the B=32 headline case (where the split-load 1x1 kernel runs),
# data-pointer keys then storage keys, every race recorded.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 400 python tools/csan_probe.py mt_ubpl_b32 1 all > gpurun_out/csan_b32.log 2>&1; echo "csan ptr rc=$?"
grep -v "Warn\|amdgpu.ids" gpurun_out/csan_b32.log | tail -25
timeout -k 10 400 python tools/csan_probe.py mt_ubpl_b32 1 storage all > gpurun_out/csan_b32_storage.log 2>&1; echo "csan storage rc=$?"
grep -v "Warn\|amdgpu.ids" gpurun_out/csan_b32_storage.log | tail -25

#!/bin/bash
# GPU box (round 4): the one-halo-buffer, two-workgroups-per-CU variant (UBPL_PSA_HALO=3) vs
# conv_psa_kernel: bit-identity on the halo cases, then the 6xbf16 microbench.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
python - <<'PY' || exit 1
import os, sys, torch, numpy as np
sys.path.insert(0, "ubpl-poseestimation_amd")
from ubpl_amd import kernels as Kn
for (B, Cin, H, Cout) in [(32, 128, 64, 128), (8, 128, 128, 128), (16, 256, 64, 256), (32, 64, 128, 64), (32, 128, 32, 128)]:
    g = torch.Generator().manual_seed(5)
    x = torch.randn(B, Cin, H, H, generator=g).cuda(); w = (torch.randn(Cout, Cin, 3, 3, generator=g) / np.sqrt(Cin * 9)).cuda()
    xs = Kn.split_activation(x, 3, 1); ws = Kn.conv_weight_split(w, 0, 3)
    outs = []
    for m in ("0", "3"):
        os.environ["UBPL_PSA_HALO"] = m
        outs.append(Kn.conv2d_forward_psa(xs, ws, None)); torch.cuda.synchronize()
    print((B, Cin, H, Cout), "bit-identical" if torch.equal(outs[0], outs[1]) else "DIFFERENT", flush=True)
    assert torch.equal(outs[0], outs[1])
PY
for v in 0 3 0 3; do
  echo "== halo=$v"; UBPL_PSA_HALO=$v timeout -k 10 120 python tools/psa_bench.py 32 50 3 || exit 1
done

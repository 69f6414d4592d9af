"""GPU-box: the HBM-bound passes of the step at the headline shapes (B=32,
64x64 planes, 128 and 256 channels), timed standalone with HIP events over
back-to-back launches, against their ALGORITHMIC bytes (what must cross HBM
at least once) and the 8 TB/s HBM peak (MI355X_MICROARCH.md).

    python tools/hbm_passes.py [reps]

Prints one line per pass and a JSON record (profiles/r02_hbm_passes.json).
"""
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "ubpl-poseestimation_amd"))

from ubpl_amd import kernels as Kn  # noqa: E402

PEAK = 8.0e12


def timed(fn, reps):
    fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    e1.synchronize()
    return e0.elapsed_time(e1) / reps * 1e-3


def main():
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 30
    dev = torch.device("cuda", 0)
    g = torch.Generator(device=dev).manual_seed(0)
    B, H = 32, 64
    rows = []

    def rec(name, t, nbytes, note):
        bw = nbytes / t
        rows.append({"pass": name, "us": round(t * 1e6, 2), "algorithmic_MB": round(nbytes / 1e6, 2),
                     "TB_s": round(bw / 1e12, 3), "frac_of_8TBs": round(bw / PEAK, 3), "bytes": note})
        print("%-34s %8.1f us  %8.1f MB  %5.2f TB/s  %.2f of 8 TB/s   (%s)" % (
            name, t * 1e6, nbytes / 1e6, bw / 1e12, bw / PEAK, note), flush=True)

    for C in (128, 256):
        n = B * C * H * H
        x = torch.randn(B, C, H, H, device=dev, generator=g)
        dz = torch.randn(B, C, H, H, device=dev, generator=g)
        gamma = torch.rand(C, device=dev, generator=g) + 0.5
        beta = torch.randn(C, device=dev, generator=g) * 0.1
        rm, rv = torch.zeros(C, device=dev), torch.ones(C, device=dev)
        mu, istd, sc, sh = (torch.empty(C, device=dev) for _ in range(4))
        part = Kn.bn_part(B, C, dev)
        rec("bn_forward_stats C=%d" % C,
            timed(lambda: Kn.bn_forward_stats(x, gamma, beta, 1e-5, 0.1, rm, rv, part, mu, istd, sc, sh), reps),
            4 * n, "read x")
        y = torch.empty_like(x)
        rec("bn_apply+relu C=%d" % C, timed(lambda: Kn.bn_apply(x, sc, sh, 1, out=y), reps), 8 * n,
            "read x, write y")
        coef = torch.empty(3 * C, device=dev)
        dg, db = torch.zeros(C, device=dev), torch.zeros(C, device=dev)
        dx = torch.empty_like(x)
        scratch = Kn.bn_part(B, C, dev)
        rec("bn_backward (stats + apply) C=%d" % C,
            timed(lambda: Kn.bn_backward(dz, x, gamma, mu, istd, sc, sh, 1, scratch, coef, dg, db, out=dx), reps),
            12 * n, "read dz, x; write dx (the statistics pass re-reads both: 20 B/elem issued)")
        npad = B * C * (H + 2) * (H + 2)
        xs = Kn.split_activation(x, 3, 1, sc, sh)
        rec("split_activation (BN+ReLU, 3 pieces) C=%d" % C,
            timed(lambda: Kn.split_activation(x, 3, 1, sc, sh, out=xs.buf), reps), 4 * n + 6 * npad,
            "read x f32, write 3 bf16 pieces with the 1-px border")
        if C == 256:
            p = torch.empty(B, C, H // 2, H // 2, device=dev)
            rec("maxpool2x2 fwd C=256", timed(lambda: Kn.maxpool2x2(x, out=p), reps), 4 * n + n,
                "read x, write y")
            low = torch.randn(B, C, H // 2, H // 2, device=dev, generator=g)
            up = torch.randn(B, C, H, H, device=dev, generator=g)
            rec("upsample2x_add fwd C=256", timed(lambda: Kn.upsample2x_add(up, low, out=up), reps),
                8 * n + n, "read up, low; write out (in place)")
            dl = torch.empty_like(low)
            rec("upsample2x_add bwd C=256", timed(lambda: Kn.upsample2x_add_backward(dz, dl, False), reps),
                4 * n + n, "read dout, write dlow")
    # fused AdamW + EMA teacher update over one HG2 student's flat buffers (optim.hip)
    from ubpl_amd.hourglass import StackedHourglass
    from ubpl_amd.optim import FlatAdamW
    m, e = StackedHourglass(16, 2, "AvgPool").to(dev), StackedHourglass(16, 2, "AvgPool").to(dev)
    o = FlatAdamW(m, lr=2.5e-4, weight_decay=0.0)
    m.flat_grads.normal_(generator=g)
    n, nl = m.flat_params.numel(), m.n_live
    rec("adamw + ema (fused, one HG2 model)", timed(lambda: o.step_and_ema(e, 0.999), reps),
        7 * nl * 4 + 2 * n * 4 + (n - nl) * 4, "AdamW p, g, m, v r/w on the live prefix; EMA read student, r/w teacher")
    with open(os.path.join(ROOT, "gpurun_out", "hbm_passes.json"), "w") as fh:
        json.dump({"B": B, "H": H, "peak_TB_s": 8.0, "passes": rows}, fh, indent=1)


if __name__ == "__main__":
    os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
    main()

"""Benchmark: MT_UBPL training step (2-stack hourglass, 256x256, K=16,
B=32 per GPU: 16 unlabeled + 16 labeled rows) on the HIP path.

    python bench.py [--gpus N] [--steps K] [--warmup W]
    torchrun --nproc-per-node N bench.py --gpus N ...   (one rank per GPU, RCCL)

One step = what projects/MT_UBPL.py:173-339 does for one batch: heatmap
targets rendered on the device from keypoints, 2 students x 2 views
forward+backward, 2 teachers x 2 views forward (train-mode BN), the MSE /
consistency / UBPL pseudo-label / FDL losses, two AdamW steps, two EMA
updates — and under torch.distributed the global-count all-reduce and the
student-gradient all-reduce.  Inputs (images, keypoints) are synthetic and
already resident in HBM when timing starts.

Rank 0 prints ONE JSON line (see the driver contract in the task notes):
value = images/s over all ranks, plus `roofline` for the dominant kernel
(the 3x3 implicit-GEMM conv forward on the f32 matrix cores, timed per
launch with HIP events on its stream inside the timed region) and
`cpu_baseline` (the oracle's CPU restatement of the same step on a bounded
sample, host threads stated).
"""
import argparse
import json
import os
import sys
import time
import types

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "ubpl-poseestimation_amd"))
sys.path.insert(0, ROOT)

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

METRIC = "images/sec training step (MT_UBPL, 2-stack HG, 256×256) at 1/2/4/8 GPUs; PCK@0.2"
MEANS = [0.4920829, 0.4920829, 0.4920829]
F32_MFMA_PEAK_TFLOPS = 157.3          # MI355X_MICROARCH.md: v_mfma_f32_32x32x2_f32, dense
BF16_PEAK_TFLOPS = 2500.0             # dense bf16 / fp16 MFMA (the fp16 32x32x16 form takes the bf16 cycles)
SPLIT6_PEAK_TFLOPS = BF16_PEAK_TFLOPS / 6   # 6xbf16: 6 piece products per f32 product
SPLIT3_PEAK_TFLOPS = BF16_PEAK_TFLOPS / 3   # 2xfp16: 3 piece products per f32 product


def piece_peak(npieces):
    """f32-equivalent peak of a split conv with npieces per operand (the piece
    products with pa + pb < npieces: 6 / 3 / 1 MFMAs per f32 product)."""
    return {3: SPLIT6_PEAK_TFLOPS, 2: SPLIT3_PEAK_TFLOPS, 1: BF16_PEAK_TFLOPS}.get(npieces, F32_MFMA_PEAK_TFLOPS)


_KS_ONLY = [None]     # (forward_flops(..., ks=3): the 3x3 convs' share alone)


def _conv(cin, cout, ks, hw):
    if _KS_ONLY[0] is not None and ks != _KS_ONLY[0]:
        return 0
    return 2 * cin * cout * ks * ks * hw * hw


def _residual(cin, cout, hw):
    half = cout // 2
    f = _conv(cin, half, 1, hw) + _conv(half, half, 3, hw) + _conv(half, cout, 1, hw)
    return f + (_conv(cin, cout, 1, hw) if cin != cout else 0)


def _hourglass(n, hw):
    f = _residual(256, 256, hw) + 2 * _residual(256, 256, hw // 2)
    return f + (_hourglass(n - 1, hw // 2) if n > 1 else _residual(256, 256, hw // 2))


def forward_flops(S, K, res, ks=None):
    """Conv FLOP of one StackedHourglass forward per sample (models/pose/hourglass.py:12-99,
    models/base/layers.py:53-111): 16.67 GF at HG2 256^2 K=16 — SURVEY.md §8d's 266.7 GF per
    training sample = 16 forward-equivalents (2 students x 2 views x fwd + 2 bwd, 2 teachers x
    2 views x fwd).  ks: only the convs of that kernel size."""
    _KS_ONLY[0] = ks
    try:
        return _forward_flops(S, K, res)
    finally:
        _KS_ONLY[0] = None


def _forward_flops(S, K, res):
    r2, r4 = res // 2, res // 4
    f = _conv(3, 64, 7, r2) + _residual(64, 128, r2) + _residual(128, 128, r4) + _residual(128, 256, r4)
    f += S * (_hourglass(4, r4) + _residual(256, 256, r4) + _conv(256, 256, 1, r4) + _conv(256, K, 1, r4))
    return f + (S - 1) * (_conv(256, 256, 1, r4) + _conv(K, 256, 1, r4))


def step_record(cfg, B, ms_per_step, precision):
    """Step-level fraction of the matrix peak: the step's conv FLOP
    (f32-equivalent; forward passes: 2 students x views + 2 teachers x views, backward =
    2x forward) against the time the MFMA pipe would need at the precision's peaks
    (2xfp16: the forwards and the 3x3 gradients at the 3-product peak, the 1x1 gradients
    at the 6-product one, where they run; the stem and heads counted at the split peaks)."""
    F = forward_flops(cfg["S"], cfg["K"], cfg["res"]) * B
    F3 = forward_flops(cfg["S"], cfg["K"], cfg["res"], ks=3) * B
    views = 1 if cfg["project"] == "DualPose_UBPL" else 2
    fwd, bwd = 2 * views * F + 2 * views * F, 2 * views * 2 * F       # students' + teachers' forwards; gradients
    bwd3 = 2 * views * 2 * F3
    pieces = {"f32": 0, "bf16": 1, "2xfp16": 2, "6xbf16": 3}[precision]
    pf, pb = piece_peak(pieces), piece_peak(3 if pieces == 2 else pieces)
    ideal_s = fwd / (pf * 1e12) + bwd3 / (pf * 1e12) + (bwd - bwd3) / (pb * 1e12)
    t = ms_per_step * 1e-3
    return {"flop_per_step": fwd + bwd, "tflops": round((fwd + bwd) / t / 1e12, 2),
            "step_frac": round(ideal_s / t, 4), "peak_tflops_fwd": round(pf, 1), "peak_tflops_bwd": round(pb, 1),
            "note": "conv FLOP of the step (f32-equivalent) / step time, against the precision's MFMA peaks"}


def make_args(B):
    return types.SimpleNamespace(
        nStack=2, pseudoScoreThr=0.95, ensemblePseudoWeight=10.0, consWeight=10.0, poseWeight=10.0,
        FDLWeight=1.0, FDL_label="labeled", FDL_type="covariance", epo=1, ema_decay=0.999, pseudoWeight=1.0,
        outRes=64, lr=2.5e-4, wd=0.0, feature_mode="AvgPool")


# BASELINE.json configs this bench can run (the driver runs the default, the headline)
CONFIGS = {
    "mt_ubpl": dict(project="MT_UBPL", S=2, K=16, B=32, res=256, desc="configs[1-2]: MT_UBPL, HG2, 256x256"),
    "mt_ubpl_hg2_256_bf16": dict(project="MT_UBPL", S=2, K=16, B=32, res=256, precision="bf16",
                                 desc="configs[1-2]: MT_UBPL, HG2, 256x256, bf16 MFMA path (conv operands bf16, "
                                      "f32 accumulation; a secondary line beside the fp32-equivalent headline)"),
    "dualpose_hg4": dict(project="DualPose_UBPL", S=4, K=17, B=16, res=256,
                         desc="configs[3]: DualPose_UBPL, dual HG4, K=17, 256x256, B=16/GPU"),
    "mt_ubpl_hg8_384": dict(project="MT_UBPL", S=8, K=16, B=16, res=384,
                            desc="configs[4]: MT_UBPL, HG8, 384x384 input / 96x96 heatmaps, B=16/GPU "
                                 "(fp32-grade split convs, the headline's precision; not the bf16 path)"),
    "mt_ubpl_hg8_384_bf16": dict(project="MT_UBPL", S=8, K=16, B=16, res=384, precision="bf16",
                                 desc="configs[4]: MT_UBPL, HG8, 384x384 input / 96x96 heatmaps, B=16/GPU, "
                                      "bf16 MFMA path (conv operands bf16, f32 accumulation)"),
}


def make_batches(n, B, K, dev, seed, res=256, dualpose=False):
    """Synthetic batches resident on the device: images
    U[0,1) minus the Mouse means, integer keypoints in [8, 248), unlabeled
    rows first and zeroed (TwoStreamBatchSampler order)."""
    g = torch.Generator().manual_seed(seed)
    nlab = B // 2
    out = []
    means = torch.tensor(MEANS)[None, :, None, None]
    for _ in range(n):
        imgs, kps = [], []
        isl = torch.tensor([0] * (B - nlab) + [1] * nlab, dtype=torch.bool)
        for _a in range(2):
            imgs.append((torch.rand(B, 3, res, res, generator=g) - means).to(dev))
            k = torch.zeros(B, K, 3)
            k[:, :, :2] = torch.randint(8, res - 8, (B, K, 2), generator=g).float()
            k[:, :, 2] = 1.0
            k[~isl] = 0.0
            kps.append(k.to(dev))
        if dualpose:       # (stu_img, stu_heatmap, ema_img, meta): DualPose_UBPL.py:171
            out.append((imgs[0], None, imgs[1], {"kps": kps[0], "islabeled": isl.to(dev)}))
        else:
            out.append((imgs, None, {"kps": kps, "islabeled": [isl.to(dev)]}))
    return out


ROOF_SHAPE = (128, 128, 3, 64, 64)   # Cin, Cout, KS, H, W of the roofline kernel's launches (headline)
# per config: (Cin, Cout, KS, H, W) of the dominant 3x3 conv launches (HG8 at 384^2 runs its top
# hourglass level on 96x96 planes)
ROOF = {"mt_ubpl": (128, 128, 3, 64, 64), "mt_ubpl_hg2_256_bf16": (128, 128, 3, 64, 64),
        "dualpose_hg4": (128, 128, 3, 64, 64), "mt_ubpl_hg8_384": (128, 128, 3, 96, 96),
        "mt_ubpl_hg8_384_bf16": (128, 128, 3, 96, 96)}


def roof_kernel(shape, npieces):
    """The instantiation ubpl_conv2d_forward_psa dispatches for these launches by default
    (conv_split.hip): the input-halo kernel, one halo buffer and two workgroups per CU on the
    split paths (<W, NP, 128, 1, 1, 256>; 96-wide planes: 192-pixel tiles), two teams on the
    bf16 path at W <= 64; UBPL_PSA_HALO=0 / 1 (the only values the library accepts) select the
    per-tap conv_psa_kernel / the double-buffered halo kernel."""
    W = shape[4]
    halo = os.environ.get("UBPL_PSA_HALO", "")
    if halo == "0":
        return "conv_psa_kernel<128, 3, %d, 256, 2> (per-tap B staging; UBPL_PSA_HALO=0)" % npieces
    if halo == "1":
        return "conv_psah_kernel<%d, %d, 128, ...> (double-buffered halo; UBPL_PSA_HALO=1)" % (W, npieces)
    if npieces == 1:
        return ("conv_psah_kernel<%d, 1, 128, 2, 2, 256>" % W) if W <= 64 else "conv_psa_kernel<128, 3, 1, 256, 2, 2>"
    return "conv_psah_kernel<%d, %d, 128, 1, 1, %d>" % (W, npieces, 192 if W == 96 else 256)


PIECE_NAME = {3: "6xbf16 split-f32 MFMA (3 bf16 pieces, 6 products)",
              2: "2xfp16 split-f32 MFMA (2 fp16 pieces of the scaled operands, 3 products)",
              1: "bf16 operands, f32 accumulation", 0: "exact f32 MFMA"}


class PsaLaunches:
    """Records, during one eager step, the C-ABI argument tuple of every
    ubpl_conv2d_forward_psa call whose shape is the roofline kernel's — the
    3x3 128->128 convs on the 64x64 planes (Residual conv2 forward and its
    data gradient), which run as ONE instantiation, conv_psah_kernel<64, 3, 128,
    1, 1> on the 6xbf16 path (rocprofv3 names it so; conv_psa_kernel<128, 3, 3,
    256, 2> with UBPL_PSA_HALO=0), with no split-K slab — and keeps every
    tensor those pointers reference alive, so the launches can be replayed."""

    def __init__(self, Kn, lib, shape=ROOF_SHAPE, npieces=None):
        self.Kn, self.lib, self.shape, self.npieces = Kn, lib, tuple(shape), npieces
        self.calls, self.keep = [], []

    def __enter__(self):
        orig_call, orig_psa = self.lib.call, self.Kn.conv2d_forward_psa
        self._orig = (orig_call, orig_psa)
        rec = self

        def call(name, *args):
            if name == "ubpl_conv2d_forward_psa" and rec._want:
                rec.calls.append(args)
            return orig_call(name, *args)

        def psa(xs, ws, bias, res=None, out=None, stat_part=None, bwd=None):
            Cout, T, _ = ws.shape
            rec._want = (xs.C, Cout, int(round(T ** 0.5)), xs.H, xs.W) == rec.shape and \
                rec.npieces in (None, ws.npieces)
            y = orig_psa(xs, ws, bias, res, out, stat_part, bwd)
            if rec._want:
                rec.keep.append((xs, ws, bias, res, y, stat_part, bwd))
            rec._want = False
            return y
        self._want = False
        self.lib.call = call
        self.Kn.call = call
        self.Kn.conv2d_forward_psa = psa
        return self

    def __exit__(self, *a):
        self.lib.call = self._orig[0]
        self.Kn.call = self._orig[0]
        self.Kn.conv2d_forward_psa = self._orig[1]

    def time(self, reps=10):
        """Replays the recorded launches back to back (reps times, queue filled
        behind a spin kernel so no host gap enters the window) between two HIP
        events on the stream they were launched on; returns the average
        duration of one launch in ms."""
        fn = self.lib.op("ubpl_conv2d_forward_psa")              # the torch op over the C-ABI entry
        calls = [c for c in self.calls if c[14] is None]        # slab pointer: none (no split-K)
        if not calls:
            return None, 0
        torch.cuda.synchronize()
        for c in calls:                                         # warm
            fn(*c)
        torch.cuda.synchronize()
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        torch.cuda._sleep(20_000_000)
        s.record()
        for _ in range(reps):
            for c in calls:
                fn(*c)
        e.record()
        torch.cuda.synchronize()
        return s.elapsed_time(e) / (reps * len(calls)), len(calls)


def roofline(Kn, lib, T, models, emas, optims, args, batch, ms_per_step, config="mt_ubpl", train=None):
    """The dominant kernel: the 3x3 conv at the config's largest 3x3 planes
    (headline: the 3x3 128->128 conv at the 64x64 planes on the input-halo kernel;
    the largest single entry of the rocprofv3 kernel summary, profiles/r0*_summary),
    its launches at the precision's piece count (forward + data gradient: on 2xfp16
    both run 2 fp16 pieces, UBPL_FP16_BWD3 default).
    achieved = algorithmic FLOP per launch (2*B*Cout*Cin*9*H*W; f32-equivalent on the
    split paths) / its average standalone launch duration (HIP events around
    replayed launches, see PsaLaunches.time), vs the pieces' peak (6xbf16: 2.5 PF
    bf16 dense / 6 piece products; 2xfp16: / 3; bf16: 2.5 PF)."""
    shape = ROOF[config]
    npieces = Kn.conv_precision_pieces()
    peak = piece_peak(npieces)
    desc = "%s (3x3 conv, %d->%d ch, %dx%d planes, %s; %s; f32-equivalent FLOP/s, peak = bf16 dense / products)" % (
        roof_kernel(shape, npieces), shape[0], shape[1], shape[3], shape[4],
        "fwd + dgrad", PIECE_NAME[npieces])
    os.environ["UBPL_MODEL_STREAMS"] = "0"
    try:
        with PsaLaunches(Kn, lib, shape, npieces) as rec, T._StepGraph.eager():
            (train or T.train_mt_ubpl)([batch], models, emas, optims, args, verbose=False)
        torch.cuda.synchronize()
        avg_ms, n = rec.time()
    finally:
        del os.environ["UBPL_MODEL_STREAMS"]
    if avg_ms is None:
        return None
    Cin, Cout, KS, H, W = shape
    B = args.batch
    flops = 2 * B * Cout * Cin * KS * KS * H * W
    achieved = flops / (avg_ms * 1e-3) / 1e12
    per_step_ms = n * avg_ms
    # standalone replays summed vs the measured step: a check, reported (never an abort after the
    # timed region — box noise, or in-situ overlap making the step shorter than serial launches)
    consistent = per_step_ms <= ms_per_step
    if not consistent:
        print("bench: roofline kernel replays sum to %.2f ms > %.2f ms/step" % (per_step_ms, ms_per_step),
              file=sys.stderr)
    # HBM traffic by PMC (profiles/pmc_roofline_psah*.json) for the default dispatch of the headline
    halo = os.environ.get("UBPL_PSA_HALO", "")
    pmc = pmc_traffic("psah%s" % ("" if npieces == 3 else npieces)) if config == "mt_ubpl" and halo == "" else None
    return {"bound": "mfma", "achieved": round(achieved, 2), "peak": round(peak, 2),
            "unit": "TFLOP/s", "frac": round(achieved / peak, 4),
            "traffic": (pmc or {}).get("hbm_bytes_per_launch"), "traffic_detail": pmc,
            "kernel": desc, "pieces": npieces,
            "flops_per_launch": flops, "launches_per_step": n, "avg_launch_us": round(avg_ms * 1e3, 2),
            "kernel_ms_per_step": round(per_step_ms, 3), "fits_in_step": consistent,
            "timing": "HIP events around back-to-back replays of the step's launches of this kernel "
                      "(standalone; inputs resident), after the timed region"}


def pmc_traffic(kind):
    """HBM bytes per launch of the roofline kernel, measured by rocprofv3 --pmc
    passes over this bench command (tools/gpu_pmc.sh bench ->
    tools/pmc_roofline.py -> profiles/pmc_roofline[_psa].json); None if absent."""
    p = os.path.join(ROOT, "profiles", "pmc_roofline_%s.json" % kind)
    if not os.path.exists(p):
        return None
    with open(p) as fh:
        d = json.load(fh)
    return {"hbm_bytes_per_launch": int(d["hbm_bytes_per_launch"]),
            "fetch_bytes_per_launch": int(d["fetch_bytes_per_launch"]),
            "write_bytes_per_launch": int(d["write_bytes_per_launch"]), "source": d.get("source")}


def pck_record():
    """PCK@0.2 — the metric's second half — of the real-data harness: the
    reference's MT_UBPL Mouse experiment (tools/mouse_pck.py: HG2, trainBS 4
    with 2 labeled, validate() on the 500-image validation split) run on the
    HIP path for 20 epochs (profiles/r0N_mouse_pck_hg2_e20.json), next to the
    REFERENCE's own train()/validate() on the same epochs, seeds, sampler and
    augmentation draws (tools/ref_pck.py -> tests/golden/ref_pck.json, CPU, in
    the build container; tests/test_gpu_mouse.py re-runs the HIP side and checks
    every validated epoch within 0.1).  It trains for minutes, so the bench
    reports the committed records instead of re-training; the 100-epoch HIP run
    is reported beside it (the reference at 100 epochs on CPU would take ~10 h)."""
    import glob
    found = sorted(glob.glob(os.path.join(ROOT, "profiles", "r0*_mouse_pck_hg2_e20.json")))
    # (the newest round's 20-epoch record; without one, round 2's 100-epoch run, no reference beside it)
    p = found[-1] if found else os.path.join(ROOT, "profiles", "r02_mouse_pck_hg2_e100.json")
    r = os.path.join(ROOT, "tests", "golden", "ref_pck.json")
    if not os.path.exists(p):
        return None
    with open(p) as fh:
        d = json.load(fh)
    ref = None
    if os.path.exists(r):
        with open(r) as fh:
            ref = json.load(fh)
    last = [e for e in d["epochs"] if "pck" in e][-1]
    rlast = [e for e in ref["epochs"] if "pck" in e][-1] if ref else None
    out = {"value": last["pck"][-1], "teachers": last["pck"][:-1], "epochs": last["epoch"], "model": d["config"]["model"],
           "split": d["config"]["split"], "thr": d["config"]["pck_thr"],
           "source": "%s (tools/mouse_pck.py)" % os.path.relpath(p, ROOT),
           "reference_value": rlast["pck"][-1] if rlast and rlast["epoch"] == last["epoch"] else None,
           "reference_teachers": rlast["pck"][:-1] if rlast and rlast["epoch"] == last["epoch"] else None,
           "reference_source": "tests/golden/ref_pck.json (tools/ref_pck.py: the reference's train()/validate(), "
                               "CPU, same seeds / sampler / augmentation draws, the reference's crop -> "
                               "skimage rotate -> resize pixel chain restated in oracle/augment_chain.py)",
           "note": "mean-of-teachers prediction (projects/MT_UBPL.py:387)"}
    p100 = os.path.join(ROOT, "profiles", "r02_mouse_pck_hg2_e100.json")
    if os.path.exists(p100):
        with open(p100) as fh:
            d100 = json.load(fh)
        out["hip_100_epochs"] = {"value": d100["final_pck"][-1], "teachers": d100["final_pck"][:-1],
                                 "source": "profiles/r02_mouse_pck_hg2_e100.json (round-2 augmentation geometry)"}
    return out


def cpu_baseline(steps=1, B=32):
    """The oracle's CPU restatement of the same MT_UBPL step (oracle/step.py,
    pinned to the reference's own train() outputs by tests/test_oracle_golden.py),
    timed on this host on a bounded sample: ONE step of the headline workload
    (B=32, 2 stacks, 256x256, K=16) after one untimed B=4 step.  Threads: the
    CPU share of a GPU box (16; os.cpu_count() reports the whole machine).
    Calibrated against the reference's train() itself in the build container:
    profiles/r02_cpu_calibration.json."""
    from oracle import hourglass as OH
    from oracle import render as OR
    from oracle import step as OS
    threads = int(os.environ.get("UBPL_CPU_THREADS", min(8, os.cpu_count() or 1)))
    torch.set_num_threads(threads)
    torch.manual_seed(1388)
    models, emas, optims = [], [], []
    for _ in range(2):
        models.append(OH.oracle_factory(16, 2, "AvgPool"))
        e = OH.oracle_factory(16, 2, "AvgPool")
        e.requires_grad_(False)
        emas.append(e)
        optims.append(torch.optim.AdamW(models[-1].parameters(), lr=2.5e-4, weight_decay=0))
    args = make_args(B)

    def host_batches(n, b, seed):
        out = []
        for (imgs, _, meta) in make_batches(n, b, 16, "cpu", seed):
            hms, gates = [], []
            for k in meta["kps"]:
                h, kk = OR.render_batch(k.numpy(), (256, 256), 256, 64)
                hms.append([torch.from_numpy(h)])
                gates.append([torch.from_numpy(kk[:, :, 2].copy())])
            out.append((imgs, hms, {"kpsWeights": gates, "islabeled": meta["islabeled"]}))
        return out
    OS.train_mt_ubpl(host_batches(1, 4, 76), models, emas, optims, args)      # warm-up
    batches = host_batches(steps, B, 77)
    t = time.time()
    OS.train_mt_ubpl(batches, models, emas, optims, args)
    dt = time.time() - t
    cal = os.path.join(ROOT, "profiles", "r03_cpu_calibration_b32.json")
    ratio, cal_threads = None, None
    if os.path.exists(cal):
        with open(cal) as fh:
            c = json.load(fh)
        ratio, cal_threads = c["port_over_reference"], c.get("threads")
    # the port/reference ratio holds at the thread count it was measured with only
    pinned = ratio is not None and cal_threads == threads
    return {"value": round(steps * B / dt, 4), "unit": "images/sec", "cores": threads, "kind": "port",
            "reference_equivalent": round(steps * B / dt / ratio, 4) if pinned else None,
            "port_over_reference": ratio, "calibration_threads": cal_threads,
            "calibration": "pinned" if pinned else "unpinned (calibrated at %s threads, run at %d)"
                           % (cal_threads, threads),
            "sample": "oracle/step.py MT_UBPL step (same math as projects/MT_UBPL.py:157-352), 2-stack, "
                      "B=%d (half labeled), 256x256, K=16, %d timed step(s) = %.1f s, torch CPU fp32; "
                      "calibration vs the reference train(): profiles/r03_cpu_calibration_b32.json"
                      % (B, steps, dt)}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--batch", type=int, default=None)
    ap.add_argument("--config", default="mt_ubpl", choices=sorted(CONFIGS))
    ap.add_argument("--no-cpu-baseline", action="store_true")
    a = ap.parse_args()
    cfg = CONFIGS[a.config]
    headline = a.config == "mt_ubpl"
    if "precision" in cfg:
        os.environ["UBPL_CONV_PRECISION"] = cfg["precision"]

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        torch.cuda.set_device(local)
        dist.init_process_group("nccl", rank=rank, world_size=world, device_id=torch.device("cuda", local))
    dev = torch.device("cuda", local)
    torch.cuda.set_device(dev)

    from ubpl_amd import _lib, kernels as Kn
    from ubpl_amd.hourglass import StackedHourglass
    from ubpl_amd.optim import FlatAdamW
    from ubpl_amd import train as T
    from ubpl_amd import dist as D
    _lib.load()

    B, K, S, res = a.batch or cfg["B"], cfg["K"], cfg["S"], cfg["res"]
    dualpose = cfg["project"] == "DualPose_UBPL"
    train = T.train_dualpose_ubpl if dualpose else T.train_mt_ubpl
    torch.manual_seed(1388)
    models, emas, optims = [], [], []
    for _ in range(2):                               # projects/MT_UBPL.py:43-50
        m = StackedHourglass(K, S, "AvgPool")
        e = StackedHourglass(K, S, "AvgPool")
        for p in e.parameters():
            p.detach_()
        models.append(m)
        emas.append(e)
        optims.append(FlatAdamW(m, lr=2.5e-4, weight_decay=0.0))
    D.broadcast_params(models + emas)
    args = make_args(B)
    args.nStack, args.outRes = S, res // 4
    batches = make_batches(2, B, K, dev, 1388 + rank, res, dualpose)
    warm = [batches[i % 2] for i in range(a.warmup)]
    timed = [batches[i % 2] for i in range(a.steps)]

    # default step: one HIP stream per network, the whole step captured in a
    # HIP graph on the last warm-up step and replayed for the timed steps (the
    # captured launches are the eager step's, bit for bit, and the replayed B=32
    # step is checked against the reference's fixtures: tests/test_gpu_train.py);
    # under torch.distributed captured as three segments with the two RCCL
    # collectives between their replays (train._StepGraph); UBPL_STEP_GRAPH=0:
    # eager launches.
    T._StepGraph.WARM = max(1, a.warmup - 1)
    train(warm, models, emas, optims, args, verbose=False)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    torch.cuda._sleep(1)          # window marker for tools/prof_summary.py (a ~1-cycle spin_kernel)
    t0 = time.perf_counter()
    train(timed, models, emas, optims, args, verbose=False)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    torch.cuda._sleep(1)          # end marker: the kernels between the two markers are the timed steps'
    # roofline kernel: its launches from one more (eager, untimed) step, replayed
    # back to back between HIP events (standalone duration; see roofline())
    args.batch = B
    roof = roofline(Kn, _lib, T, models, emas, optims, args, timed[0], dt / a.steps * 1e3, a.config, train)
    if world > 1:
        t = torch.tensor([dt], device=dev, dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        dt = float(t.item())
    images = world * B * a.steps
    if rank == 0:
        cpu = None
        if not a.no_cpu_baseline and world == 1 and headline:
            cpu = cpu_baseline()
        line = {
            "metric": METRIC if headline else "images/sec training step (%s)" % cfg["desc"],
            "value": round(images / dt, 3), "unit": "images/sec", "n_gpus": world,
            "steps": a.steps, "warmup": a.warmup, "ms_per_step": round(dt / a.steps * 1e3, 3),
            "higher_is_better": True, "scaling": "weak", "vs_baseline": None,
            "dtype": "bf16" if Kn.conv_precision_name() == "bf16" else "fp32",
            "conv_precision": Kn.conv_precision_name(),
            "data": "synthetic (U[0,1) images - means, integer keypoints, half labeled; heatmaps rendered on device)",
            "config": {"workload": ("%s train step, 2 students + 2 EMA teachers, %s" % (
                                        cfg["project"], "student / teacher views" if dualpose else "2 views")),
                       "model": "StackedHourglass HG%d (K=%d, AvgPool features)" % (S, K), "global_batch": B * world,
                       "per_gpu_batch": B, "input": "%dx%dx3" % (res, res),
                       "heatmap": "%dx%dx%d" % (K, res // 4, res // 4), "parallelism": "dp%d" % world,
                       "baseline_config": cfg["desc"]},
            "roofline": roof, "step": step_record(cfg, B, dt / a.steps * 1e3, Kn.conv_precision_name()),
            "cpu_baseline": cpu, "pck": pck_record() if headline else None,
        }
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()

"""PCK@0.2 of the REFERENCE's own MT_UBPL train() / validate()
(projects/MT_UBPL.py:157-408) on the Mouse split, on the same batches the HIP
harness (tools/mouse_pck.py) trains on — so the two PCK trajectories can be
compared epoch by epoch (north_star "PCK@0.2 within ±0.1
of reference").

TEST INFRASTRUCTURE ONLY: runs in the build container (imports /root/reference
through tests/golden/gen_golden.py's stub recipe, CPU).  skimage is absent
here, so the reference's own loader (DS_mds) cannot run; the batches are
instead built by the CPU restatement of the device augmentation — the same
host draws (ubpl_amd.augment.draw_view: python random, torch CPU generator,
the loader's float32 arithmetic), the same sampler (TwoStreamBatchSampler,
numpy RNG), the same order (view-major per batch, as mouse_pck.py's loader)
and the same seeds (1388, projects/MT_UBPL.py:424-428) — with the bilinear
warp of augment.hip restated in numpy.  The heatmap targets come from the
reference's own ProcessUtils.kps_heatmap, the models from its
StackedHourglass (PoseModel minus .cuda()), the optimiser is torch AdamW.

    python tools/ref_pck.py [--epochs 20] [--threads 8] [--out tests/golden/ref_pck.json]
"""
import argparse
import contextlib
import io
import json
import os
import random
import sys
import time
import types

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "ubpl-poseestimation_amd"), os.path.join(ROOT, "tests", "golden"), ROOT]

import numpy as np  # noqa: E402
import torch  # noqa: E402


def warp_np(img, m, noise, mu, means, res):
    """augment.hip augment_warp_kernel restated in numpy (float32 source
    coordinates as the kernel computes them)."""
    H, W, _ = img.shape
    v = img.astype(np.float32) / np.float32(255.)
    a, b, on = noise
    if on > 0:
        v = np.clip(np.float32(a) * (v - np.float32(mu)) + np.float32(mu) + np.float32(b), 0, 1)
    m = np.asarray(m, np.float32)
    ys, xs = np.mgrid[0:res, 0:res].astype(np.float32)
    sx = m[0] * xs + m[1] * ys + m[2]
    sy = m[3] * xs + m[4] * ys + m[5]
    fx, fy = np.floor(sx), np.floor(sy)
    x0, y0 = fx.astype(int), fy.astype(int)
    wx, wy = (sx - fx)[..., None], (sy - fy)[..., None]

    def tap(x, y):
        ok = (x >= 0) & (x < W) & (y >= 0) & (y < H)
        r = np.zeros((res, res, 3), np.float32)
        r[ok] = v[y[ok], x[ok]]
        return r
    t00, t01, t10, t11 = tap(x0, y0), tap(x0 + 1, y0), tap(x0, y0 + 1), tap(x0 + 1, y0 + 1)
    top = t00 + wx * (t01 - t00)
    bot = t10 + wx * (t11 - t10)
    val = top + wy * (bot - top)
    return torch.from_numpy(np.ascontiguousarray(np.transpose(val, (2, 0, 1)) - np.array(means, np.float32)[:, None,
                                                                                                                None]))


def chain_np(img, geo, noise, mu, means, res):
    """The reference's own pixel path for one view (utils/augment.py:86-137
    after fliplr and noisy_mean: integer crop, skimage rotate, skimage resize;
    oracle/augment_chain.py restates scikit-image 0.20), colorNorm'ed — what
    DS_mds would hand train() (datasets/dataset_mds.py:88-113)."""
    from oracle import augment_chain as AC
    (flip, ulx, uly, Hp, Wp, Hc, Wc), (cs, sn) = geo
    v = img.astype(np.float32) / np.float32(255.)
    if flip:
        v = v[:, ::-1]
    a, b, on = noise
    if on > 0:
        v = np.clip(np.float32(a) * (v - np.float32(mu)) + np.float32(mu) + np.float32(b), 0, 1)
    pad = (Hp - Hc) // 2
    angle = float(np.rad2deg(np.arctan2(sn, cs))) if pad else 0.0
    val = AC.affine_view(v.astype(np.float64), (ulx, uly), (ulx + Wp, uly + Hp), pad, angle, (res, res))
    return torch.from_numpy(np.ascontiguousarray(np.transpose(val, (2, 0, 1)).astype(np.float32)
                                                 - np.array(means, np.float32)[:, None, None]))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--pixels", choices=("chain", "warp"), default="chain",
                    help="chain: the reference's crop -> rotate -> resize (default); warp: one bilinear sample")
    ap.add_argument("--epochs", type=int, default=20)
    ap.add_argument("--valid-every", type=int, default=5)
    ap.add_argument("--threads", type=int, default=8)
    ap.add_argument("--seed", type=int, default=1388)
    ap.add_argument("--out", default=os.path.join(ROOT, "tests", "golden", "ref_pck.json"))
    a = ap.parse_args()
    torch.set_num_threads(a.threads)

    import gen_golden as GG
    R = GG.import_reference()
    proj = GG._import_project("MT_UBPL")
    from ubpl_amd import mouse
    from ubpl_amd import parameters as PR
    from ubpl_amd.augment import draw_view

    random.seed(a.seed)
    np.random.seed(a.seed)
    torch.manual_seed(a.seed)                                          # projects/MT_UBPL.py:424-428
    data = mouse.MouseData.from_pack()
    semi, valid, lab, unlab, lidx, uidx, means, stds = data.getSemiData(100, 500, 0.3)
    args = types.SimpleNamespace(
        device="cpu", debug=False, br_augNum=1, br_gtNum=1, nStack=2, pseudoScoreThr=0.95,
        ensemblePseudoWeight=10.0, poseWeight=10.0, consWeight_max=10.0, consWeight_min=0.0, consWeight_rampup=5,
        FDLWeight_max=1.0, FDLWeight_min=1.0, FDLWeight_rampup=100, pseudoWeight_max=1.0, pseudoWeight_min=1.0,
        pseudoWeight_rampup=100, FDL_label="labeled", FDL_type="covariance", useEnsemblePseudo=True,
        ema_decay=0.999, lr=2.5e-4, outRes=data.outRes, pck_ref=data.pck_ref, pck_thr=data.pck_thr,
        feature_mode="AvgPool", epo=0, best_epoch=[0, 0, 0])
    models, emas, optims = [], [], []
    for _ in range(2):                                                 # :43-50 student, teacher per branch
        models.append(R["SH"](data.kpsCount, 2, "AvgPool"))
        e = R["SH"](data.kpsCount, 2, "AvgPool")
        for p in e.parameters():                                       # models/pose/pose_model.py:10-12 nograd
            p.detach_()
        emas.append(e)
        optims.append(torch.optim.AdamW(models[-1].parameters(), lr=args.lr, weight_decay=0.0))
    imgs = data.images("train")
    img_mean = imgs.reshape(imgs.shape[0], -1).astype(np.float64).mean(1) / 255.
    kps_all = np.array([it["kps"] for it in semi], np.float32)
    isl_all = np.array([it["islabeled"] for it in semi], bool)
    sampler = R["MD"].TwoStreamBatchSampler(uidx, lidx, 4, 2)
    H, W = imgs.shape[1:3]
    vb = mouse.valid_batches(data, 128, "cpu")
    vloader = [(x, torch.zeros(x.shape[0], data.kpsCount, data.outRes, data.outRes), meta) for x, _, meta in vb]

    def loader():
        for idx in sampler:
            idx = list(idx)
            views, hms, gates = [], [], []
            for _ in range(2):                                         # view-major, as mouse_pck.py
                vx, vh, vg = [], [], []
                for i in idx:
                    m, noise, kk, geo = draw_view(kps_all[i], W, H, data.inpRes, 0.25, 30.0, with_geometry=True)
                    if a.pixels == "chain":
                        vx.append(chain_np(imgs[i], geo, noise, img_mean[i], means, data.inpRes))
                    else:
                        vx.append(warp_np(imgs[i], m, noise, img_mean[i], means, data.inpRes))
                    hm, kv = R["P"].kps_heatmap(torch.from_numpy(kk), (3, data.inpRes, data.inpRes), data.inpRes,
                                                data.outRes)
                    vh.append(hm)
                    vg.append(kv[:, 2].clone())
                views.append(torch.stack(vx))
                hms.append([torch.stack(vh)])
                gates.append([torch.stack(vg)])
            B = len(idx)
            meta = {"kpsWeights": gates, "warpmat": [torch.zeros(B, 2, 3) for _ in range(2)],
                    "isflip": [torch.zeros(B, dtype=torch.bool) for _ in range(2)],
                    "islabeled": [torch.tensor(isl_all[idx])]}
            yield views, hms, meta

    log = {"what": "reference projects/MT_UBPL.py train()/validate() on CPU, Mouse_100_500_0.3, HG2, trainBS 4 "
                   "(2 labeled), batches from the CPU restatement of the device augmentation (tools/ref_pck.py), "
                   "pixels: " + ("the reference's crop -> skimage rotate -> skimage resize chain (oracle/augment_chain.py)"
                                 if a.pixels == "chain" else "one bilinear warp"),
           "threads": a.threads, "seed": a.seed, "epochs": []}
    t0 = time.time()
    for epo in range(a.epochs):
        args.epo = epo
        args.consWeight = PR.consWeight_increase(epo, args)
        args.FDLWeight = PR.FDLWeight_decrease(epo, args)
        args.pseudoWeight = PR.pseudoWeight_increase(epo, args)
        te = time.time()
        with contextlib.redirect_stdout(io.StringIO()):
            pec, mtc, epc, fdc = proj.train(loader(), models, emas, optims, args)
        rec = {"epoch": epo + 1, "train_s": round(time.time() - te, 1), "pec": pec, "mtc": mtc, "epc": epc,
               "fdc": fdc}
        if (epo + 1) % a.valid_every == 0 or epo + 1 == a.epochs:
            with contextlib.redirect_stdout(io.StringIO()):
                _, accs, errs = proj.validate(vloader, emas, args)
            for e in emas:
                e.train()
            rec["pck"] = [round(float(v[-1]), 4) for v in accs]
        log["epochs"].append(rec)
        print(json.dumps(rec), "%.0f s" % (time.time() - t0), flush=True)
        with open(a.out, "w") as f:
            json.dump(log, f, indent=1)


if __name__ == "__main__":
    main()

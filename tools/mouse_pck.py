"""Real-data PCK@0.2 harness: the reference's MT_UBPL experiment on the Mouse
split (projects/MT_UBPL.py:27-154 main(): 2 students + 2 EMA teachers,
TwoStreamBatchSampler over 70 unlabeled / 30 labeled images, trainBS 4 with
2 labeled, AdamW lr 2.5e-4, two augmented views per sample, ramped loss
weights, validate() on the 500 validation images every few epochs), entirely
on the HIP path: device augmentation (augment.hip), device heatmap targets,
the fused train step, HIP decode + PCK.

    python tools/mouse_pck.py [--epochs 100] [--model HG2] [--out profiles/r02_mouse_pck.json]

Needs data/mouse_100_500_0.3.npz (tools/pack_mouse.py).
"""
import argparse
import json
import os
import random
import sys
import time
import types

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "ubpl-poseestimation_amd"))

import numpy as np  # noqa: E402
import torch  # noqa: E402


def parser():
    ap = argparse.ArgumentParser()
    ap.add_argument("--epochs", type=int, default=100)
    ap.add_argument("--model", default="HG2")
    ap.add_argument("--trainBS", type=int, default=4)
    ap.add_argument("--trainBS_labeled", type=int, default=2)
    ap.add_argument("--inferBS", type=int, default=128)
    ap.add_argument("--valid-every", type=int, default=5)
    ap.add_argument("--no-aug", action="store_true")
    ap.add_argument("--seed", type=int, default=1388)
    ap.add_argument("--out", default=os.path.join(ROOT, "gpurun_out", "mouse_pck.json"))
    return ap


def main():
    log = run(parser().parse_args())
    print(json.dumps({"best_pck": log["best_pck"], "best_epoch": log["best_epoch"], "final_pck": log["final_pck"],
                      "wall_s": log["wall_s"]}))


def run(a, write=True):
    """The experiment of main() with options `a` (parser() defaults); returns the log."""

    from ubpl_amd import _lib, mouse
    from ubpl_amd import parameters as PR
    from ubpl_amd import train as T
    from ubpl_amd.augment import DeviceAugment
    from ubpl_amd.hourglass import pose_model
    from ubpl_amd.optim import FlatAdamW
    from ubpl_amd.sampler import TwoStreamBatchSampler
    _lib.load()
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    random.seed(a.seed)
    np.random.seed(a.seed)
    torch.manual_seed(a.seed)                                          # projects/MT_UBPL.py:424-428

    data = mouse.MouseData.from_pack()
    semi, valid, lab, unlab, lidx, uidx, means, stds = data.getSemiData(100, 500, 0.3)
    args = types.SimpleNamespace(
        nStack=int(a.model[2:]), pseudoScoreThr=0.95, ensemblePseudoWeight=10.0, poseWeight=10.0,
        consWeight_max=10.0, consWeight_min=0.0, consWeight_rampup=5, FDLWeight_max=1.0, FDLWeight_min=1.0,
        FDLWeight_rampup=100, pseudoWeight_max=1.0, pseudoWeight_min=1.0, pseudoWeight_rampup=100,
        FDL_label="labeled", FDL_type="covariance", useEnsemblePseudo=True, ema_decay=0.999, lr=2.5e-4,
        outRes=data.outRes, pck_ref=data.pck_ref, pck_thr=data.pck_thr, feature_mode="AvgPool", epo=0)
    models, emas, optims = [], [], []
    for _ in range(2):                                                 # :43-50 student, teacher per branch
        models.append(pose_model(a.model, data.kpsCount, "AvgPool"))
        emas.append(pose_model(a.model, data.kpsCount, "AvgPool", nograd=True))
        optims.append(FlatAdamW(models[-1], lr=args.lr, weight_decay=0.0))
    aug = DeviceAugment(data.images("train"), means, inp_res=data.inpRes, use_flip=not a.no_aug,
                        use_noise=not a.no_aug, sf=0.0 if a.no_aug else 0.25, rf=0.0 if a.no_aug else 30.0,
                        device=dev)
    kps_all = np.array([it["kps"] for it in semi], np.float32)
    isl_all = np.array([it["islabeled"] for it in semi], bool)
    sampler = TwoStreamBatchSampler(uidx, lidx, a.trainBS, a.trainBS_labeled)
    vb = mouse.valid_batches(data, a.inferBS, dev)

    def loader():
        for idx in sampler:
            idx = list(idx)
            views, kps = [], []
            for _ in range(2):                                         # DS_mds augCount = 2
                x, k = aug.views(idx, kps_all[idx])
                views.append(x)
                kps.append(k)
            yield views, None, {"kps": kps, "islabeled": [torch.tensor(isl_all[idx], device=dev)]}

    log = {"config": {"model": a.model, "trainBS": a.trainBS, "trainBS_labeled": a.trainBS_labeled,
                      "epochs": a.epochs, "augment": not a.no_aug, "seed": a.seed, "split": "Mouse_100_500_0.3",
                      "pck_ref": data.pck_ref, "pck_thr": data.pck_thr, "means": means},
           "epochs": []}
    best = (-1.0, -1)
    t0 = time.time()
    for epo in range(a.epochs):                                        # :68-152
        args.epo = epo
        args.consWeight = PR.consWeight_increase(epo, args)
        args.FDLWeight = PR.FDLWeight_decrease(epo, args)
        args.pseudoWeight = PR.pseudoWeight_increase(epo, args)
        te = time.time()
        pec, mtc, epc, fdc = T.train_mt_ubpl(loader(), models, emas, optims, args, verbose=False)
        torch.cuda.synchronize()
        rec = {"epoch": epo + 1, "train_s": round(time.time() - te, 2), "pec": pec, "mtc": mtc, "epc": epc,
               "fdc": fdc}
        if (epo + 1) % a.valid_every == 0 or epo + 1 == a.epochs:
            _, accs, errs = T.validate(vb, emas, args)
            rec["pck"] = [round(v[-1], 4) for v in accs]               # teacher 1, teacher 2, mean
            rec["pck_per_kp_mean"] = [round(v, 4) for v in accs[-1][:-1]]
            m = max(rec["pck"])
            if m > best[0]:
                best = (m, epo + 1)
            print("epoch %3d  pck@0.2 t1 %.4f t2 %.4f mean %.4f  (%.1f s)" % (
                epo + 1, rec["pck"][0], rec["pck"][1], rec["pck"][2], time.time() - t0), flush=True)
        log["epochs"].append(rec)
    log["best_pck"], log["best_epoch"] = best
    log["final_pck"] = log["epochs"][-1]["pck"]
    log["wall_s"] = round(time.time() - t0, 1)
    if write:
        os.makedirs(os.path.dirname(a.out), exist_ok=True)
        with open(a.out, "w") as f:
            json.dump(log, f, indent=1)
    return log


if __name__ == "__main__":
    main()

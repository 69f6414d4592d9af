"""T1 — one training step of each project, restated on the CPU (oracle).

TEST INFRASTRUCTURE ONLY (see oracle/__init__.py).

Same batch format and args namespace as the reference train() functions
(projects/MT_UBPL.py:157-352, projects/DualPose_UBPL.py:156-295,
projects/MT.py:161-268, projects/supervised.py:135-175); returns the same
records.  Used (a) to pin the restatement against the reference's own train()
outputs (tests/golden/steps.npz) and (b) as bench.py's CPU baseline.
"""
import torch

from . import losses as L
from .decode import AvgCounter
from .schedule import ema_update


def _norm(s, n):
    return s / n if n > 0 else s


def _ema_all(models, emas, args):
    for m, e in zip(models, emas):
        ema_update(e.parameters(), [p.detach() for p in m.parameters()], args.epo, args.ema_decay)


def _fdc(features_a, features_b, sw, args):
    """Multi-view feature decorrelation (projects/MT_UBPL.py:301-330): labeled
    rows only (FDL_label 'labeled'), covariance (default) or distance."""
    rows = sw.reshape(-1) > 0
    if args.FDL_label == "unlabeled":
        rows = sw.reshape(-1) == 0
    elif args.FDL_label == "all":
        rows = torch.ones_like(rows)
    v1, v2 = features_a[rows], features_b[rows]
    if args.FDL_type == "covariance":
        return L.features_cov(v1, v2)
    return L.joint_feature_dist(v1, v2)


def train_mt_ubpl(loader, models, emas, optims, args, on_grads=None):
    """projects/MT_UBPL.py:157-352.  on_grads(models) is called with the
    students' final gradients, just before the optimizer steps."""
    M = len(models)
    pec_c = [AvgCounter() for _ in range(M)]
    mtc_c = [AvgCounter() for _ in range(M)]
    epc_c = [AvgCounter() for _ in range(M)]
    fdc_c = AvgCounter()
    counts = []
    for m in models:
        m.train()
    for e in emas:
        e.train()                                                  # :169 teachers in train mode
    for imgs, hms, meta in loader:
        for o in optims:
            o.zero_grad()
        isl = meta["islabeled"][0]
        sw = L.sample_weight(isl)                                  # :182 getSampleWeight
        nega = L.sample_weight_nega(isl, args.pseudoWeight)         # :183 getSampleWeight_nega
        gates = [kw[0] for kw in meta["kpsWeights"]]
        A = len(imgs)
        outs, feats, outs_ema = [], [], []
        for mi in range(M):                                        # :228-243
            o_a, f_a, e_a = [], [], []
            for a in range(A):
                o, f = models[mi](imgs[a])
                o_a.append(o)
                f_a.append(f)
                with torch.no_grad():
                    e_a.append(emas[mi](imgs[a])[0])
            outs.append(o_a)
            feats.append(f_a)
            outs_ema.append(e_a)
        mtc, pec, epc = [], [], []
        for mi in range(M):                                        # :247-256
            s, n = 0., 0
            for a in range(A):
                ls, ln = L.joint_dist(outs[mi][a][:, -1], outs_ema[mi][a][:, -1])
                s, n = s + ls, n + ln
            mtc.append(args.consWeight * _norm(s, n))
            mtc_c[mi].update(mtc[-1].item(), n)
        for mi in range(M):                                        # :259-268
            s, n = 0., 0
            for a in range(A):
                ls, ln = L.joint_mse(outs[mi][a], hms[a][0], args.nStack, gates[a], sw, True, True)
                s, n = s + ls, n + ln
            pec.append(args.poseWeight * _norm(s, n))
            pec_c[mi].update(pec[-1].item(), n)
        n_ps, n_sel = 0, 0
        if getattr(args, "useEnsemblePseudo", True):
            for mi in range(M):                                    # :271-291
                s, n = 0., 0
                for a in range(A):
                    tg = torch.stack([outs_ema[j][a] for j in range(M)]).detach()
                    ls, ln, ns, _, _, _ = L.joint_pseudo3(outs[mi][a], tg, nega, args.nStack, args.pseudoScoreThr)
                    s, n = s + ls, n + ln
                    n_ps, n_sel = n_ps + ln, n_sel + ns
                epc.append(args.ensemblePseudoWeight * _norm(s, n))
                epc_c[mi].update(epc[-1].item(), n)
            counts.append((n_sel, n_ps))
        else:                                                      # :292-293
            epc = [0.] * M
            for c in epc_c:
                c.update(0., imgs[0].shape[0])
        if args.FDLWeight <= 0:                                     # :298-330
            fdc = 0.
            fdc_c.update(0., imgs[0].shape[0])
        else:
            s, n = 0., 0
            for a in range(A):
                cs, cn = _fdc(feats[0][a], feats[1][a], sw, args)
                s, n = s + cs, n + cn
            fdc = args.FDLWeight * _norm(s, n)
            fdc_c.update(fdc.item(), n)
        for mi in range(M):                                        # :334-336 (fdc in both totals)
            (pec[mi] + mtc[mi] + epc[mi] + fdc).backward(retain_graph=True)
        if on_grads is not None:
            on_grads(models)
        for o in optims:
            o.step()
        _ema_all(models, emas, args)                               # :338
    rec = ([c.avg for c in pec_c], [c.avg for c in mtc_c], [c.avg for c in epc_c], fdc_c.avg)
    return rec, counts


def train_dualpose_ubpl(loader, models, emas, optims, args, on_grads=None):
    """projects/DualPose_UBPL.py:156-295."""
    M = len(models)
    pec_c = [AvgCounter() for _ in range(M)]
    mtc_c = [AvgCounter() for _ in range(M)]
    epc_c = [AvgCounter() for _ in range(M)]
    fdc_c = AvgCounter()
    counts = []
    for m in models:
        m.train()
    for e in emas:
        e.train()
    for stu_img, stu_hm, ema_img, meta in loader:
        for o in optims:
            o.zero_grad()
        isl = meta["islabeled"]
        gate = meta["kpsWeight"]
        sw = L.sample_weight(isl)                                  # getSampleWeight_mt
        nega = L.sample_weight_nega(isl, args.pseudoWeight)         # getSampleWeight_mt_nega
        cons = L.sample_weight_cons(isl, args.pseudoWeight)         # getSampleWeight_mt_cons
        outs, feats = [], []
        for mi in range(M):                                        # :185-190
            o, f = models[mi](stu_img)
            outs.append(o)
            feats.append(f)
        with torch.no_grad():                                      # :192-196 teacher sees ema_img
            outs_ema = torch.stack([emas[mi](ema_img)[0] for mi in range(M)])
        mtc, pec, epc = [], [], []
        c_ps, c_sel = 0, 0
        for mi in range(M):                                        # :200-214
            s, n, nps, nsel, _ = L.joint_dist_mt2(outs[mi][:, -1], outs_ema[mi][:, -1], sw=cons,
                                                  use_sw=True, thr=args.pseudoScoreThr)
            c_ps, c_sel = c_ps + nps, c_sel + nsel
            mtc.append(args.consWeight * _norm(s, n))
            mtc_c[mi].update(mtc[-1].item(), n)
        counts.append((c_sel, c_ps))
        for mi in range(M):                                        # :218-222
            s, n = L.joint_mse(outs[mi], stu_hm, args.nStack, gate, sw, True, True)
            pec.append(args.poseWeight * _norm(s, n))
            pec_c[mi].update(pec[-1].item(), n)
        e_ps, e_sel = 0, 0
        if getattr(args, "useEnsemblePseudo", True):
            for mi in range(M):                                    # :226-236
                s, n, nsel, _, _, _ = L.joint_pseudo3(outs[mi], outs_ema.detach(), nega, args.nStack,
                                                      args.pseudoScoreThr)
                e_ps, e_sel = e_ps + n, e_sel + nsel
                epc.append(args.ensemblePseudoWeight * _norm(s, n))
                epc_c[mi].update(epc[-1].item(), n)
            counts.append((e_sel, e_ps))
        else:                                                      # :243-245 (outs.shape[2] = nStack)
            epc = [0.] * M
            for c in epc_c:
                c.update(0., args.nStack)
        if args.FDLWeight <= 0:
            fdc = 0.
            fdc_c.update(0., args.nStack)                         # :249 outs.shape[2] = nStack
        else:
            cs, cn = _fdc(feats[0], feats[1], sw, args)             # :246-270
            fdc = args.FDLWeight * _norm(cs, cn)
            fdc_c.update(fdc.item(), cn)
        for mi in range(M):
            (pec[mi] + mtc[mi] + epc[mi] + fdc).backward(retain_graph=True)
        if on_grads is not None:
            on_grads(models)
        for o in optims:
            o.step()
        _ema_all(models, emas, args)
    rec = ([c.avg for c in pec_c], [c.avg for c in mtc_c], [c.avg for c in epc_c], fdc_c.avg)
    return rec, counts


def train_mt(loader, model, ema, optim, args, on_grads=None):
    """projects/MT.py:161-268 (one student + EMA teacher)."""
    pec_c, mtc_c = AvgCounter(), AvgCounter()
    model.train()
    ema.train()
    for imgs, hms, meta in loader:
        optim.zero_grad()
        isl = meta["islabeled"][0]
        sw = L.sample_weight(isl)
        gates = [kw[0] for kw in meta["kpsWeights"]]
        pick = (lambda r: r) if args.feature_mode == "default" else (lambda r: r[0])
        outs, outs_ema = [], []
        for a in range(len(imgs)):
            outs.append(pick(model(imgs[a])))
            with torch.no_grad():
                outs_ema.append(pick(ema(imgs[a])))
        s, n = 0., 0
        for a in range(len(imgs)):
            ls, ln = L.joint_dist(outs[a][:, -1], outs_ema[a][:, -1])
            s, n = s + ls, n + ln
        mtc = args.consWeight * _norm(s, n)
        mtc_c.update(mtc.item(), n)
        s, n = 0., 0
        for a in range(len(imgs)):
            ls, ln = L.joint_mse(outs[a], hms[a][0], args.nStack, gates[a], sw, True, True)
            s, n = s + ls, n + ln
        pec = args.poseWeight * _norm(s, n)
        pec_c.update(pec.item(), n)
        (pec + mtc).backward()
        if on_grads is not None:
            on_grads([model])
        optim.step()
        _ema_all([model], [ema], args)
    return (pec_c.avg, mtc_c.avg), []


def train_supervised(loader, model, optim, args, on_grads=None):
    """projects/supervised.py:135-175."""
    pec_c = AvgCounter()
    model.train()
    for img, hm, meta in loader:
        optim.zero_grad()
        out = model(img) if args.feature_mode == "default" else model(img)[0]
        s, n = L.joint_mse(out, hm, args.nStack)
        pec = args.poseWeight * _norm(s, n)
        pec_c.update(pec.item(), n)
        pec.backward()
        if on_grads is not None:
            on_grads([model])
        optim.step()
    return pec_c.avg, []

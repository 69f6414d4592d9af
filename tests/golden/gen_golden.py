"""Generate golden vectors for the hot path by running the REFERENCE itself.

TEST INFRASTRUCTURE ONLY.  This script imports /root/reference (read-only,
never shipped) through the stub recipe of SURVEY.md Appendix B and writes
small fixtures into tests/golden/*.npz / *.json.  It runs only in the build
container; the GPU box never sees /root/reference, it sees only the fixtures.

Inputs are regenerated from seeds (torch CPU Generator, numpy RandomState),
so the fixtures hold mostly outputs.  The seeding helpers used here live in
tests/golden/seeds.py and are shared with the tests, so that tests rebuild the
exact same inputs.

Usage:  python tests/golden/gen_golden.py
"""
import contextlib
import io
import json
import os
import re
import sys
import types

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
import seeds  # noqa: E402

REF = "/root/reference"


def import_reference():
    sys.dont_write_bytecode = True
    sys.path.insert(0, REF)
    for name in ["cv2", "openpyxl", "openpyxl.styles", "skimage", "skimage.transform",
                 "skimage.data", "imageio", "torchvision"]:
        try:
            __import__(name)
        except ImportError:
            sys.modules[name] = types.ModuleType(name)
    sys.modules["openpyxl.styles"].PatternFill = object
    cuda = torch.Tensor.cuda
    torch.Tensor.cuda = lambda self, *a, **k: self  # utils/udaap/imutils.py:190
    import utils.losses  # noqa: F401
    import utils.process  # noqa: F401
    import utils.evaluation  # noqa: F401
    import utils.augment  # noqa: F401
    torch.Tensor.cuda = cuda
    mods = {}
    import utils.losses as L
    import utils.process as P
    import utils.evaluation as E
    import utils.parameters as PR
    import utils.udaap.evaluation as UE
    import utils.mt.data as MD
    import utils.udaap.transforms as UT
    import projects.tools as T
    from models.pose.hourglass import StackedHourglass
    mods.update(L=L, P=P.ProcessUtils, E=E.EvaluationUtils, PR=PR, UE=UE, MD=MD, UT=UT,
                T=T.ProjectTools, SH=StackedHourglass)
    return mods


# --------------------------------------------------------------------------
# R1 renderer
# --------------------------------------------------------------------------
def gen_render(R):
    out = {}
    cases = seeds.render_cases()
    for name, (kps, imgshape, inp, outr) in cases.items():
        k = torch.from_numpy(kps.copy())
        hm, kps_after = R["P"].kps_heatmap(k, imgshape, inp, outr)
        out[name + "/kps"] = kps
        out[name + "/hm"] = hm.numpy()
        out[name + "/kps_after"] = kps_after.numpy()
        out[name + "/meta"] = np.array([imgshape[1], imgshape[2], inp, outr], np.int64)
    # the multi-kps variant (utils/process.py:288) on two maps
    kpa = [torch.from_numpy(cases["mixed16"][0].copy()), torch.from_numpy(cases["edges16"][0].copy())]
    hms, kpsn = R["P"].kps_heatmap_mulKps(kpa, (3, 256, 256), 256, 64)
    out["mul/hm0"], out["mul/hm1"] = hms[0].numpy(), hms[1].numpy()
    out["mul/kps0"], out["mul/kps1"] = kpsn[0].numpy(), kpsn[1].numpy()
    np.savez_compressed(os.path.join(HERE, "render.npz"), **out)


# --------------------------------------------------------------------------
# L1-L7 losses (+ gradients)
# --------------------------------------------------------------------------
def _grad(loss_tuple_fn, *tensors):
    ts = [t.clone().requires_grad_(True) for t in tensors]
    res = loss_tuple_fn(*ts)
    res[0].backward()
    return res, [t.grad.numpy().copy() for t in ts]


def _sub(a, R):
    """Full gradient for small maps; a strided subsample (every 4th pixel) at R > 16."""
    return a if R <= 16 else a[..., ::4, ::4].copy()


def gen_losses(R):
    L = R["L"]
    out = {}
    for cname, cfg in seeds.loss_cases().items():
        d = seeds.loss_inputs(**cfg)
        B, S, K = cfg["B"], cfg["S"], cfg["K"]
        # L1 JointMSELoss, gated + sample weighted (projects/MT_UBPL.py:162)
        crit = L.JointMSELoss(nStack=S, useKPsGate=True, useSampleWeight=True)
        (s, n), (g,) = _grad(lambda p: crit(p, d["gts"], d["gate"], d["sw_lab"]), d["preds"])
        out[cname + "/mse_sum"], out[cname + "/mse_n"], out[cname + "/mse_dp"] = s.item(), n, _sub(g, cfg["R"])
        # L1 ungated (projects/supervised.py:138)
        crit = L.JointMSELoss(nStack=S)
        (s, n), (g,) = _grad(lambda p: crit(p, d["gts"]), d["preds"])
        out[cname + "/mse0_sum"], out[cname + "/mse0_n"], out[cname + "/mse0_dp"] = s.item(), n, _sub(g, cfg["R"])
        # L2 JointDistLoss on last stack (projects/MT_UBPL.py:163,250)
        crit = L.JointDistLoss()
        (s, n), (g,) = _grad(lambda p: crit(p, d["tlast"][0]), d["preds"][:, -1].contiguous())
        out[cname + "/dist_sum"], out[cname + "/dist_n"], out[cname + "/dist_dp"] = s.item(), n, _sub(g, cfg["R"])
        # L3 JointDistLoss_mt2 (projects/DualPose_UBPL.py:163,203)
        crit = L.JointDistLoss_mt2(useSampleWeight=True, scoreThr=cfg["thr"])
        (s, n, npse, nsel, sc), (g,) = _grad(
            lambda p: crit(p, d["tlast"][0], sampleWeight=d["sw_cons"]), d["preds"][:, -1].contiguous())
        out[cname + "/mt2_sum"], out[cname + "/mt2_n"] = s.item(), n
        out[cname + "/mt2_npse"], out[cname + "/mt2_nsel"] = npse, nsel
        out[cname + "/mt2_score"], out[cname + "/mt2_dp"] = sc.detach().numpy(), _sub(g, cfg["R"])
        # L4 JointPseudoLoss3 (projects/MT_UBPL.py:279)
        crit = L.JointPseudoLoss3(nStack=S, scoreThr=cfg["thr"])
        if cfg.get("pseudo", True):
            (s, n, nsel, sc, t1, t2), (g,) = _grad(
                lambda p: crit(p, d["teachers"], d["sw_nega"]), d["preds"])
            out[cname + "/ps_sum"], out[cname + "/ps_n"], out[cname + "/ps_nsel"] = s.item(), n, nsel
            out[cname + "/ps_score"], out[cname + "/ps_dp"] = sc.detach().numpy(), _sub(g, cfg["R"])
        # L6 JointFeatureDistLoss and L5 features_cov (utils/process.py:18)
        f1, f2 = d["f1"], d["f2"]
        crit = L.JointFeatureDistLoss()
        (s, n), (g1, g2) = _grad(lambda a, b: crit(a, b), f1, f2)
        out[cname + "/fdist_sum"], out[cname + "/fdist_n"] = s.item(), n
        out[cname + "/fdist_g1"], out[cname + "/fdist_g2"] = g1, g2
        (s, n), (g1, g2) = _grad(lambda a, b: R["P"].features_cov(a, b), f1, f2)
        out[cname + "/cov_val"], out[cname + "/cov_n"] = s.item(), n
        out[cname + "/cov_g1"], out[cname + "/cov_g2"] = g1, g2
        # L7 sample weights (projects/tools.py:13-54)
        args = types.SimpleNamespace(device="cpu", pseudoWeight=cfg["pw"])
        isl = d["islabeled"]
        out[cname + "/w"] = R["T"].getSampleWeight([isl], args)[0].detach().numpy()
        out[cname + "/w_nega"] = R["T"].getSampleWeight_nega([isl], args)[0].detach().numpy()
        out[cname + "/w_mt"] = R["T"].getSampleWeight_mt(isl, args).detach().numpy()
        out[cname + "/w_mt_nega"] = R["T"].getSampleWeight_mt_nega(isl, args).detach().numpy()
        out[cname + "/w_mt_cons"] = R["T"].getSampleWeight_mt_cons(isl, args).detach().numpy()
    # the all-labeled batch makes JointPseudoLoss3 raise (utils/losses.py:201)
    d = seeds.loss_inputs(**seeds.loss_cases()["alllab"])
    try:
        L.JointPseudoLoss3(nStack=2, scoreThr=0.95)(d["preds"], d["teachers"], d["sw_nega"])
        out["alllab/ps_raises"] = 0
    except RuntimeError:
        out["alllab/ps_raises"] = 1
    np.savez_compressed(os.path.join(HERE, "losses.npz"), **out)


# --------------------------------------------------------------------------
# D1-D4 decoder + PCK
# --------------------------------------------------------------------------
def gen_decode(R):
    out = {}
    for cname, cfg in seeds.decode_cases().items():
        hm, center, scale = seeds.decode_inputs(**cfg)
        preds, scores = R["P"].kps_fromHeatmap(hm.clone(), center, scale, [cfg["R"], cfg["R"]])
        out[cname + "/preds"] = preds.numpy()
        out[cname + "/scores"] = scores.numpy()
        out[cname + "/raw"] = R["UE"].get_preds(hm.clone()).numpy()
    for cname, cfg in seeds.pck_cases().items():
        preds, gts = seeds.pck_inputs(**cfg)
        errs, accs = R["E"].acc_pck(preds, gts, cfg["ref"], cfg["thr"])
        out[cname + "/errs"], out[cname + "/accs"] = errs.numpy(), accs.numpy()
    np.savez_compressed(os.path.join(HERE, "decode.npz"), **out)


# --------------------------------------------------------------------------
# E1 EMA, E2 ramps, S1 sampler
# --------------------------------------------------------------------------
def gen_misc(R):
    PR = R["PR"]
    out = {}
    for epo in [0, 1, 5, 2000]:
        ema, cur = seeds.ema_inputs()
        m_ema, m = torch.nn.Module(), torch.nn.Module()
        m_ema.p = torch.nn.ParameterList([torch.nn.Parameter(t.clone()) for t in ema])
        m.p = torch.nn.ParameterList([torch.nn.Parameter(t.clone()) for t in cur])
        PR.update_ema_variables(m, m_ema, types.SimpleNamespace(epo=epo, ema_decay=0.999))
        for i, p in enumerate(m_ema.p):
            out["ema/epo%d/%d" % (epo, i)] = p.detach().numpy()
    np.savez_compressed(os.path.join(HERE, "ema.npz"), **out)

    ramps = {}
    a = types.SimpleNamespace(consWeight_max=10.0, consWeight_min=0.0, consWeight_rampup=5,
                              pseudoWeight_max=1.0, pseudoWeight_min=1.0, pseudoWeight_rampup=100,
                              FDLWeight_max=1.0, FDLWeight_min=0.2, FDLWeight_rampup=30)
    for e in range(0, 40):
        ramps["cons/%d" % e] = PR.consWeight_increase(e, a)
        ramps["pseudo/%d" % e] = PR.pseudoWeight_increase(e, a)
        ramps["fdl_dec/%d" % e] = PR.FDLWeight_decrease(e, a)
        ramps["fdl_inc/%d" % e] = PR.FDLWeight_increase(e, a)

    samp = {}
    for cname, (prim, sec, bs, sbs, seed) in seeds.sampler_cases().items():
        np.random.seed(seed)
        sm = R["MD"].TwoStreamBatchSampler(prim, sec, bs, sbs)
        samp[cname] = {"len": len(sm), "batches": [[int(i) for i in b] for b in sm]}
    with open(os.path.join(HERE, "misc.json"), "w") as f:
        json.dump({"ramps": ramps, "sampler": samp}, f, indent=0, sort_keys=True)


# --------------------------------------------------------------------------
# f1 augmentation geometry: keypoints through transform() (utils/udaap/transforms.py:151-158)
# --------------------------------------------------------------------------
def gen_augment(R):
    """The reference's own transform() / get_transform() on the loader's
    operand types (float32 keypoint tensor rows, int64 centre tensor,
    float32 0-d scale / angle tensors: utils/augment.py:150-156), and the
    integer crop corners affine_image computes (utils/augment.py:108-110:
    transform([0, 0] / res, invert=1) of the unrotated transform)."""
    out = {}
    for cname, (center, scale, rot, pts) in seeds.augment_cases().items():
        c = torch.tensor(center)
        res = [[int(v) for v in R["UT"].transform(p, c, scale, [256, 256], rot=rot)] for p in pts]
        out[cname + "/kps"] = np.array(res, np.int64)
        out[cname + "/t"] = R["UT"].get_transform(c, scale, [256, 256], rot=rot)
        out[cname + "/ul"] = np.array(R["UT"].transform([0, 0], c, scale, [256, 256], invert=1))
        out[cname + "/br"] = np.array(R["UT"].transform([256, 256], c, scale, [256, 256], invert=1))
    np.savez_compressed(os.path.join(HERE, "augment.npz"), **out)


def gen_occlusion(R):
    """f1 occlusion: the reference's own paste_over (utils/udaap/utils_augment.py:
    131-163) on synthetic occluders and images (Augment.__init__ needs Pascal VOC
    and resize_by_factor needs cv2 — both absent — so the pastes are made with
    already-sized occluders): pins the clipping geometry and the blend."""
    import utils.udaap.utils_augment as UA
    aug = object.__new__(UA.Augment)
    out = {}
    for cname, (dst, occ, center) in seeds.occlusion_cases().items():
        d = dst.copy()
        aug.paste_over(im_src=occ, im_dst=d, center=np.asarray(center, np.float64))
        out[cname + "/out"] = d
    np.savez_compressed(os.path.join(HERE, "occlusion.npz"), **out)


# --------------------------------------------------------------------------
# H1-H6 hourglass forward/backward
# --------------------------------------------------------------------------
def _param_stats(model):
    names, stats = [], []
    for n, p in model.named_parameters():
        names.append(n)
        v = p.detach().double()
        stats.append([v.sum().item(), (v * v).sum().item()])
    return names, np.array(stats)


def _buf_stats(model):
    names, stats = [], []
    for n, b in model.named_buffers():
        names.append(n)
        v = b.detach().double()
        stats.append([v.sum().item(), (v * v).sum().item()])
    return names, np.array(stats)


def gen_hourglass(R):
    out = {}
    meta = {}
    for cname, cfg in seeds.hg_cases().items():
        torch.manual_seed(cfg["seed"])
        m = R["SH"](cfg["K"], cfg["S"], cfg["mode"])
        names, pst = _param_stats(m)
        bnames, _ = _buf_stats(m)
        meta[cname] = {"param_names": names, "param_shapes": [list(p.shape) for p in m.parameters()],
                       "buffer_names": bnames}
        out[cname + "/param_stats"] = pst
        x, gp, gf = seeds.hg_inputs(**cfg)
        m.train()
        res = m(x)
        preds, feats = (res, None) if cfg["mode"] == "default" else res
        out[cname + "/preds"] = preds.detach().numpy()[:, :, :, ::cfg["sub"], ::cfg["sub"]].copy()
        out[cname + "/preds_sum"] = np.array([preds.double().sum().item(), (preds.double() ** 2).sum().item()])
        loss = (preds * gp).sum()
        if feats is not None:
            out[cname + "/feats_sum"] = np.array([feats.double().sum().item(), (feats.double() ** 2).sum().item()])
            out[cname + "/feats"] = feats.detach().numpy()[:, :, :8, ::4, ::4].copy()
            loss = loss + (feats * gf).sum()
        loss.backward()
        gst = []
        for n, p in m.named_parameters():
            if p.grad is None:
                gst.append([0.0, 0.0, 0.0])
            else:
                g = p.grad.double()
                gst.append([g.sum().item(), (g * g).sum().item(), 1.0])
        out[cname + "/grad_stats"] = np.array(gst)
        _, bst = _buf_stats(m)
        out[cname + "/buf_stats_after_train_fwd"] = bst
        # eval-mode forward with the updated running stats (projects/MT_UBPL.py:362)
        m.eval()
        with torch.no_grad():
            res = m(x)
        preds = res if cfg["mode"] == "default" else res[0]
        out[cname + "/eval_preds_sum"] = np.array([preds.double().sum().item(), (preds.double() ** 2).sum().item()])
        out[cname + "/eval_preds"] = preds.numpy()[:, :, :, ::cfg["sub"], ::cfg["sub"]].copy()
    np.savez_compressed(os.path.join(HERE, "hourglass.npz"), **out)
    with open(os.path.join(HERE, "hourglass_meta.json"), "w") as f:
        json.dump(meta, f)


# --------------------------------------------------------------------------
# T1 one full training step of each project (reference train())
# --------------------------------------------------------------------------
_PRINT_RE = re.compile(r"\((\s*\d+)/(\s*\d+)\)")


def _import_project(name):
    cuda = torch.Tensor.cuda
    torch.Tensor.cuda = lambda self, *a, **k: self
    try:
        mod = __import__("projects." + name, fromlist=["train"])
    finally:
        torch.Tensor.cuda = cuda
    return mod


def gen_steps(R):
    out = {}
    for cname, cfg in seeds.step_cases().items():
        print("  step case", cname, flush=True)
        proj = _import_project(cfg["project"])
        models, emas, optims = seeds.step_models(R["SH"], cfg)
        before = [[p.detach().clone() for p in m.parameters()] for m in models + emas]
        loader, args = seeds.step_batch(cfg, R["P"].kps_heatmap)
        # each student's gradients as the reference's optimizer sees them (step pre-hook)
        grads = {}
        for mi, (m, o) in enumerate(zip(models, optims)):
            def hook(opt, a, kw, m=m, mi=mi):
                grads[mi] = seeds.grad_record([(n, p.grad) for n, p in m.named_parameters()])
            o.register_step_pre_hook(hook)
        buf = io.StringIO()
        with contextlib.redirect_stdout(buf):
            if cfg["project"] in ("MT_UBPL", "DualPose_UBPL"):
                rec = proj.train(loader, models, emas, optims, args)
            elif cfg["project"] == "MT":
                rec = proj.train(loader, models[0], emas[0], optims[0], args)
            else:
                rec = proj.train(loader, models[0], optims[0], args)
        counts = [[int(a), int(b)] for a, b in _PRINT_RE.findall(buf.getvalue())]
        out[cname + "/printed_counts"] = np.array(counts, np.int64).reshape(-1, 2)
        out[cname + "/records"] = np.array(_flatten(rec), np.float64)
        for mi, (m, bp) in enumerate(zip(models + emas, before)):
            upd, absu, psum = [], [], []
            for p, p0 in zip(m.parameters(), bp):
                d = (p.detach().double() - p0.double()) / args.lr
                upd.append(d.sum().item())
                absu.append(d.abs().sum().item())
                psum.append(p.detach().double().sum().item())
            out[cname + "/model%d/upd" % mi] = np.array(upd)
            out[cname + "/model%d/absupd" % mi] = np.array(absu)
            out[cname + "/model%d/psum" % mi] = np.array(psum)
            _, bst = _buf_stats(m)
            out[cname + "/model%d/buf" % mi] = bst
            if mi in grads:
                out[cname + "/model%d/grad_stats" % mi], out[cname + "/model%d/grad_samp" % mi] = grads[mi]
    np.savez_compressed(os.path.join(HERE, "steps.npz"), **out)


def _flatten(x):
    if isinstance(x, (list, tuple)):
        r = []
        for v in x:
            r.extend(_flatten(v))
        return r
    return [float(x)]


if __name__ == "__main__":
    torch.set_num_threads(8)
    R = import_reference()
    which = sys.argv[1:] or ["render", "losses", "decode", "misc", "augment", "occlusion", "hourglass", "steps"]
    for w in which:
        print("generating", w, flush=True)
        globals()["gen_" + w](R)
    print("done")

"""The drop-in boundary driven the way the reference's own train() drives it.

dropin/ goes first on sys.path, so `models`, `utils.losses`,
`utils.parameters`, `utils.process` and `projects.tools` resolve to the
MI355X-native modules under the reference's module paths.  The body below is
a build-authored harness that makes the reference's calls, in the order of
projects/MT_UBPL.py:173-339 (not a copy of that file): per batch zero_grad,
setVariable, getSampleWeight(_nega), per (model, view) student forward and
no_grad teacher forward, torch.stack of the outputs, JointDistLoss /
JointMSELoss / JointPseudoLoss3(outs_ema.clone()[:, a].detach()) with their
.item() counters, the per-sample FDL row selection feeding
ProcessUtils.features_cov, total_i.backward(retain_graph=True) per student,
torch.optim.AdamW.step() and update_ema_variables.  Checked against the
reference's own records and printed counts for the golden mt_ubpl batch
(steps.npz), with the fp64 noise-floor criterion of test_gpu_train.
"""
import os
import sys
import types

import numpy as np
import pytest
import torch

import seeds

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GD = os.path.join(ROOT, "tests", "golden")
DROPIN = os.path.join(ROOT, "ubpl-poseestimation_amd", "dropin")


@pytest.fixture
def dropin_modules(monkeypatch):
    monkeypatch.syspath_prepend(DROPIN)
    for name in [m for m in sys.modules if m.split(".")[0] in ("models", "utils", "projects")]:
        monkeypatch.delitem(sys.modules, name)
    import models
    import projects.tools
    import utils.losses
    import utils.parameters
    import utils.process
    yield types.SimpleNamespace(models=models, L=utils.losses, PR=utils.parameters,
                                proc=utils.process.ProcessUtils, proj=projects.tools.ProjectTools)
    for name in [m for m in sys.modules if m.split(".")[0] in ("models", "utils", "projects")]:
        sys.modules.pop(name, None)


def _reference_style_train(R, loader, models, models_ema, optims, args):
    """The call sequence of projects/MT_UBPL.py:157-352 over the drop-in modules."""
    L, proc, proj = R.L, R.proc, R.proj
    pec_c = [L.AvgCounter() for _ in models]
    mtc_c = [L.AvgCounter() for _ in models]
    epc_c = [L.AvgCounter() for _ in models]
    fdc_c = L.AvgCounter()
    pose_criterion = L.JointMSELoss(nStack=args.nStack, useKPsGate=True, useSampleWeight=True)
    consistency_criterion = L.JointDistLoss()
    pseudo_criterion2 = L.JointPseudoLoss3(nStack=args.nStack, scoreThr=args.pseudoScoreThr)
    printed = []
    for m in models:
        m.train()
    for m in models_ema:
        m.train()
    for bat, (augs_imgMap, augs_heatmaps, meta) in enumerate(loader):
        for o in optims:
            o.zero_grad()
        augs_heatmaps = [[proj.setVariable(h, args.device) for h in hs] for hs in augs_heatmaps]
        augs_kpsGate = [[proj.setVariable(k, args.device) for k in ks] for ks in meta["kpsWeights"]]
        augs_imgMap = [proj.setVariable(x, args.device) for x in augs_imgMap]
        sw = proj.getSampleWeight(meta["islabeled"], args)
        nega = proj.getSampleWeight_nega(meta["islabeled"], args)
        outs, features, outs_ema = [], [], []
        for mi in range(len(models)):
            oa, fa, ea = [], [], []
            for img in augs_imgMap:
                out, feature = models[mi](img)
                oa.append(out)
                fa.append(feature)
                with torch.no_grad():
                    out_ema, _ = models_ema[mi](img)
                    ea.append(out_ema)
            outs.append(torch.stack(oa, dim=0))
            features.append(torch.stack(fa, dim=0))
            outs_ema.append(torch.stack(ea, dim=0))
        outs, features, outs_ema = torch.stack(outs, 0), torch.stack(features, 0), torch.stack(outs_ema, 0)
        mtc_losses = []
        for mi in range(len(outs)):
            s, n = 0., 0
            for a in range(len(outs[mi])):
                loss, c = consistency_criterion(outs[mi, a, :, -1], outs_ema[mi, a, :, -1])
                s, n = s + loss, n + c
            mtc_losses.append(args.consWeight * ((s / n) if n > 0 else s))
            mtc_c[mi].update(mtc_losses[mi].item(), n)
        pec_losses = []
        for mi in range(len(outs)):
            s, n = 0., 0
            for a in range(len(outs[mi])):
                loss, c = pose_criterion(outs[mi, a], augs_heatmaps[a][0], augs_kpsGate[a][0], sw[0])
                s, n = s + loss, n + c
            pec_losses.append(args.poseWeight * ((s / n) if n > 0 else s))
            pec_c[mi].update(pec_losses[mi].item(), n)
        n_ps, n_sel, epc_losses = 0, 0, []
        for mi in range(len(outs)):
            s, n = 0., 0
            for a in range(len(outs[mi])):
                loss, c, ns, _, _, _ = pseudo_criterion2(outs[mi, a], outs_ema.clone()[:, a].detach(), nega[0])
                s, n = s + loss, n + c
                n_ps, n_sel = n_ps + c, n_sel + ns
            epc_losses.append(args.ensemblePseudoWeight * ((s / n) if n > 0 else s))
            epc_c[mi].update(epc_losses[mi].item(), n)
        printed.append((n_sel, n_ps))
        s, n = 0., 0
        for a in range(features.shape[1]):
            v1 = torch.stack([features[0, a, i] for i, w in enumerate(sw[0]) if w > 0], 0)
            v2 = torch.stack([features[1, a, i] for i, w in enumerate(sw[0]) if w > 0], 0)
            c_cov, c_num = proc.features_cov(v1, v2)
            s, n = s + c_cov, n + c_num
        fdc_loss = args.FDLWeight * ((s / n) if n > 0 else s)
        fdc_c.update(fdc_loss.item(), n)
        for mi in range(len(models)):
            (pec_losses[mi] + mtc_losses[mi] + epc_losses[mi] + fdc_loss).backward(retain_graph=True)
        for o in optims:
            o.step()
        for mi, m in enumerate(models):
            R.PR.update_ema_variables(m, models_ema[mi], args)
    return ([c.avg for c in pec_c], [c.avg for c in mtc_c], [c.avg for c in epc_c], fdc_c.avg), printed


def test_reference_call_order_on_dropin_modules(dropin_modules):
    R = dropin_modules
    from oracle import render as OR
    cfg = seeds.step_cases()["mt_ubpl"]
    PoseModel = R.models.__dict__["PoseModel"]                      # projects/MT_UBPL.py:43
    torch.manual_seed(1388)
    models, emas, optims = [], [], []
    for _ in range(cfg["brNum"]):                                   # :43-50
        models.append(PoseModel("HG%d" % cfg["S"], cfg["K"], cfg["mode"]))
        emas.append(PoseModel("HG%d" % cfg["S"], cfg["K"], cfg["mode"], nograd=True))
        optims.append(torch.optim.AdamW(models[-1].parameters(), lr=cfg["lr"], weight_decay=0))
    loader, args = seeds.step_batch(cfg, OR.kps_heatmap_torch)
    args.device = torch.device("cuda")
    rec, printed = _reference_style_train(R, loader, models, emas, optims, args)
    g = np.load(os.path.join(GD, "steps.npz"))
    g64 = np.load(os.path.join(GD, "steps64.npz"))
    flat = np.array([v for x in rec for v in (x if isinstance(x, list) else [x])], np.float64)
    r32, r64 = g["mt_ubpl/records"], g64["mt_ubpl/records"]
    assert (np.abs(flat - r64) <= 3 * np.abs(r32 - r64) + 1e-4 * np.abs(r64) + 1e-12).all(), (flat, r32)
    assert np.array_equal(np.array(printed, np.int64).reshape(-1, 2), g["mt_ubpl/printed_counts"])
    # the teachers moved by the EMA (alpha keyed on epoch 1 = 0.5) away from their own init
    torch.manual_seed(1388)
    PoseModel("HG%d" % cfg["S"], cfg["K"], cfg["mode"])
    t0 = PoseModel("HG%d" % cfg["S"], cfg["K"], cfg["mode"], nograd=True)
    s_new = dict(models[0].named_parameters())["preds.1.conv.weight"].detach()
    want = 0.5 * dict(t0.named_parameters())["preds.1.conv.weight"].detach() + 0.5 * s_new
    got = dict(emas[0].named_parameters())["preds.1.conv.weight"].detach()
    assert torch.allclose(got, want, rtol=1e-6, atol=1e-7)

"""HIP kernels vs the oracle / golden fixtures / torch-CPU fp32 references.

Every test here needs an MI355X (pytest -m gpu).  Tolerances are stated per
test: integer / index work bit-exact, fp32 heatmaps and losses 1e-4 relative
(BASELINE.json north_star), single conv layers ~1e-5 (exact-f32 MFMA chains
vs MKL ordering).
"""
import os

import numpy as np
import pytest
import torch
import torch.nn.functional as F

import seeds
from oracle import decode as OD
from oracle import losses as OL
from oracle import render as OR

pytestmark = pytest.mark.gpu
GD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
DEV = "cuda"


@pytest.fixture(scope="module", autouse=True)
def _lib_loaded():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from ubpl_amd import _lib
    _lib.load()


def _npz(n):
    return np.load(os.path.join(GD, n))


def _close(a, b, rtol=1e-4, atol=1e-6):
    a = a.detach().cpu().double().numpy() if torch.is_tensor(a) else np.asarray(a, np.float64)
    b = b.detach().cpu().double().numpy() if torch.is_tensor(b) else np.asarray(b, np.float64)
    np.testing.assert_allclose(a, b, rtol=rtol, atol=atol)


# ----------------------------------------------------------------- R1
def test_render_matches_golden_bit_exact():
    from ubpl_amd import kernels as Kn
    g = _npz("render.npz")
    for name, (kps, shape, inp, out) in seeds.render_cases().items():
        k = torch.from_numpy(kps).to(DEV).reshape(1, -1, 3).contiguous()
        hm, ko = Kn.render_heatmaps(k, (shape[1], shape[2]), inp, out)
        assert np.array_equal(hm[0].cpu().numpy(), g[name + "/hm"]), name
        assert np.array_equal(ko[0].cpu().numpy(), g[name + "/kps_after"]), name


def test_render_batch_vs_oracle():
    from ubpl_amd.process import render_batch
    rs = np.random.RandomState(5)
    kps = np.zeros((32, 16, 3), np.float32)
    kps[..., :2] = rs.randint(-5, 262, (32, 16, 2))
    kps[..., 2] = 1
    kps[::3] = 0.0   # unlabeled rows
    hm, ko = render_batch(torch.from_numpy(kps).to(DEV), (256, 256), 256, 64)
    rh, rk = OR.render_batch(kps, (256, 256), 256, 64)
    assert np.array_equal(hm.cpu().numpy(), rh)
    assert np.array_equal(ko.cpu().numpy(), rk)


def test_process_kps_heatmap_inplace_cpu_io():
    from ubpl_amd.process import ProcessUtils
    kps, shape, inp, out = seeds.render_cases()["edges16"]
    k = torch.from_numpy(kps.copy())
    hm, k2 = ProcessUtils.kps_heatmap(k, shape, inp, out)
    assert hm.device.type == "cpu" and k2 is k
    assert np.array_equal(hm.numpy(), _npz("render.npz")["edges16/hm"])
    assert np.array_equal(k.numpy(), _npz("render.npz")["edges16/kps_after"])


# ----------------------------------------------------------------- L1-L7
def _g(fn, *ts):
    ts = [t.clone().to(DEV).requires_grad_(True) for t in ts]
    r = fn(*ts)
    r[0].backward()
    return r, [t.grad.cpu() for t in ts]


def _sub(a, R):
    return a if R <= 16 else a[..., ::4, ::4]


@pytest.mark.parametrize("case", list(seeds.loss_cases().keys()))
def test_losses_vs_golden(case):
    from ubpl_amd import losses as L
    g = _npz("losses.npz")
    cfg = seeds.loss_cases()[case]
    d = {k: (v.to(DEV) if torch.is_tensor(v) else v) for k, v in seeds.loss_inputs(**cfg).items()}
    S, R = cfg["S"], cfg["R"]
    tol = dict(rtol=1e-4, atol=1e-7)
    crit = L.JointMSELoss(nStack=S, useKPsGate=True, useSampleWeight=True)
    (s, n), (dp,) = _g(lambda p: crit(p, d["gts"], d["gate"], d["sw_lab"]), d["preds"])
    _close(s, g[case + "/mse_sum"], **tol); assert n == g[case + "/mse_n"]
    _close(_sub(dp.numpy(), R), g[case + "/mse_dp"], rtol=1e-4, atol=1e-8)
    crit = L.JointMSELoss(nStack=S)
    (s, n), (dp,) = _g(lambda p: crit(p, d["gts"]), d["preds"])
    _close(s, g[case + "/mse0_sum"], **tol); assert n == g[case + "/mse0_n"]
    _close(_sub(dp.numpy(), R), g[case + "/mse0_dp"], rtol=1e-4, atol=1e-8)
    last = d["preds"][:, -1].contiguous()
    crit = L.JointDistLoss()
    (s, n), (dp,) = _g(lambda p: crit(p, d["tlast"][0]), last)
    _close(s, g[case + "/dist_sum"], **tol); assert n == g[case + "/dist_n"]
    _close(_sub(dp.numpy(), R), g[case + "/dist_dp"], rtol=1e-4, atol=1e-8)
    crit = L.JointDistLoss_mt2(useSampleWeight=True, scoreThr=cfg["thr"])
    (s, n, nps, nsel, sc), (dp,) = _g(lambda p: crit(p, d["tlast"][0], sampleWeight=d["sw_cons"]), last)
    _close(s, g[case + "/mt2_sum"], **tol); assert n == g[case + "/mt2_n"]
    assert nps == g[case + "/mt2_npse"] and nsel == g[case + "/mt2_nsel"]
    _close(sc, g[case + "/mt2_score"], rtol=1e-5)
    _close(_sub(dp.numpy(), R), g[case + "/mt2_dp"], rtol=1e-4, atol=1e-8)
    crit = L.JointPseudoLoss3(nStack=S, scoreThr=cfg["thr"])
    if cfg.get("pseudo", True):
        (s, n, nsel, sc, _, _), (dp,) = _g(lambda p: crit(p, d["teachers"], d["sw_nega"]), d["preds"])
        _close(s, g[case + "/ps_sum"], **tol); assert n == g[case + "/ps_n"]
        assert nsel == g[case + "/ps_nsel"]
        _close(sc, g[case + "/ps_score"], rtol=1e-5)
        _close(_sub(dp.numpy(), R), g[case + "/ps_dp"], rtol=1e-4, atol=1e-8)
    else:
        with pytest.raises(RuntimeError):
            crit(d["preds"], d["teachers"], d["sw_nega"])
    crit = L.JointFeatureDistLoss()
    (s, n), (g1, g2) = _g(lambda a, b: crit(a, b), d["f1"], d["f2"])
    _close(s, g[case + "/fdist_sum"], **tol); assert n == g[case + "/fdist_n"]
    _close(g1, g[case + "/fdist_g1"], atol=1e-6); _close(g2, g[case + "/fdist_g2"], atol=1e-6)
    from ubpl_amd.process import ProcessUtils
    (s, n), (g1, g2) = _g(lambda a, b: ProcessUtils.features_cov(a, b), d["f1"], d["f2"])
    _close(s, g[case + "/cov_val"], **tol); assert n == g[case + "/cov_n"]
    _close(g1, g[case + "/cov_g1"], atol=1e-6); _close(g2, g[case + "/cov_g2"], atol=1e-6)


def test_features_cov_rowmask_matches_selection():
    """The fused labeled-row selection (projects/MT_UBPL.py:309-320) equals
    selecting the rows first."""
    from ubpl_amd import losses as L
    gen = torch.Generator().manual_seed(3)
    f1 = torch.randn(8, 2, 16, 32, 32, generator=gen)
    f2 = 0.3 * f1 + torch.randn(8, 2, 16, 32, 32, generator=gen)
    mask = torch.tensor([0, 0, 1, 0, 1, 1, 0, 1.0])
    a, b = f1.to(DEV).requires_grad_(True), f2.to(DEV).requires_grad_(True)
    v, c = L.features_cov(a, b, mask.to(DEV))
    v.backward()
    sel = mask > 0
    ra, rb = f1[sel].clone().requires_grad_(True), f2[sel].clone().requires_grad_(True)
    rv, rn = OL.features_cov(ra, rb)
    rv.backward()
    _close(v, rv, rtol=1e-5)
    assert int(c.item()) == rn
    _close(a.grad.cpu()[sel], ra.grad, rtol=1e-4, atol=1e-9)
    assert float(a.grad.cpu()[~sel].abs().max()) == 0.0


# ----------------------------------------------------------------- D1-D4
def test_decode_bit_exact():
    from ubpl_amd.process import ProcessUtils
    from ubpl_amd.evaluation import get_preds
    g = _npz("decode.npz")
    for name, cfg in seeds.decode_cases().items():
        hm, center, scale = seeds.decode_inputs(**cfg)
        raw = get_preds(hm.to(DEV)).cpu()
        assert np.array_equal(raw.numpy(), g[name + "/raw"]), name
        preds, scores = ProcessUtils.kps_fromHeatmap(hm, center, scale, [cfg["R"], cfg["R"]])
        assert np.array_equal(preds.numpy(), g[name + "/preds"]), name
        assert np.array_equal(scores.numpy(), g[name + "/scores"]), name


def test_decode_large_vs_oracle():
    from ubpl_amd.process import ProcessUtils
    gen = torch.Generator().manual_seed(9)
    hm = torch.randn(32, 16, 64, 64, generator=gen)
    hm[:, :, 10, 20] = 3.0
    hm[:, :, 30, 5] = 3.0     # tie: row-major first wins (10,20)
    hm[3] = -1.0
    center = torch.tensor([[128, 128]] * 32)
    scale = torch.full((32,), 1.28)
    p, s = ProcessUtils.kps_fromHeatmap(hm.to(DEV), center, scale, [64, 64])
    rp, rs_ = OD.kps_from_heatmap(hm, center, scale, [64, 64])
    assert np.array_equal(p.cpu().numpy(), rp.numpy())
    assert np.array_equal(s.cpu().numpy(), rs_.numpy())


def test_pck_vs_golden():
    from ubpl_amd.evaluation import EvaluationUtils
    g = _npz("decode.npz")
    for name, cfg in seeds.pck_cases().items():
        preds, gts = seeds.pck_inputs(**cfg)
        errs, accs = EvaluationUtils.acc_pck(preds.to(DEV), gts.to(DEV), cfg["ref"], cfg["thr"])
        _close(errs, g[name + "/errs"], rtol=1e-6)
        assert np.array_equal(accs.cpu().numpy(), g[name + "/accs"]), name


# ----------------------------------------------------------------- E1 + AdamW
def test_ema_bit_exact():
    from ubpl_amd import kernels as Kn
    g = _npz("ema.npz")
    for epo in [0, 1, 5, 2000]:
        ema, cur = seeds.ema_inputs()
        alpha = min(1 - 1 / (epo + 1), 0.999)
        for i, (e, c) in enumerate(zip(ema, cur)):
            ed = e.reshape(-1).to(DEV).contiguous()
            Kn.ema_update_(ed, c.reshape(-1).to(DEV).contiguous(), alpha)
            ref = g["ema/epo%d/%d" % (epo, i)].reshape(-1)
            got = ed.cpu().numpy()
            assert np.max(np.abs(got - ref) / (np.abs(ref) + 1e-30)) <= 1.2e-7, (epo, i)


def test_adamw_matches_torch():
    from ubpl_amd import kernels as Kn
    gen = torch.Generator().manual_seed(4)
    n = 10007
    p0 = torch.randn(n, generator=gen)
    ref = p0.clone().requires_grad_(True)
    opt = torch.optim.AdamW([ref], lr=2.5e-4, weight_decay=0.01)
    p, m, v = p0.clone().to(DEV), torch.zeros(n, device=DEV), torch.zeros(n, device=DEV)
    for step in range(1, 6):
        gr = torch.randn(n, generator=gen)
        ref.grad = gr.clone()
        opt.step()
        Kn.adamw_step_(p, gr.to(DEV), m, v, 2.5e-4, 0.9, 0.999, 1e-8, 0.01, step)
    _close(p, ref, rtol=1e-6, atol=1e-7)


# ----------------------------------------------------------------- BN / pool
def test_bn_forward_backward_vs_torch():
    from ubpl_amd import kernels as Kn
    gen = torch.Generator().manual_seed(2)
    for (B, C, H) in [(4, 64, 32), (3, 128, 4), (2, 256, 2)]:
        x = torch.randn(B, C, H, H, generator=gen) * 3 + 5
        gam = torch.rand(C, generator=gen) + 0.5
        bet = torch.randn(C, generator=gen)
        rm, rv = torch.randn(C, generator=gen), torch.rand(C, generator=gen) + 0.5
        dz = torch.randn(B, C, H, H, generator=gen)
        # reference: relu(bn(x)) train mode
        xr = x.clone().requires_grad_(True)
        gr, br = gam.clone().requires_grad_(True), bet.clone().requires_grad_(True)
        rmr, rvr = rm.clone(), rv.clone()
        y = F.relu(F.batch_norm(xr, rmr, rvr, gr, br, True, 0.1, 1e-5))
        y.backward(dz)
        xd = x.to(DEV)
        part = Kn.bn_part(B, C, DEV)
        mean, istd, sc, sh = [torch.empty(C, device=DEV) for _ in range(4)]
        rmd, rvd = rm.to(DEV), rv.to(DEV)
        Kn.bn_forward_stats(xd, gam.to(DEV), bet.to(DEV), 1e-5, 0.1, rmd, rvd, part, mean, istd, sc, sh)
        yd = Kn.bn_apply(xd, sc, sh, relu=1)
        _close(yd, y, rtol=1e-5, atol=1e-5)
        _close(rmd, rmr, rtol=1e-6, atol=1e-6)
        _close(rvd, rvr, rtol=1e-5, atol=1e-6)
        dg, db = torch.zeros(C, device=DEV), torch.zeros(C, device=DEV)
        coef = torch.empty(3 * C, device=DEV)
        dx = Kn.bn_backward(dz.to(DEV).clone(), xd, gam.to(DEV), mean, istd, sc, sh, 1, part, coef, dg, db)
        _close(dx, xr.grad, rtol=1e-4, atol=1e-5)
        _close(dg, gr.grad, rtol=1e-4, atol=1e-4)
        _close(db, br.grad, rtol=1e-4, atol=1e-4)


def test_pool_upsample_vs_torch():
    from ubpl_amd import kernels as Kn
    gen = torch.Generator().manual_seed(8)
    x = torch.randn(2, 8, 16, 16, generator=gen)
    x[0, 0, 0, :2] = 1.5      # tie inside a window: first max gets the gradient
    dy = torch.randn(2, 8, 8, 8, generator=gen)
    xr = x.clone().requires_grad_(True)
    y = F.max_pool2d(xr, 2, 2)
    y.backward(dy)
    xd = x.to(DEV)
    _close(Kn.maxpool2x2(xd), y, rtol=0, atol=0)
    dx = torch.zeros_like(xd)
    Kn.maxpool2x2_backward(xd, dy.to(DEV), dx, accumulate=False)
    _close(dx, xr.grad, rtol=0, atol=0)
    xr = x.clone().requires_grad_(True)
    y = F.avg_pool2d(xr, 2, 2)
    y.backward(dy)
    _close(Kn.avgpool2x2(xd), y, rtol=1e-7, atol=1e-7)
    dx = torch.zeros_like(xd)
    Kn.avgpool2x2_backward(dy.to(DEV), dx, accumulate=False)
    _close(dx, xr.grad, rtol=1e-7, atol=1e-7)
    up = torch.randn(2, 8, 16, 16, generator=gen)
    low = torch.randn(2, 8, 8, 8, generator=gen).requires_grad_(True)
    out = up + F.interpolate(low, scale_factor=2, mode="nearest")
    dout = torch.randn(2, 8, 16, 16, generator=gen)
    out.backward(dout)
    _close(Kn.upsample2x_add(up.to(DEV), low.detach().to(DEV)), out, rtol=0, atol=0)
    ud = up.to(DEV)                                   # in place (out aliases up), float4 path
    Kn.upsample2x_add(ud, low.detach().to(DEV), out=ud)
    _close(ud, out, rtol=0, atol=0)
    u6, l3 = torch.randn(2, 3, 6, 6, generator=gen), torch.randn(2, 3, 3, 3, generator=gen)   # W % 4 != 0
    _close(Kn.upsample2x_add(u6.to(DEV), l3.to(DEV)), u6 + F.interpolate(l3, scale_factor=2, mode="nearest"),
           rtol=0, atol=0)
    dl = torch.zeros(2, 8, 8, 8, device=DEV)
    Kn.upsample2x_add_backward(dout.to(DEV), dl, accumulate=False)
    _close(dl, low.grad, rtol=1e-6, atol=1e-6)


# ----------------------------------------------------------------- conv
CONV_CASES = [
    # B, Cin, H, Cout, KS, stride, prologue, residual
    (2, 256, 64, 128, 1, 1, True, False),
    (2, 128, 64, 256, 1, 1, True, True),
    (3, 128, 16, 128, 3, 1, True, False),
    (2, 64, 128, 64, 3, 1, True, True),
    (4, 256, 4, 16, 1, 1, False, False),     # heads: Cout 16
    (2, 17, 8, 256, 1, 1, False, True),      # merge_preds: Cin 17
    (2, 3, 64, 64, 7, 2, False, False),      # stem
    (1, 256, 2, 256, 3, 1, True, True),      # tiny spatial
    (8, 128, 32, 128, 3, 1, True, False),    # split-K in every pass
    (2, 64, 6, 32, 3, 1, True, False),       # Wo % 4 != 0: scalar wgrad path
    (3, 32, 5, 48, 1, 1, True, True),        # P % 4 != 0: scalar wgrad path
]


def test_conv_wgrad_misaligned_dy():
    """dy at a 4-byte (not 16-byte) offset takes the scalar weight-gradient path."""
    from ubpl_amd import kernels as Kn
    gen = torch.Generator().manual_seed(5)
    x = torch.randn(2, 64, 16, 16, generator=gen)
    dy = torch.randn(2, 64, 16, 16, generator=gen)
    w = torch.zeros(64, 64, 3, 3, requires_grad=True)
    F.conv2d(x, w, None, 1, 1).backward(dy)
    buf = torch.empty(dy.numel() + 1, device=DEV)
    dyd = buf[1:].view_as(dy)
    dyd.copy_(dy.to(DEV))
    dw, db = torch.zeros(64, 64, 3, 3, device=DEV), torch.zeros(64, device=DEV)
    Kn.conv2d_wgrad(dyd, x.to(DEV), 3, 1, dw, db, accumulate=False)
    _close(dw, w.grad, rtol=1e-4, atol=1e-5 * float(w.grad.abs().max()))
    _close(db, dy.sum((0, 2, 3)), rtol=1e-4, atol=1e-4)


@pytest.mark.parametrize("case", CONV_CASES)
def test_conv_fwd_dgrad_wgrad_vs_torch(case):
    from ubpl_amd import kernels as Kn
    B, Cin, H, Cout, KS, st, pro, resid = case
    gen = torch.Generator().manual_seed(hash(case) % 1000)
    x = torch.randn(B, Cin, H, H, generator=gen)
    w = torch.randn(Cout, Cin, KS, KS, generator=gen) / np.sqrt(Cin * KS * KS)
    b = torch.randn(Cout, generator=gen)
    sc = torch.rand(Cin, generator=gen) + 0.5
    sh = torch.randn(Cin, generator=gen) * 0.5
    xr = x.clone().requires_grad_(True)
    wr, br = w.clone().requires_grad_(True), b.clone().requires_grad_(True)
    inp = F.relu(xr * sc[None, :, None, None] + sh[None, :, None, None]) if pro else xr
    y = F.conv2d(inp, wr, br, st, (KS - 1) // 2)
    Ho = y.shape[-1]
    res = torch.randn(B, Cout, Ho, Ho, generator=gen) if resid else None
    yref = y + res if resid else y
    dy = torch.randn(B, Cout, Ho, Ho, generator=gen)
    yref.backward(dy)
    xd, wd, bd = x.to(DEV), w.to(DEV), b.to(DEV)
    scd, shd = (sc.to(DEV), sh.to(DEV)) if pro else (None, None)
    yd = Kn.conv2d_forward(xd, wd, bd, st, scd, shd, res=res.to(DEV) if resid else None)
    # exact-f32 MFMA chains vs MKL: elementwise within 1e-4 relative, or 1e-5 of
    # the tensor's scale for elements near a cancellation to ~0
    sc_ = lambda t: 1e-5 * float(t.detach().abs().max())
    _close(yd, yref, rtol=1e-4, atol=sc_(yref))
    dw, db = torch.zeros_like(wd), torch.zeros_like(bd)
    Kn.conv2d_wgrad(dy.to(DEV), xd, KS, st, dw, db, scd, shd, accumulate=True)
    _close(dw, wr.grad, rtol=1e-4, atol=sc_(wr.grad))
    _close(db, br.grad, rtol=1e-4, atol=sc_(br.grad))
    if st == 1:
        # dgrad w.r.t. the conv input (after the prologue)
        inp_r = inp.detach().clone().requires_grad_(True)
        F.conv2d(inp_r, w, b, st, (KS - 1) // 2).backward(dy)
        dx = Kn.conv2d_dgrad(dy.to(DEV), wd)
        _close(dx, inp_r.grad, rtol=1e-4, atol=sc_(inp_r.grad))


@pytest.mark.parametrize("case", [
    (2, 256, 16, 128, True, False), (2, 128, 16, 256, True, True), (3, 64, 32, 128, False, False),
    (2, 256, 4, 256, True, True), (2, 16, 8, 256, False, True), (2, 256, 8, 16, False, False)])
def test_conv1x1_dma_vs_torch(case):
    """LDS-DMA 1x1 kernel (k-major weights): forward with prologue / residual
    (also aliasing the output) and the data gradient (weights as they lie)."""
    from ubpl_amd import kernels as Kn
    B, Cin, H, Cout, pro, resid = case
    gen = torch.Generator().manual_seed(31 + hash(case) % 1000)
    x = torch.randn(B, Cin, H, H, generator=gen)
    w = torch.randn(Cout, Cin, 1, 1, generator=gen) / np.sqrt(Cin)
    b = torch.randn(Cout, generator=gen)
    sc, sh = torch.rand(Cin, generator=gen) + 0.5, torch.randn(Cin, generator=gen) * 0.5
    res = torch.randn(B, Cout, H, H, generator=gen)
    inp = F.relu(x * sc[None, :, None, None] + sh[None, :, None, None]) if pro else x
    yref = F.conv2d(inp, w, b) + (res if resid else 0)
    d = lambda t: t.to(DEV)
    wk = Kn.conv_weight_flip(d(w))
    ps, ph = (d(sc), d(sh)) if pro else (None, None)
    y = Kn.conv1x1_forward_kmajor(d(x), wk, d(b), ps, ph, res=d(res) if resid else None)
    sc_ = lambda t: 1e-5 * float(t.abs().max())
    _close(y, yref, rtol=1e-4, atol=sc_(yref))
    if resid:
        r2 = d(res)
        y2 = Kn.conv1x1_forward_kmajor(d(x), wk, d(b), ps, ph, res=r2, out=r2)
        _close(y2, yref, rtol=1e-4, atol=sc_(yref))
    dy = torch.randn(B, Cout, H, H, generator=gen)
    dxref = torch.nn.grad.conv2d_input(x.shape, w, dy)
    dx = Kn.conv1x1_forward_kmajor(d(dy), d(w), None)
    _close(dx, dxref, rtol=1e-4, atol=sc_(dxref))


@pytest.mark.parametrize("case", [(4, 128, 32, 128, 1), (32, 256, 4, 128, 1), (2, 128, 64, 128, 3),
                                  (4, 128, 8, 128, 3)])
def test_conv_epilogue_bn_partials(case):
    """BatchNorm statistics from the partials the conv epilogue writes (and the
    split-K fallback pass) equal the statistics of the conv output."""
    from ubpl_amd import kernels as Kn
    B, Cin, H, Cout, KS = case
    gen = torch.Generator().manual_seed(7 + hash(case) % 1000)
    x = torch.randn(B, Cin, H, H, generator=gen).to(DEV)
    w = (torch.randn(Cout, Cin, KS, KS, generator=gen) / np.sqrt(Cin * KS * KS)).to(DEV)
    b = (torch.randn(Cout, generator=gen) * 3).to(DEV)
    gamma, beta = torch.rand(Cout, device=DEV) + 0.5, torch.randn(Cout, device=DEV)
    part = Kn.bn_partial_buffer(Cout, B * H * H, DEV)
    if KS == 1:
        y = Kn.conv1x1_forward_kmajor(x, Kn.conv_weight_flip(w), b, stat_part=part)
    else:
        xs = Kn.split_activation(x, 3, 1)
        y = Kn.conv2d_forward_psa(xs, Kn.conv_weight_split(w, 0, 3), b, stat_part=part)
    rm, rv = torch.zeros(Cout, device=DEV), torch.ones(Cout, device=DEV)
    mu, istd, sc, sh = (torch.empty(Cout, device=DEV) for _ in range(4))
    Kn.bn_stats_from_partials(part, Cout, B * H * H, gamma, beta, 1e-5, 0.1, rm, rv, mu, istd, sc, sh)
    yd = y.double().cpu()
    m_ref = yd.mean((0, 2, 3))
    v_ref = yd.var((0, 2, 3), unbiased=False)
    _close(mu, m_ref, rtol=1e-6, atol=1e-6)
    _close(istd, 1.0 / torch.sqrt(v_ref + 1e-5), rtol=1e-5, atol=0)
    _close(rv, 0.9 + 0.1 * yd.var((0, 2, 3), unbiased=True), rtol=1e-5, atol=0)


@pytest.mark.parametrize("kind", ["maxpool", "upsample"])
@pytest.mark.parametrize("shape", [(4, 128, 16, 16), (3, 64, 32, 32), (2, 256, 8, 8)])
def test_pool_stats_partials(kind, shape):
    """The max-pool / upsample-add outputs are bit-identical with and without
    the BatchNorm partials, and the statistics from those partials equal the
    output's own (the residual bn1 that reads them, hourglass.py residual)."""
    from ubpl_amd import kernels as Kn
    B, C, H, W = shape
    gen = torch.Generator().manual_seed(3)
    x = (torch.randn(B, C, 2 * H, 2 * W, generator=gen) * 2 + 1).to(DEV)
    up = (torch.randn(B, C, H, W, generator=gen) + 3).to(DEV)
    low = torch.randn(B, C, H // 2, W // 2, generator=gen).to(DEV)
    part = Kn.bn_partial_buffer(C, B * H * W, DEV)
    if kind == "maxpool":
        y0 = Kn.maxpool2x2(x)
        y = Kn.maxpool2x2(x, stat_part=part)
    else:
        y0 = Kn.upsample2x_add(up, low)
        y = Kn.upsample2x_add(up.clone(), low, stat_part=part)
    assert torch.equal(y, y0)
    gamma, beta = torch.rand(C, device=DEV) + 0.5, torch.randn(C, device=DEV)
    rm, rv = torch.zeros(C, device=DEV), torch.ones(C, device=DEV)
    mu, istd, sc, sh = (torch.empty(C, device=DEV) for _ in range(4))
    Kn.bn_stats_from_partials(part, C, B * H * W, gamma, beta, 1e-5, 0.1, rm, rv, mu, istd, sc, sh)
    yd = y.double().cpu()
    _close(mu, yd.mean((0, 2, 3)), rtol=1e-6, atol=1e-6)
    _close(istd, 1.0 / torch.sqrt(yd.var((0, 2, 3), unbiased=False) + 1e-5), rtol=1e-5, atol=0)

"""Pin the oracle (CPU restatement) against the reference's own outputs.

The fixtures in tests/golden/ were produced by running the reference code
(tests/golden/gen_golden.py); these tests prove the restatement in oracle/
reproduces them, so the oracle can stand in for the reference on the GPU box.
"""
import json
import os

import numpy as np
import pytest
import torch

import seeds
from oracle import decode as D
from oracle import hourglass as H
from oracle import losses as L
from oracle import render as R
from oracle import schedule as S
from oracle import step as T

GD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def _npz(name):
    return np.load(os.path.join(GD, name))


def _close(a, b, rtol=1e-5, atol=1e-7):
    np.testing.assert_allclose(np.asarray(a, np.float64), np.asarray(b, np.float64), rtol=rtol, atol=atol)


# ---------------------------------------------------------------- R1
def test_render_bit_exact():
    g = _npz("render.npz")
    for name, (kps, shape, inp, out) in seeds.render_cases().items():
        hm, ka = R.render_one(kps, (shape[1], shape[2]), inp, out)
        assert np.array_equal(hm, g[name + "/hm"]), name
        assert np.array_equal(ka, g[name + "/kps_after"]), name
    c = seeds.render_cases()
    for i, key in enumerate(["mixed16", "edges16"]):
        hm, ka = R.render_one(c[key][0], (256, 256), 256, 64)
        assert np.array_equal(hm, g["mul/hm%d" % i])
        assert np.array_equal(ka, g["mul/kps%d" % i])


# ---------------------------------------------------------------- L1-L7
def _g(fn, *ts):
    ts = [t.clone().requires_grad_(True) for t in ts]
    r = fn(*ts)
    r[0].backward()
    return r, [t.grad.numpy() for t in ts]


def _sub(a, R_):
    return a if R_ <= 16 else a[..., ::4, ::4]


@pytest.mark.parametrize("case", list(seeds.loss_cases().keys()))
def test_losses(case):
    g = _npz("losses.npz")
    cfg = seeds.loss_cases()[case]
    d = seeds.loss_inputs(**cfg)
    S_, Rr = cfg["S"], cfg["R"]
    (s, n), (dp,) = _g(lambda p: L.joint_mse(p, d["gts"], S_, d["gate"], d["sw_lab"], True, True), d["preds"])
    _close(s.item(), g[case + "/mse_sum"]); assert n == g[case + "/mse_n"]
    _close(_sub(dp, Rr), g[case + "/mse_dp"], atol=1e-9)
    (s, n), (dp,) = _g(lambda p: L.joint_mse(p, d["gts"], S_), d["preds"])
    _close(s.item(), g[case + "/mse0_sum"]); assert n == g[case + "/mse0_n"]
    _close(_sub(dp, Rr), g[case + "/mse0_dp"], atol=1e-9)
    last = d["preds"][:, -1].contiguous()
    (s, n), (dp,) = _g(lambda p: L.joint_dist(p, d["tlast"][0]), last)
    _close(s.item(), g[case + "/dist_sum"]); assert n == g[case + "/dist_n"]
    _close(_sub(dp, Rr), g[case + "/dist_dp"], atol=1e-9)
    (s, n, nps, nsel, sc), (dp,) = _g(
        lambda p: L.joint_dist_mt2(p, d["tlast"][0], sw=d["sw_cons"], use_sw=True, thr=cfg["thr"]), last)
    _close(s.item(), g[case + "/mt2_sum"]); assert n == g[case + "/mt2_n"]
    assert nps == g[case + "/mt2_npse"] and nsel == g[case + "/mt2_nsel"]
    _close(sc.detach().numpy(), g[case + "/mt2_score"])
    _close(_sub(dp, Rr), g[case + "/mt2_dp"], atol=1e-9)
    if cfg.get("pseudo", True):
        (s, n, nsel, sc, _, _), (dp,) = _g(
            lambda p: L.joint_pseudo3(p, d["teachers"], d["sw_nega"], S_, cfg["thr"]), d["preds"])
        _close(s.item(), g[case + "/ps_sum"]); assert n == g[case + "/ps_n"]
        assert nsel == g[case + "/ps_nsel"]
        _close(sc.detach().numpy(), g[case + "/ps_score"])
        _close(_sub(dp, Rr), g[case + "/ps_dp"], atol=1e-9)
    else:
        with pytest.raises(RuntimeError):
            L.joint_pseudo3(d["preds"], d["teachers"], d["sw_nega"], S_, cfg["thr"])
        assert g["alllab/ps_raises"] == 1
    (s, n), (g1, g2) = _g(L.joint_feature_dist, d["f1"], d["f2"])
    _close(s.item(), g[case + "/fdist_sum"]); assert n == g[case + "/fdist_n"]
    _close(g1, g[case + "/fdist_g1"], atol=1e-7); _close(g2, g[case + "/fdist_g2"], atol=1e-7)
    (s, n), (g1, g2) = _g(L.features_cov, d["f1"], d["f2"])
    _close(s.item(), g[case + "/cov_val"]); assert n == g[case + "/cov_n"]
    _close(g1, g[case + "/cov_g1"], atol=1e-7); _close(g2, g[case + "/cov_g2"], atol=1e-7)
    isl = d["islabeled"]
    assert np.array_equal(L.sample_weight(isl).numpy(), g[case + "/w"])
    assert np.array_equal(L.sample_weight_nega(isl, cfg["pw"]).numpy(), g[case + "/w_nega"])
    assert np.array_equal(L.sample_weight(isl).numpy(), g[case + "/w_mt"])
    assert np.array_equal(L.sample_weight_nega(isl, cfg["pw"]).numpy(), g[case + "/w_mt_nega"])
    assert np.array_equal(L.sample_weight_cons(isl, cfg["pw"]).numpy(), g[case + "/w_mt_cons"])


# ---------------------------------------------------------------- D1-D4
def test_decode_bit_exact():
    g = _npz("decode.npz")
    for name, cfg in seeds.decode_cases().items():
        hm, center, scale = seeds.decode_inputs(**cfg)
        assert np.array_equal(D.get_preds(hm).numpy(), g[name + "/raw"]), name
        preds, scores = D.kps_from_heatmap(hm, center, scale, [cfg["R"], cfg["R"]])
        assert np.array_equal(preds.numpy(), g[name + "/preds"]), name
        assert np.array_equal(scores.numpy(), g[name + "/scores"]), name


def test_pck():
    g = _npz("decode.npz")
    for name, cfg in seeds.pck_cases().items():
        preds, gts = seeds.pck_inputs(**cfg)
        errs, accs = D.acc_pck(preds, gts, cfg["ref"], cfg["thr"])
        _close(errs.numpy(), g[name + "/errs"], rtol=1e-6)
        assert np.array_equal(accs.numpy(), g[name + "/accs"]), name


# ---------------------------------------------------------------- E1 E2 S1
def test_ema_bit_exact():
    g = _npz("ema.npz")
    for epo in [0, 1, 5, 2000]:
        ema, cur = seeds.ema_inputs()
        S.ema_update(ema, cur, epo, 0.999)
        for i, t in enumerate(ema):
            assert np.array_equal(t.numpy(), g["ema/epo%d/%d" % (epo, i)]), (epo, i)


def test_ramps_and_sampler():
    m = json.load(open(os.path.join(GD, "misc.json")))
    for e in range(40):
        assert S.value_increase(e, 10.0, 0.0, 5) == m["ramps"]["cons/%d" % e]
        assert S.value_increase(e, 1.0, 1.0, 100) == m["ramps"]["pseudo/%d" % e]
        assert S.value_decrease(e, 1.0, 0.2, 30) == m["ramps"]["fdl_dec/%d" % e]
        assert S.value_increase(e, 1.0, 0.2, 30) == m["ramps"]["fdl_inc/%d" % e]
    for name, (prim, sec, bs, sbs, seed) in seeds.sampler_cases().items():
        np.random.seed(seed)
        batches = S.two_stream_batches(prim, sec, bs, sbs)
        assert len(batches) == m["sampler"][name]["len"]
        assert [[int(i) for i in b] for b in batches] == m["sampler"][name]["batches"]


# ---------------------------------------------------------------- H1
def _stats(t):
    v = t.detach().double()
    return [v.sum().item(), (v * v).sum().item()]


@pytest.mark.parametrize("case", list(seeds.hg_cases().keys()))
def test_hourglass(case):
    g = _npz("hourglass.npz")
    meta = json.load(open(os.path.join(GD, "hourglass_meta.json")))[case]
    cfg = seeds.hg_cases()[case]
    torch.manual_seed(cfg["seed"])
    m = H.OracleHourglass(cfg["K"], cfg["S"], cfg["mode"]).requires_grad_(True)
    assert [n for n, _ in m.named_parameters()] == meta["param_names"]
    # bit-identical default init
    assert np.array_equal(np.array([_stats(p) for p in m.parameters()]), g[case + "/param_stats"])
    x, gp, gf = seeds.hg_inputs(**cfg)
    res = m(x)
    preds, feats = (res, None) if cfg["mode"] == "default" else res
    sub = cfg["sub"]
    _close(preds.detach().numpy()[:, :, :, ::sub, ::sub], g[case + "/preds"], rtol=1e-4, atol=1e-5)
    _close(_stats(preds), g[case + "/preds_sum"], rtol=1e-4)
    loss = (preds * gp).sum()
    if feats is not None:
        _close(_stats(feats), g[case + "/feats_sum"], rtol=1e-4)
        loss = loss + (feats * gf).sum()
    loss.backward()
    gst = np.array([[0.0, 0.0, 0.0] if p.grad is None else _stats(p.grad) + [1.0] for p in m.parameters()])
    ref = g[case + "/grad_stats"]
    assert np.array_equal(gst[:, 2], ref[:, 2])
    _close(gst[:, 1], ref[:, 1], rtol=2e-3, atol=1e-12)
    bst = np.array([_stats(b) for _, b in m.named_buffers()])
    _close(bst, g[case + "/buf_stats_after_train_fwd"], rtol=1e-4, atol=1e-6)
    m.eval()
    with torch.no_grad():
        res = m(x)
    preds = res if cfg["mode"] == "default" else res[0]
    _close(_stats(preds), g[case + "/eval_preds_sum"], rtol=1e-4)


# ---------------------------------------------------------------- T1
# the B=32 headline step takes ~2 min of CPU: pinned here only with UBPL_SLOW=1 (passed in
# rounds 5 and 6).  The GPU suite checks the HIP step at B=32 against the reference's own
# fixtures (tests/golden/steps.npz / steps64.npz records, test_gpu_train.py), not the oracle.
_STEP_CASES = [pytest.param(c, marks=pytest.mark.skipif(seeds.step_cases()[c]["B"] > 8 and
                                                        os.environ.get("UBPL_SLOW") != "1",
                                                        reason="slow CPU case (UBPL_SLOW=1)"))
               for c in seeds.step_cases()]


@pytest.mark.parametrize("case", _STEP_CASES)
def test_train_step(case):
    g = _npz("steps.npz")
    cfg = seeds.step_cases()[case]
    torch.set_num_threads(min(8, os.cpu_count() or 1))
    models, emas, optims = seeds.step_models(H.oracle_factory, cfg)
    before = [[p.detach().clone() for p in m.parameters()] for m in models + emas]
    loader, args = seeds.step_batch(cfg, R.kps_heatmap_torch)
    grads = {}

    def on_grads(ms):
        for mi, m in enumerate(ms):
            grads[mi] = seeds.grad_record([(n, p.grad) for n, p in m.named_parameters()])
    fn = {"MT_UBPL": T.train_mt_ubpl, "DualPose_UBPL": T.train_dualpose_ubpl}.get(cfg["project"])
    if fn is not None:
        rec, counts = fn(loader, models, emas, optims, args, on_grads=on_grads)
    elif cfg["project"] == "MT":
        rec, counts = T.train_mt(loader, models[0], emas[0], optims[0], args, on_grads=on_grads)
    else:
        rec, counts = T.train_supervised(loader, models[0], optims[0], args, on_grads=on_grads)
    # the students' gradients as the reference's optimizer saw them (gen_golden.py step pre-hook):
    # per-parameter norm within 1e-5, sampled elements within 1e-4 of the parameter's largest sample
    for mi, (st, sa) in grads.items():
        rs, ra = g[case + "/model%d/grad_stats" % mi], g[case + "/model%d/grad_samp" % mi]
        names = [n for n, _ in models[mi].named_parameters()]
        nz = [i for i, n in enumerate(names) if rs[i, 1] > 0 and not seeds.bn_cancelled(n)]
        assert np.array_equal(st[:, 1] > 0, rs[:, 1] > 0), mi
        rn, on = np.sqrt(rs[nz, 1]), np.sqrt(st[nz, 1])
        assert (np.abs(on - rn) <= 1e-5 * rn).all(), (mi, names[nz[int(np.argmax(np.abs(on - rn) / rn))]])
        scale = np.nanmax(np.abs(ra[nz]), axis=1)
        dev = np.nanmax(np.abs(sa[nz] - ra[nz]), axis=1)
        assert (dev <= 1e-4 * scale).all(), (mi, names[nz[int(np.argmax(dev / scale))]])
    flat = []

    def fl(x):
        if isinstance(x, (list, tuple)):
            for v in x:
                fl(v)
        else:
            flat.append(float(x))
    fl(rec)
    _close(flat, g[case + "/records"], rtol=2e-4, atol=1e-9)
    assert np.array_equal(np.array(counts, np.int64).reshape(-1, 2), g[case + "/printed_counts"])
    for mi, (m, b0) in enumerate(zip(models + emas, before)):
        upd = np.array([((p.detach().double() - q.double()) / args.lr).sum().item()
                        for p, q in zip(m.parameters(), b0)])
        ref = g[case + "/model%d/upd" % mi]
        absu = g[case + "/model%d/absupd" % mi]
        # AdamW's first step moves each weight by ~lr*sign(g): allow a few sign
        # flips of near-zero gradients per tensor (each flip moves the sum by 2).
        names = [n for n, _ in m.named_parameters()]
        noisy = np.array([seeds.bn_cancelled(n) for n in names])
        bad = (np.abs(upd - ref) > 1e-3 * absu + 6.0) & ~noisy
        assert not bad.any(), (mi, [names[i] for i in np.nonzero(bad)[0]])
        bst = np.array([_stats(b) for _, b in m.named_buffers()])
        _close(bst, g[case + "/model%d/buf" % mi], rtol=1e-3, atol=1e-6)

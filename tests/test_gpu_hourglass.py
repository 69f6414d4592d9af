"""Stacked hourglass on the HIP path vs the reference (H1-H6).

Parity criteria (and why):
* init, parameter/buffer names and order: bit-exact against the reference's
  golden statistics (seeded default init);
* forward heatmaps at a realistic batch (B=4, 256x256, 2 stacks): relative
  L2 error <= 1e-4 against the reference's fp32 result (BASELINE north star);
* the golden tiny-batch fixtures (B=1-2, down to 2x2 BatchNorm planes) are
  ill-conditioned: the reference's OWN fp32 output is up to 5% from the exact
  (fp64) result there.  For them, and for every gradient (deep train-mode BN
  backward cancels heavily: the reference's fp32 parameter gradients sit
  ~2% from exact even at B=8), the criterion is "no further from the exact
  result than the reference's fp32 is": err(ours, fp64) <= 3 * err(ref32,
  fp64) + 1e-4.  The fp64 result is the oracle restatement run in float64.
Conv biases with an exactly-zero gradient (seeds.bn_cancelled) are noise in
every implementation and are skipped in gradient comparisons.
"""
import json
import os

import numpy as np
import pytest
import torch

import seeds
from oracle import hourglass as OH

pytestmark = pytest.mark.gpu
GD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
DEV = "cuda"


def _stats(t):
    v = t.detach().double().cpu()
    return [v.sum().item(), (v * v).sum().item()]


def _rel(a, b):
    a = a.detach().double().cpu() if torch.is_tensor(a) else torch.as_tensor(np.asarray(a, np.float64))
    b = b.detach().double().cpu() if torch.is_tensor(b) else torch.as_tensor(np.asarray(b, np.float64))
    return float((a - b).norm() / (b.norm() + 1e-30))


def _oracles(K, S, mode, seed):
    """fp32 oracle (the reference's arithmetic) and its fp64 twin, same weights."""
    torch.manual_seed(seed)
    m32 = OH.OracleHourglass(K, S, mode).requires_grad_(True)
    p64 = {k: v.detach().double().requires_grad_(True) for k, v in m32.P.items()}
    m64 = OH.OracleHourglass(K, S, mode, params=p64)
    for k in list(m64.buf):
        if m64.buf[k].is_floating_point():
            m64.buf[k] = m64.buf[k].double()
    return m32, m64


def _run(model, x, gp, gf, mode, dtype=None):
    xx = x if dtype is None else x.to(dtype)
    r = model(xx)
    p, f = (r, None) if mode == "default" else r
    loss = (p * (gp if dtype is None else gp.to(dtype))).sum()
    if f is not None:
        loss = loss + (f * (gf if dtype is None else gf.to(dtype))).sum()
    loss.backward()
    return p, f


def _check_grads(ours, m32, m64, names):
    bad = []
    for n in names:
        if seeds.bn_cancelled(n):
            continue
        g32, g64 = m32.P[n].grad, m64.P[n].grad
        go = ours[n]
        if g64 is None:
            assert go is None or float(go.abs().max()) == 0.0, n
            continue
        e_ref = _rel(g32, g64)
        e_our = _rel(go, g64)
        if e_our > 3 * e_ref + 1e-4:
            bad.append((n, e_our, e_ref))
    assert not bad, bad[:8]


def _our_grads(model):
    return {n: (None if p.grad is None else p.grad.detach().cpu()) for n, p in model.named_parameters()}


@pytest.mark.parametrize("case", [pytest.param(c, marks=pytest.mark.timeout(600)) if c == "hg8_384" else c
                                  for c in seeds.hg_cases()])
def test_hourglass_vs_golden(case):
    from ubpl_amd.hourglass import StackedHourglass
    g = np.load(os.path.join(GD, "hourglass.npz"))
    meta = json.load(open(os.path.join(GD, "hourglass_meta.json")))[case]
    cfg = seeds.hg_cases()[case]
    torch.manual_seed(cfg["seed"])
    m = StackedHourglass(cfg["K"], cfg["S"], cfg["mode"])
    names = [n for n, _ in m.named_parameters()]
    assert names == meta["param_names"]
    assert [n for n, _ in m.named_buffers()] == meta["buffer_names"]
    assert np.array_equal(np.array([_stats(p) for p in m.parameters()]), g[case + "/param_stats"])
    x, gp, gf = seeds.hg_inputs(**cfg)
    m.train()
    p, f = _run(m, x.to(DEV), gp.to(DEV), gf.to(DEV), cfg["mode"])
    m32, m64 = _oracles(cfg["K"], cfg["S"], cfg["mode"], cfg["seed"])
    p32, _ = _run(m32, x, gp, gf, cfg["mode"])
    p64, _ = _run(m64, x, gp, gf, cfg["mode"], torch.float64)
    sub = cfg["sub"]
    e_ref, e_our = _rel(p32, p64), _rel(p, p64)
    # the fp32 oracle on THIS host reproduces the reference's golden output to
    # within the same fp32 noise floor (other CPUs round differently)
    assert _rel(p32[:, :, :, ::sub, ::sub], g[case + "/preds"]) <= 3 * e_ref + 1e-6
    assert e_our <= 3 * e_ref + 1e-4, (e_our, e_ref)
    _check_grads(_our_grads(m), m32, m64, names)
    # running statistics after one train-mode forward
    bst = np.array([_stats(b) for _, b in m.named_buffers()])
    ref = g[case + "/buf_stats_after_train_fwd"]
    assert np.array_equal(bst[2::3], ref[2::3])                       # num_batches_tracked
    # eval mode uses the running statistics (same noise-floor criterion)
    m.eval()
    m32.eval()
    m64.eval()
    with torch.no_grad():
        r = m(x.to(DEV))
        r32, r64 = m32(x), m64(x.double())
    pick = (lambda v: v) if cfg["mode"] == "default" else (lambda v: v[0])
    pe, pe32, pe64 = pick(r), pick(r32), pick(r64)
    e_ref = _rel(pe32, pe64)
    assert _rel(pe32[:, :, :, ::sub, ::sub], g[case + "/eval_preds"]) <= 3 * e_ref + 1e-6
    assert _rel(pe, pe64) <= 3 * e_ref + 1e-4


def test_hourglass_b4_256_vs_oracle():
    """Well-conditioned: 2 stacks, B=4, 256x256, AvgPool features."""
    from ubpl_amd.hourglass import StackedHourglass
    K, S, mode, B = 16, 2, "AvgPool", 4
    torch.manual_seed(1388)
    m = StackedHourglass(K, S, mode)
    gen = torch.Generator().manual_seed(5)
    x = torch.rand(B, 3, 256, 256, generator=gen) - 0.45
    gp = torch.randn(B, S, K, 64, 64, generator=gen)
    gf = torch.randn(B, S, 256, 32, 32, generator=gen)
    p, f = _run(m, x.to(DEV), gp.to(DEV), gf.to(DEV), mode)
    m32, m64 = _oracles(K, S, mode, 1388)
    p32, f32 = _run(m32, x, gp, gf, mode)
    p64, f64 = _run(m64, x, gp, gf, mode, torch.float64)
    assert _rel(p, p32) < 1e-4, _rel(p, p32)
    assert _rel(f, f32) < 1e-4, _rel(f, f32)
    for s in range(S):
        assert _rel(p[:, s], p32[:, s]) < 1e-4
    _check_grads(_our_grads(m), m32, m64, [n for n, _ in m.named_parameters()])
    # running stats (train-mode BN momentum update) vs the oracle
    for n, b in m.named_buffers():
        if n.endswith("num_batches_tracked"):
            continue
        assert _rel(b, m32.buf[n]) < 1e-4, n


def test_state_dict_roundtrip_and_flat_alias():
    from ubpl_amd.hourglass import StackedHourglass
    torch.manual_seed(0)
    m = StackedHourglass(16, 2, "AvgPool")
    sd = {k: v.clone() for k, v in m.state_dict().items()}
    assert len([k for k in sd if not k.endswith(("running_mean", "running_var", "num_batches_tracked"))]) == 454
    assert sum(p.numel() for p in m.parameters()) == 8429088
    p = dict(m.named_parameters())["preds.1.conv.bias"]
    p.data.add_(1.0)
    s, n, _ = m._offs["preds.1.conv.bias"]
    assert torch.equal(m.flat_params[s:s + n], p.data.reshape(-1))
    m2 = StackedHourglass(16, 2, "AvgPool")
    m2.load_state_dict(sd)
    assert torch.equal(m2.state_dict()["preds.0.conv.weight"], sd["preds.0.conv.weight"])
    assert torch.equal(dict(m2.named_parameters())["preds.1.conv.bias"].data, sd["preds.1.conv.bias"])


def _fit(prec, K, S, B, R, steps, seed=2024):
    """`steps` AdamW steps of a fresh seeded hourglass on one fixed batch
    (JointMSELoss-style heatmap MSE to random Gaussian-blob targets); returns
    the loss after each step."""
    from ubpl_amd.hourglass import StackedHourglass
    from ubpl_amd.optim import FlatAdamW
    torch.manual_seed(seed)
    m = StackedHourglass(K, S, "AvgPool")
    m.set_conv_precision(prec)
    opt = FlatAdamW(m, lr=2.5e-4, weight_decay=0.0)
    gen = torch.Generator().manual_seed(seed + 1)
    x = (torch.rand(B, 3, R, R, generator=gen) - 0.45).to(DEV)
    r = R // 4
    yy, xx = torch.meshgrid(torch.arange(r).float(), torch.arange(r).float(), indexing="ij")
    cy, cx = torch.randint(4, r - 4, (2, B, K), generator=gen).float()
    tgt = torch.exp(-((yy - cy[..., None, None]) ** 2 + (xx - cx[..., None, None]) ** 2) / 8.0).to(DEV)
    losses = []
    for _ in range(steps):
        opt.zero_grad()
        p, _ = m(x)
        loss = ((p - tgt[:, None]) ** 2).mean()
        loss.backward()
        opt.step()
        losses.append(float(loss))
    return losses


@pytest.mark.timeout(600)
@pytest.mark.parametrize("S,R,B", [(2, 256, 4), (8, 384, 2)])
def test_bf16_precision_trains_like_fp32(S, R, B):
    """The "bf16" conv precision (BASELINE config 5's throughput path: one bf16
    piece per operand, f32 accumulation).  Each kernel on it is pinned exactly
    against bf16-rounded operands in test_gpu_split.py (rel <= 2e-6); at the
    network level a randomly initialised hourglass in train-mode BatchNorm
    amplifies any perturbation ~1e3x (rounding only the WEIGHTS to bf16 moves
    the stack-1 heatmaps by ~25 %, tools/bf16_drift.py), so heatmaps cannot be
    compared element-wise.  The bar is the training signal: fitting one fixed
    batch, the bf16 run's loss curve must follow the fp32-equivalent (6xbf16)
    run's — every step within 5 % of the initial loss and the loss falling as
    much (within 10 %).  The per-step bar is relative to the initial loss, not
    to the current one: two builds of the 6xbf16 path that differ only in
    summation order (round 3: f64 split-K slab sums, residual added after the
    K loop) already end 12 steps apart by 7 % of the final loss (S=2:
    0.0362 vs 0.0338), so a bar on the late, small losses measures the
    trajectory's chaos, not the precision."""
    K = 16
    l6 = _fit("6xbf16", K, S, B, R, 12)
    l1 = _fit("bf16", K, S, B, R, 12)
    print("S=%d R=%d 6xbf16 %s\n          bf16   %s" % (S, R, ["%.5f" % v for v in l6], ["%.5f" % v for v in l1]))
    assert all(np.isfinite(l1))
    assert l1 != l6                                   # the bf16 kernels really ran
    for a, b in zip(l1, l6):
        assert abs(a - b) <= 0.05 * l6[0], (l1, l6)
    assert (l6[0] - l6[-1]) > 0 and abs((l1[0] - l1[-1]) - (l6[0] - l6[-1])) <= 0.1 * (l6[0] - l6[-1])



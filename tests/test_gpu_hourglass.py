"""Stacked hourglass on the HIP path vs the reference's golden outputs (H1-H6).

Weights come from the same seeded default init as the reference (checked
bit-exact); forward outputs are compared as whole-tensor relative L2 error
and elementwise within the north-star 1e-4 (relative) with a small absolute
floor; parameter gradients as per-tensor L2 norms.  Conv biases whose exact
gradient is zero (tests/golden/seeds.py:bn_cancelled) carry only rounding
noise and are checked for magnitude only.
"""
import json
import os

import numpy as np
import pytest
import torch

import seeds

pytestmark = pytest.mark.gpu
GD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
DEV = "cuda"


def _stats(t):
    v = t.detach().double().cpu()
    return [v.sum().item(), (v * v).sum().item()]


def _rel_l2(a, b):
    a = np.asarray(a, np.float64)
    b = np.asarray(b, np.float64)
    return float(np.linalg.norm(a - b) / (np.linalg.norm(b) + 1e-30))


@pytest.mark.parametrize("case", list(seeds.hg_cases().keys()))
def test_hourglass_vs_golden(case):
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
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
    res = m(x.to(DEV))
    preds, feats = (res, None) if cfg["mode"] == "default" else res
    sub = cfg["sub"]
    p_sub = preds.detach().cpu().numpy()[:, :, :, ::sub, ::sub]
    ref = g[case + "/preds"]
    assert _rel_l2(p_sub, ref) < 1e-4, _rel_l2(p_sub, ref)
    np.testing.assert_allclose(p_sub, ref, rtol=1e-4, atol=2e-4 * np.abs(ref).max())
    np.testing.assert_allclose(_stats(preds), g[case + "/preds_sum"], rtol=1e-4)
    loss = (preds * gp.to(DEV)).sum()
    if feats is not None:
        np.testing.assert_allclose(_stats(feats), g[case + "/feats_sum"], rtol=1e-4)
        loss = loss + (feats * gf.to(DEV)).sum()
    loss.backward()
    ref_g = g[case + "/grad_stats"]
    for i, (n, p) in enumerate(m.named_parameters()):
        if ref_g[i, 2] == 0:
            assert p.grad is None, n
            continue
        got = (p.grad.double().cpu() ** 2).sum().item()
        if seeds.bn_cancelled(n):
            continue
        assert abs(np.sqrt(got) - np.sqrt(ref_g[i, 1])) <= 1e-3 * np.sqrt(ref_g[i, 1]) + 1e-6, (n, got, ref_g[i, 1])
    bst = np.array([_stats(b) for _, b in m.named_buffers()])
    np.testing.assert_allclose(bst, g[case + "/buf_stats_after_train_fwd"], rtol=1e-4, atol=1e-5)
    m.eval()
    with torch.no_grad():
        r = m(x.to(DEV))
    pe = r if cfg["mode"] == "default" else r[0]
    np.testing.assert_allclose(_stats(pe), g[case + "/eval_preds_sum"], rtol=1e-4)
    e_sub = pe.cpu().numpy()[:, :, :, ::sub, ::sub]
    assert _rel_l2(e_sub, g[case + "/eval_preds"]) < 1e-4


def test_state_dict_roundtrip_and_flat_alias():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from ubpl_amd.hourglass import StackedHourglass
    torch.manual_seed(0)
    m = StackedHourglass(16, 2, "AvgPool")
    sd = m.state_dict()
    assert len([k for k in sd if not k.endswith(("running_mean", "running_var", "num_batches_tracked"))]) == 454
    n_params = sum(p.numel() for p in m.parameters())
    assert n_params == 8429088
    # parameters alias the flat buffer: an in-place update is visible in both
    p = dict(m.named_parameters())["preds.1.conv.bias"]
    p.data.add_(1.0)
    s, n, _ = m._offs["preds.1.conv.bias"]
    assert torch.equal(m.flat_params[s:s + n], p.data.reshape(-1))
    m2 = StackedHourglass(16, 2, "AvgPool")
    m2.load_state_dict(sd)
    assert torch.equal(m2.flat_params[:m2.n_live], m.flat_params[:m.n_live])

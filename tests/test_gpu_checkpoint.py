"""f2 — checkpoint interchange (projects/MT_UBPL.py:97-103, utils/base/comm.py:92-103).

FlatAdamW (one fused HIP AdamW over the flat parameter buffer) against
torch.optim.AdamW over the oracle hourglass (reference parameter order) fed
the same gradients: parameters after 3 steps, the state_dicts (keys, moments,
step, param_groups) and a resume in both directions (torch state into
FlatAdamW, FlatAdamW state into torch AdamW) followed by one more step.
Tolerance: fp32 elementwise arithmetic in a different operation order,
rtol 1e-5 / atol 1e-6.
"""
import os

import pytest
import torch

from oracle import hourglass as OH

pytestmark = pytest.mark.gpu
TOL = dict(rtol=1e-5, atol=1e-6)


def _pair(lr=1e-3, wd=0.01):
    from ubpl_amd.hourglass import StackedHourglass
    from ubpl_amd.optim import FlatAdamW
    torch.manual_seed(0)
    model = StackedHourglass(16, 1, "default")
    ref = _oracle_copy(model)
    return model, FlatAdamW(model, lr=lr, weight_decay=wd), ref, torch.optim.AdamW(ref.parameters(), lr=lr,
                                                                                     weight_decay=wd)


def _oracle_copy(model):
    params = {n: p.detach().cpu().clone() for n, p in model.named_parameters()}
    return OH.OracleHourglass(model.k, model.nStack, model.mode, params=params).requires_grad_(True)


def _live(model):
    return [n for n, _ in model.named_parameters() if model._offs[n][0] < model.n_live]


def _step(model, opt, ref, ropt, g):
    grads = {n: torch.randn(model.P(n).shape, generator=g) for n in _live(model)}
    model.flat_grads.zero_()
    for n, gr in grads.items():
        model.G(n).copy_(gr)
    opt.step()
    ropt.zero_grad(set_to_none=True)
    rp = dict(ref.named_parameters())
    for n, gr in grads.items():
        rp[n].grad = gr.clone()
    ropt.step()


def _same_params(model, ref):
    rp = dict(ref.named_parameters())
    for n, p in model.named_parameters():
        torch.testing.assert_close(p.detach().cpu(), rp[n].detach(), **TOL)


def test_flat_adamw_matches_torch_adamw_and_state_layout():
    model, opt, ref, ropt = _pair()
    g = torch.Generator().manual_seed(1)
    assert opt.state_dict()["state"] == {}            # torch keeps no state before the first step
    for _ in range(3):
        _step(model, opt, ref, ropt, g)
    torch.cuda.synchronize()
    _same_params(model, ref)
    sd, rsd = opt.state_dict(), ropt.state_dict()
    assert sd["param_groups"] == rsd["param_groups"]
    assert sorted(sd["state"]) == sorted(rsd["state"])   # live params only (dead skip_layer: no grad, no state)
    for i, e in rsd["state"].items():
        assert float(sd["state"][i]["step"]) == float(e["step"]) == 3.0
        torch.testing.assert_close(sd["state"][i]["exp_avg"].cpu(), e["exp_avg"], **TOL)
        torch.testing.assert_close(sd["state"][i]["exp_avg_sq"].cpu(), e["exp_avg_sq"], **TOL)


def test_resume_both_directions(tmp_path):
    from ubpl_amd.hourglass import StackedHourglass
    from ubpl_amd.optim import FlatAdamW
    from ubpl_amd import checkpoint as CK
    model, opt, ref, ropt = _pair()
    g = torch.Generator().manual_seed(2)
    for _ in range(2):
        _step(model, opt, ref, ropt, g)
    torch.cuda.synchronize()
    # torch AdamW state (a reference checkpoint's optim state) -> a fresh FlatAdamW
    m2 = StackedHourglass(16, 1, "default")
    m2.load_state_dict(model.state_dict())
    o2 = FlatAdamW(m2, lr=0.5, weight_decay=0.0)
    o2.load_state_dict(ropt.state_dict())
    assert o2.step_count == 2 and o2.param_groups[0]["lr"] == 1e-3 and o2.param_groups[0]["weight_decay"] == 0.01
    # FlatAdamW state -> a fresh torch AdamW over the oracle model
    ref2 = _oracle_copy(model)
    r2 = torch.optim.AdamW(ref2.parameters(), lr=0.5)
    r2.load_state_dict(opt.state_dict())
    # one more step on both resumed pairs with the same gradients
    g3 = torch.Generator().manual_seed(3)
    _step(m2, o2, ref2, r2, g3)
    torch.cuda.synchronize()
    _same_params(m2, ref2)
    # whole-checkpoint round trip in the reference's schema (weights_only load)
    args = type("A", (), {})()
    args.best_acc, args.best_epoch = [0.1, 0.2, 0.3], [0, 0, 0]
    assert CK.select_best([[0.0, 0.5], [0.0, 0.1], [0.0, 0.4]], args, 4) == [True, False, True]
    ck = CK.checkpoint_state([m2], [model], [o2], args, 4)
    assert set(ck) == {"current_epoch", "best_acc", "best_epoch", "model1_state", "model1_ema_state", "optim1_state"}
    path = CK.save_checkpoint(ck, True, str(tmp_path))
    assert os.path.isfile(os.path.join(str(tmp_path), "checkpoint_best.pth.tar"))
    m3 = StackedHourglass(16, 1, "default")
    e3 = StackedHourglass(16, 1, "default")
    o3 = FlatAdamW(m3)
    epo, best_acc, best_epoch = CK.load_checkpoint(path, [m3], [e3], [o3], map_location="cpu")
    assert epo == 4 and best_acc == [0.5, 0.2, 0.4] and best_epoch == [4, 0, 4]
    assert torch.equal(m3.flat_params, m2.flat_params) and torch.equal(m3.flat_stats, m2.flat_stats)
    assert torch.equal(o3.exp_avg, o2.exp_avg) and o3.step_count == o2.step_count
    assert torch.equal(e3.state_dict()["hgs.0.0.up1.bn1.running_mean"],
                       model.state_dict()["hgs.0.0.up1.bn1.running_mean"])


def test_fused_adamw_ema_bit_identical_to_separate():
    """FlatAdamW.step_and_ema (one pass) == step() followed by
    update_ema_variables (utils/parameters.py:4-8), bit for bit, incl. the
    never-trained tail the EMA still blends."""
    import types
    from ubpl_amd.hourglass import StackedHourglass
    from ubpl_amd.optim import FlatAdamW
    from ubpl_amd.parameters import ema_alpha, update_ema_variables
    torch.manual_seed(0)
    sa, ta = StackedHourglass(16, 1, "AvgPool"), StackedHourglass(16, 1, "AvgPool")
    sb, tb = StackedHourglass(16, 1, "AvgPool"), StackedHourglass(16, 1, "AvgPool")
    sb.load_state_dict(sa.state_dict())
    tb.load_state_dict(ta.state_dict())
    oa, ob = FlatAdamW(sa, lr=1e-3, weight_decay=0.01), FlatAdamW(sb, lr=1e-3, weight_decay=0.01)
    g = torch.Generator(device="cuda").manual_seed(5)
    for epo in (1, 3):
        args = types.SimpleNamespace(epo=epo, ema_decay=0.999)
        gr = torch.randn(sa.n_total, device="cuda", generator=g)
        sa.flat_grads.copy_(gr)
        sb.flat_grads.copy_(gr)
        oa.step()
        update_ema_variables(sa, ta, args)
        ob.step_and_ema(tb, ema_alpha(epo, 0.999))
    torch.cuda.synchronize()
    assert torch.equal(sa.flat_params, sb.flat_params)
    assert torch.equal(ta.flat_params, tb.flat_params)
    assert torch.equal(oa.exp_avg, ob.exp_avg) and torch.equal(oa.exp_avg_sq, ob.exp_avg_sq)
    assert oa.step_count == ob.step_count == 2
    assert not torch.equal(ta.flat_params[sa.n_live:], sa.flat_params[sa.n_live:])   # tail blended, not copied

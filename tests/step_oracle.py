"""Full-tensor student gradients of the oracle's step (fp32 = the reference's
arithmetic, pinned by test_oracle_golden; fp64 = the exact result), taken just
before the optimizer step.  TEST INFRASTRUCTURE ONLY."""
import torch

import gen_oracle64 as G64
import seeds
from oracle import hourglass as H
from oracle import render as R
from oracle import step as T


def oracle_grads(cfg, f64):
    models, emas, optims = seeds.step_models(H.oracle_factory, cfg)
    if f64:
        for i, m in enumerate(models + emas):
            for k in m.P:
                m.P[k] = m.P[k].detach().double().requires_grad_(i < len(models))
            for k in m.buf:
                if m.buf[k].is_floating_point():
                    m.buf[k] = m.buf[k].double()
        optims = [torch.optim.AdamW(m.parameters(), lr=cfg["lr"], weight_decay=0) for m in models]
    loader, args = seeds.step_batch(cfg, R.kps_heatmap_torch)
    if f64:
        loader = [G64.to64(b) for b in loader]
    got = {}

    def hook(ms):
        for mi, m in enumerate(ms):
            got[mi] = {n: p.grad.detach().double().clone() for n, p in m.named_parameters() if p.grad is not None}
    if cfg["project"] == "MT_UBPL":
        T.train_mt_ubpl(loader, models, emas, optims, args, on_grads=hook)
    elif cfg["project"] == "DualPose_UBPL":
        T.train_dualpose_ubpl(loader, models, emas, optims, args, on_grads=hook)
    elif cfg["project"] == "MT":
        T.train_mt(loader, models[0], emas[0], optims[0], args, on_grads=hook)
    else:
        T.train_supervised(loader, models[0], optims[0], args, on_grads=hook)
    return got



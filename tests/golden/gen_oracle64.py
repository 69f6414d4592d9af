"""Float64 twin of every T1 step fixture: the noise floor of the step tests.

TEST INFRASTRUCTURE ONLY.  Runs the oracle's restatement of each project's
train() (oracle/step.py, pinned to the reference's own fp32 results by
tests/test_oracle_golden.py::test_train_step) in float64 on the same seeded
inputs as tests/golden/gen_golden.py, and stores the students' gradient
records (seeds.grad_record, taken just before the optimizer step) and the
loss records in tests/golden/steps64.npz.

The GPU step tests compare the HIP step against this exact result with the
criterion of tests/test_gpu_hourglass.py: no further from float64 than the
reference's own float32 result (steps.npz) is, plus 1e-4 relative.

Usage:  python tests/golden/gen_oracle64.py [case ...]
"""
import os
import sys

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path[:0] = [HERE, ROOT]
import seeds  # noqa: E402
from oracle import hourglass as H  # noqa: E402
from oracle import render as R  # noqa: E402
from oracle import step as T  # noqa: E402


def to64(x):
    if torch.is_tensor(x):
        return x.double() if x.is_floating_point() else x
    if isinstance(x, (list, tuple)):
        return type(x)(to64(v) for v in x)
    if isinstance(x, dict):
        return {k: to64(v) for k, v in x.items()}
    return x


def run_case(cfg):
    models, emas, _ = seeds.step_models(H.oracle_factory, cfg)
    for i, m in enumerate(models + emas):
        for k in m.P:
            m.P[k] = m.P[k].detach().double().requires_grad_(i < len(models))
        for k in m.buf:
            if m.buf[k].is_floating_point():
                m.buf[k] = m.buf[k].double()
    optims = [torch.optim.AdamW(m.parameters(), lr=cfg["lr"], weight_decay=0) for m in models]
    loader, args = seeds.step_batch(cfg, R.kps_heatmap_torch)
    loader = [to64(b) for b in loader]
    grads = {}

    def on_grads(ms):
        for mi, m in enumerate(ms):
            grads[mi] = seeds.grad_record([(n, p.grad) for n, p in m.named_parameters()])
    if cfg["project"] == "MT_UBPL":
        rec, _ = T.train_mt_ubpl(loader, models, emas, optims, args, on_grads=on_grads)
    elif cfg["project"] == "DualPose_UBPL":
        rec, _ = T.train_dualpose_ubpl(loader, models, emas, optims, args, on_grads=on_grads)
    elif cfg["project"] == "MT":
        rec, _ = T.train_mt(loader, models[0], emas[0], optims[0], args, on_grads=on_grads)
    else:
        rec, _ = T.train_supervised(loader, models[0], optims[0], args, on_grads=on_grads)
    return rec, grads


def _flatten(x):
    if isinstance(x, (list, tuple)):
        r = []
        for v in x:
            r.extend(_flatten(v))
        return r
    return [float(x)]


if __name__ == "__main__":
    torch.set_num_threads(os.cpu_count() or 8)
    path = os.path.join(HERE, "steps64.npz")
    out = dict(np.load(path)) if os.path.exists(path) else {}
    for cname in sys.argv[1:] or list(seeds.step_cases()):
        print("fp64 step", cname, flush=True)
        rec, grads = run_case(seeds.step_cases()[cname])
        out[cname + "/records"] = np.array(_flatten(rec), np.float64)
        for mi, (st, sa) in grads.items():
            out[cname + "/model%d/grad_stats" % mi] = st
            out[cname + "/model%d/grad_samp" % mi] = sa
        np.savez_compressed(path, **out)
    print("done")

"""Diagnostic: full-tensor relative L2 error of the HIP step's student
gradients against the oracle's float64 step, next to the oracle's float32
step (= the reference's arithmetic), per parameter.

    python tools/step_grad_diag.py CASE   (env selects the mode: UBPL_MODEL_STREAMS,
                                           UBPL_CONV_PRECISION, UBPL_SPLIT_BWD ...)
"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "ubpl-poseestimation_amd"), os.path.join(ROOT, "tests", "golden"),
                os.path.join(ROOT, "tests")]
import numpy as np  # noqa: E402
import pytest  # noqa: E402
import torch  # noqa: E402
import seeds  # noqa: E402
from step_oracle import oracle_grads  # noqa: E402
import test_gpu_train as TG  # noqa: E402


def main(case):
    torch.set_num_threads(min(16, os.cpu_count() or 1))
    mp = pytest.MonkeyPatch()
    cfg = seeds.step_cases()[case]
    from ubpl_amd import train as Tr
    models_ref = {}
    orig = Tr._step_and_ema

    def snap(models, *a, **k):
        torch.cuda.synchronize()
        for mi, m in enumerate(models):
            models_ref[mi] = {n: p.grad.detach().double().cpu().clone() for n, p in m.named_parameters()
                              if p.grad is not None}
        return orig(models, *a, **k)
    mp.setattr(Tr, "_step_and_ema", snap)
    TG._run_ours(cfg, True, mp)
    t = time.time()
    g32 = oracle_grads(cfg, False)
    g64 = oracle_grads(cfg, True)
    print("oracle %.1f s" % (time.time() - t))
    for mi in range(cfg["brNum"]):
        rows = []
        for n, gg in g64[mi].items():
            if seeds.bn_cancelled(n) or float(gg.norm()) == 0:
                continue
            eo = float((models_ref[mi][n] - gg).norm() / gg.norm())
            er = float((g32[mi][n] - gg).norm() / gg.norm())
            rows.append((eo, er, n))
        eo = np.array([r[0] for r in rows])
        er = np.array([r[1] for r in rows])
        print("%s model%d [%s]: relL2 ours median %.2e p95 %.2e max %.2e | ref32 median %.2e p95 %.2e max %.2e"
              " | >3x+1e-4: %d" % (case, mi, os.environ.get("MODE", ""), np.median(eo), np.percentile(eo, 95),
                                   eo.max(), np.median(er), np.percentile(er, 95), er.max(),
                                   int((eo > 3 * er + 1e-4).sum())))
        for r in sorted(rows, key=lambda r: -r[0] / (3 * r[1] + 1e-4))[:8]:
            print("    %-44s ours %.2e ref %.2e" % (r[2], r[0], r[1]))
    mp.undo()


if __name__ == "__main__":
    main(sys.argv[1])

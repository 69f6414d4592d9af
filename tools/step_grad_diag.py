"""Diagnostic: how far the HIP step's student gradients sit from the fp64
step (steps64.npz) vs the reference's fp32 step (steps.npz), per mode.

    python tools/step_grad_diag.py CASE   (env selects the mode: UBPL_MODEL_STREAMS,
                                           UBPL_CONV_PRECISION, UBPL_SPLIT_BWD ...)
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "ubpl-poseestimation_amd"), os.path.join(ROOT, "tests", "golden"),
                os.path.join(ROOT, "tests")]
import numpy as np  # noqa: E402
import pytest  # noqa: E402
import seeds  # noqa: E402
import test_gpu_train as TG  # noqa: E402


def main(case):
    mp = pytest.MonkeyPatch()
    cfg = seeds.step_cases()[case]
    g = np.load(os.path.join(ROOT, "tests/golden/steps.npz"))
    g64 = np.load(os.path.join(ROOT, "tests/golden/steps64.npz"))
    ours, before, rec, counts, args, grads = TG._run_ours(cfg, True, mp)
    names = [n for n, _ in ours[0].named_parameters()]
    for mi in range(cfg["brNum"]):
        st, sa = grads[mi]
        st32, st64 = g[case + "/model%d/grad_stats" % mi], g64[case + "/model%d/grad_stats" % mi]
        rows = []
        for i, n in enumerate(names):
            if st64[i, 1] <= 0 or seeds.bn_cancelled(n):
                continue
            n64 = np.sqrt(st64[i, 1])
            eo = abs(np.sqrt(st[i, 1]) - n64) / n64
            er = abs(np.sqrt(st32[i, 1]) - n64) / n64
            rows.append((eo, er, n))
        eo = np.array([r[0] for r in rows])
        er = np.array([r[1] for r in rows])
        worst = sorted(rows, key=lambda r: -(r[0] / (3 * r[1] + 1e-4)))[:5]
        print("%s model%d [%s]: norm err ours median %.2e max %.2e | ref32 median %.2e max %.2e | fails %d"
              % (case, mi, os.environ.get("MODE", ""), np.median(eo), eo.max(), np.median(er), er.max(),
                 int((eo > 3 * er + 1e-4).sum())))
        for r in worst:
            print("    %-40s ours %.2e ref %.2e" % (r[2], r[0], r[1]))
    mp.undo()


if __name__ == "__main__":
    main(sys.argv[1])

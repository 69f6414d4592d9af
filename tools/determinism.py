"""GPU-box: repeatability of the MT_UBPL step (tests/test_gpu_train.py case).

Runs 4 steps per configuration on fresh seeded models and prints, for pairs
of runs, the max |diff| of the students' / teachers' parameters, gradients
and BN statistics:  eager vs eager, graph vs graph, eager vs graph, with the
second-view backward on the teacher stream (split) and without.
"""
import contextlib
import io
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "tests", "golden"), os.path.join(ROOT, "tests"), os.path.join(ROOT, "ubpl-poseestimation_amd"), ROOT]

import torch  # noqa: E402

import seeds  # noqa: E402
from oracle import render as OR  # noqa: E402
from ubpl_amd import train as T  # noqa: E402
from ubpl_amd.hourglass import StackedHourglass  # noqa: E402
from ubpl_amd.optim import FlatAdamW  # noqa: E402


def run(graph, split, steps=4):
    os.environ["UBPL_STEP_GRAPH"] = "1" if graph else "0"
    T._SPLIT_BWD = split
    cfg = seeds.step_cases()["mt_ubpl"]
    models, emas, _ = seeds.step_models(lambda k, s, m: StackedHourglass(k, s, m), cfg, device="cuda")
    optims = [FlatAdamW(m, lr=cfg["lr"], weight_decay=0) for m in models]
    loader, args = seeds.step_batch(cfg, OR.kps_heatmap_torch)
    with contextlib.redirect_stdout(io.StringIO()):
        T.train_mt_ubpl(list(loader) * steps, models, emas, optims, args)
    torch.cuda.synchronize()
    return {"params": [m.flat_params.clone() for m in models + emas],
            "grads": [m.flat_grads.clone() for m in models],
            "stats": [m.flat_stats.clone() for m in models + emas]}


def cmp(tag, a, b):
    out = []
    for k in a:
        d = max(float((x - y).abs().max()) for x, y in zip(a[k], b[k]))
        out.append("%s=%.3g" % (k, d))
    print("%-28s %s" % (tag, "  ".join(out)), flush=True)


def poison(val, release=False):
    """Fill the caching allocator's free blocks with val (uninitialised reads then show)."""
    bufs = []
    for mb in (1, 2, 4, 8, 16, 32, 64, 128, 256):
        for _ in range(12):
            bufs.append(torch.full((mb * 262144,), val, device="cuda"))
    for n in (1000, 4096, 17000, 65536, 300000):
        for _ in range(40):
            bufs.append(torch.full((n,), val, device="cuda"))
    torch.cuda.synchronize()
    del bufs
    if release:
        torch.cuda.empty_cache()


def main():
    if len(sys.argv) > 2 and sys.argv[2] == "poison":
        e1 = run(False, True, 1)
        poison(float("nan"))
        e2 = run(False, True, 1)
        cmp("1 step eager clean/nan", e1, e2)
        poison(1e30)
        e3 = run(False, True, 1)
        cmp("1 step eager clean/1e30", e1, e3)
        poison(float("nan"), True)
        g = run(True, True, 4)
        poison(float("nan"))
        e4 = run(False, True, 4)
        cmp("4 steps eager/graph nan", e4, g)
        return
    steps = int(sys.argv[1]) if len(sys.argv) > 1 else 4
    e1, e2 = run(False, True, steps), run(False, True, steps)
    cmp("eager/eager split", e1, e2)
    g1, g2 = run(True, True, steps), run(True, True, steps)
    cmp("graph/graph split", g1, g2)
    cmp("eager/graph split", e1, g1)
    e0, g0 = run(False, False, steps), run(True, False, steps)
    cmp("eager/graph nosplit", e0, g0)
    cmp("eager split/nosplit", e1, e0)
    e1b = run(False, True, 1)
    e0b = run(False, False, 1)
    cmp("1 step split/nosplit", e1b, e0b)


if __name__ == "__main__":
    main()

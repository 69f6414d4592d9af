"""GPU-box: bit-repeatability of one eager MT_UBPL training step of a
tests/test_gpu_train.py case (default the B=32 headline case): the step is
run REPS times on freshly seeded models and every student gradient / updated
parameter / BN statistic is compared bit for bit with the first run.

    python tools/det_step.py [case] [reps]
"""
import contextlib
import io
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "tests", "golden"), os.path.join(ROOT, "tests"),
                os.path.join(ROOT, "ubpl-poseestimation_amd"), ROOT]

import torch  # noqa: E402

import seeds  # noqa: E402
from oracle import render as OR  # noqa: E402
from ubpl_amd import train as T  # noqa: E402
from ubpl_amd.hourglass import StackedHourglass  # noqa: E402
from ubpl_amd.optim import FlatAdamW  # noqa: E402


OUTS = []


def _record_forward():
    """Wrap StackedHourglass.forward: clone every network output on its stream."""
    orig = StackedHourglass.forward

    def fwd(self, imgs):
        r = orig(self, imgs)
        p = r[0] if isinstance(r, tuple) else r
        OUTS.append((self.tag, p.detach().clone()))
        return r
    StackedHourglass.forward = fwd


def run(case):
    cfg = seeds.step_cases()[case]
    OUTS.clear()
    models, emas, _ = seeds.step_models(lambda k, s, m: StackedHourglass(k, s, m), cfg, device="cuda")
    for i, m in enumerate(models):
        m.tag = "student%d" % i
    for i, m in enumerate(emas):
        m.tag = "teacher%d" % i
    optims = [FlatAdamW(m, lr=cfg["lr"], weight_decay=0) for m in models]
    loader, args = seeds.step_batch(cfg, OR.kps_heatmap_torch)
    grads = {}
    orig = T._step_and_ema

    def snap(*a, **k):
        torch.cuda.synchronize()
        grads["g"] = [m.flat_grads.clone() for m in models]
        return orig(*a, **k)
    T._step_and_ema = snap
    try:
        with contextlib.redirect_stdout(io.StringIO()):
            T.train_mt_ubpl(loader, models, emas, optims, args)
    finally:
        T._step_and_ema = orig
    torch.cuda.synchronize()
    names = [m.tag for m in models + emas]
    per_bn = {}
    for m in models + emas:
        for b in m._bn_names:
            rm, rv = m.stats(b)
            per_bn[(m.tag, b)] = torch.cat([rm, rv]).clone()
    return {"grads": grads["g"], "params": [m.flat_params.clone() for m in models + emas],
            "stats": [m.flat_stats.clone() for m in models + emas], "names": names, "bn": per_bn,
            "outs": list(OUTS)}


def poison(val):
    """DET_POISON=1: fill the caching allocator's free blocks with val before a run —
    a result that then changes read memory it never wrote (uninitialised or out of range)."""
    bufs = []
    free = torch.cuda.mem_get_info()[0]
    for mb in (1, 4, 16, 64, 256):
        for _ in range(8):
            if mb * 2 ** 20 * 8 < free:
                bufs.append(torch.full((mb * 262144,), val, device="cuda"))
    torch.cuda.synchronize()
    del bufs


def main():
    case = sys.argv[1] if len(sys.argv) > 1 else "mt_ubpl_b32"
    reps = int(sys.argv[2]) if len(sys.argv) > 2 else 4
    pz = os.environ.get("DET_POISON") == "1"
    _record_forward()
    if pz:
        poison(0.0)
    ref = run(case)
    bad = 0
    for r in range(1, reps):
        if pz:
            poison(float("nan") if r % 2 else 1e30)
        cur = run(case)
        d = {k: max(float((x - y).abs().max()) for x, y in zip(ref[k], cur[k])) for k in ("grads", "params", "stats")}
        bad += any(v != 0 for v in d.values())
        print("run %d vs 0: %s" % (r, "  ".join("%s=%.3g" % kv for kv in d.items())), flush=True)
        for (tag, a), (_, b) in zip(ref["outs"], cur["outs"]):
            print("   forward output %-9s max |d| %.3g" % (tag, float((a - b).abs().max())), flush=True)
        shown = 0
        for key, a in ref["bn"].items():
            dd = float((a - cur["bn"][key]).abs().max())
            if dd != 0 and shown < 6:
                print("   first differing BN running stats: %s %s (max |d| %.3g)" % (key[0], key[1], dd), flush=True)
                shown += 1
    print("det_step %s streams=%s: %d of %d repeats differ" % (
        case, os.environ.get("UBPL_MODEL_STREAMS", "1"), bad, reps - 1), flush=True)


if __name__ == "__main__":
    main()

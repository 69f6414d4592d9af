"""GPU-box race probe (round 4): forwards only.  NET train-mode hourglass
forwards (HG2, K=16, AvgPool, B=32, 256x256 — the headline step's networks),
VIEWS views each, every network on its own HIP stream as the training step
runs them (train._ModelStreams order: a network's views in sequence), repeated
REPS times on the SAME models and inputs: train-mode BatchNorm normalises with
the batch statistics, so every repeat must produce the same bits.  Prints, per
repeat, which (network, view) outputs differ from the first repeat.

    python tools/fwd_race.py [reps] [nets] [views]
    env: FWD_STREAMS=0 (all on the current stream), FWD_GRAD=1 (forwards that
         save for backward, as the students'), FWD_SYNC=1 (synchronize between
         networks: no overlap), FWD_KEEPALL=1 (every tensor an op allocates kept
         alive until the repeat ends: no memory block reused inside a repeat),
         =2 (kept for the whole run: no block ever reused), UBPL_RELAYOUT_ONCE=1
         (hourglass.py: the weight re-layouts only in each model's first forward)
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "ubpl-poseestimation_amd"), ROOT]

import torch  # noqa: E402


def main():
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 4
    nets = int(sys.argv[2]) if len(sys.argv) > 2 else 4
    views = int(sys.argv[3]) if len(sys.argv) > 3 else 2
    streams = os.environ.get("FWD_STREAMS", "1") != "0"
    grad = os.environ.get("FWD_GRAD", "0") == "1"
    sync = os.environ.get("FWD_SYNC", "0") == "1"
    from ubpl_amd import _lib
    from ubpl_amd.hourglass import StackedHourglass
    _lib.load()
    dev = torch.device("cuda", 0)
    torch.manual_seed(1388)
    models = [StackedHourglass(16, 2, "AvgPool") for _ in range(nets)]
    g = torch.Generator().manual_seed(7)
    imgs = [(torch.rand(32, 3, 256, 256, generator=g) - 0.49).to(dev) for _ in range(views)]
    side = [torch.cuda.Stream(device=dev) for _ in range(nets)]
    main_s = torch.cuda.current_stream(dev)

    keep_mode = os.environ.get("FWD_KEEPALL", "0")
    kept_all = []

    def once():
        from torch.utils._python_dispatch import TorchDispatchMode
        kept = kept_all if keep_mode == "2" else []

        class Keep(TorchDispatchMode):
            def __torch_dispatch__(self, func, types, args=(), kwargs=None):
                out = func(*args, **(kwargs or {}))
                kept.append(out)
                return out
        import contextlib
        with (Keep() if keep_mode in ("1", "2") else contextlib.nullcontext()):
            return _once()

    def _once():
        outs = [[None] * views for _ in range(nets)]
        for s in side:
            s.wait_stream(main_s)
        for n in range(nets):
            with torch.cuda.stream(side[n]) if streams else torch.cuda.stream(main_s):
                for v in range(views):
                    with torch.set_grad_enabled(grad):
                        o = models[n](imgs[v])[0]
                    outs[n][v] = o.detach().clone()
            if sync:
                torch.cuda.synchronize()
        for s in side:
            main_s.wait_stream(s)
        torch.cuda.synchronize()
        return outs

    ref = once()
    bad = 0
    for r in range(1, reps):
        cur = once()
        diff = [(n, v, float((a - b).abs().max())) for n in range(nets) for v in range(views)
                for a, b in [(ref[n][v], cur[n][v])] if not torch.equal(a, b)]
        bad += bool(diff)
        print("rep %d: %s" % (r, " ".join("net%d/v%d %.3g" % d for d in diff) or "identical"), flush=True)
    print("fwd_race nets=%d views=%d streams=%d grad=%d sync=%d keep=%s precision=%s: %d of %d repeats differ" % (
        nets, views, streams, grad, sync, keep_mode, os.environ.get("UBPL_CONV_PRECISION", "default"), bad,
        reps - 1), flush=True)


if __name__ == "__main__":
    main()

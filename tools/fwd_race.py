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
         (hourglass.py: the weight re-layouts only in each model's first forward),
         FWD_LOCATE=1 (forwards that save for backward; every saved activation of
         every (network, view) compared with the first repeat's, in execution
         order: names the first layer whose output differs)
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "ubpl-poseestimation_amd"), ROOT]

import torch  # noqa: E402


def analyse_add(r, n, v, k, up, low, out):
    """out should be up + nearest-upsample(low); name what the wrong elements hold instead."""
    lu = low.repeat_interleave(2, dim=2).repeat_interleave(2, dim=3)
    want = up + lu
    bad = (out != want).reshape(-1)
    nb = int(bad.sum())
    if nb == 0:
        return
    o, u, w, l2 = out.reshape(-1)[bad], up.reshape(-1)[bad], want.reshape(-1)[bad], lu.reshape(-1)[bad]
    idx = bad.nonzero().reshape(-1)
    # 4 floats per thread, 256 threads per block: block-sized chunks of the flat index
    blk = torch.unique(idx // 1024)
    print("   rep %d net%d/v%d %s: %d of %d wrong (%.2f%%); =up (add missing) %d, =up+2low (added twice) %d, "
          "=0 %d; flat index %d..%d, %d distinct 1024-element chunks (first %s)" % (
              r, n, v, k, nb, bad.numel(), 100.0 * nb / bad.numel(), int((o == u).sum()),
              int((o == u + 2 * l2).sum()), int((o == 0).sum()), int(idx[0]), int(idx[-1]), blk.numel(),
              blk[:6].tolist()), flush=True)


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
    locate = os.environ.get("FWD_LOCATE", "0") == "1"
    if locate:
        grad = True
        orig = StackedHourglass._forward_impl

        def fwd_impl(self, imgs, save):
            P, F, ex = orig(self, imgs, save)
            self._last_saved = [(k, v) for k, v in ex.saved.items()]
            return P, F, ex
        StackedHourglass._forward_impl = fwd_impl
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
                    if locate:
                        flat = []
                        for k, val in models[n]._last_saved:
                            for i, t in enumerate(val if isinstance(val, tuple) else (val,)):
                                flat.append(("%s[%d]" % (k, i), t.detach().clone()))
                        outs[n][v] = (outs[n][v], flat)
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
        if locate:
            for n in range(nets):
                for v in range(views):
                    shown = 0
                    cd = dict(cur[n][v][1])
                    for k, b in cur[n][v][1]:
                        if k.endswith(".add_out[0]") and k.replace(".add_out[0]", ".add_in[0]") in cd:
                            analyse_add(r, n, v, k, cd[k.replace(".add_out[0]", ".add_in[0]")],
                                        cd[k.replace(".add_out[0]", ".add_in[1]")], b)
                    for (k, a), (_, b) in zip(ref[n][v][1], cur[n][v][1]):
                        if not torch.equal(a, b):
                            print("   rep %d net%d/v%d %s differing saved tensor: %s %s max |d| %.3g" % (
                                r, n, v, "first" if not shown else "next", k, tuple(a.shape),
                                float((a - b).abs().max())), flush=True)
                            shown += 1
                            if shown >= int(os.environ.get("FWD_SHOW", "1")):
                                break
            strip = lambda o: [[x[0] for x in row] for row in o]
            rr, cc = strip(ref), strip(cur)
        else:
            rr, cc = ref, cur
        diff = [(n, v, float((a - b).abs().max())) for n in range(nets) for v in range(views)
                for a, b in [(rr[n][v], cc[n][v])] if not torch.equal(a, b)]
        bad += bool(diff)
        print("rep %d: %s" % (r, " ".join("net%d/v%d %.3g" % d for d in diff) or "identical"), flush=True)
    print("fwd_race nets=%d views=%d streams=%d grad=%d sync=%d keep=%s precision=%s: %d of %d repeats differ" % (
        nets, views, streams, grad, sync, keep_mode, os.environ.get("UBPL_CONV_PRECISION", "default"), bad,
        reps - 1), flush=True)


if __name__ == "__main__":
    main()

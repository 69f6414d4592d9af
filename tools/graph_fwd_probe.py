"""GPU-box: the ubpl hourglass forward (train-mode BatchNorm, no autograd) of
four independent networks, one per side stream, captured in one graph with
fork/join branches — every replay compared bit for bit with the eager run on
the same streams.  Isolates the forward kernels from the training step's
losses, backward and optimiser.

usage: python tools/graph_fwd_probe.py [replays] [B] [stacks] [same_stream] [eager|locate|trace]
(eager: no graph — the eager forward itself repeated and compared;
 locate: autograd forwards, and on a differing replay the first saved
 activation, in execution order, that differs is named;
 trace: every op's written tensors are snapshotted (cloned, in-stream) right
 after the op, in the eager reference and inside the graph; on a differing
 replay the first differing snapshots are named with their network)
"""
import contextlib
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "ubpl-poseestimation_amd"), ROOT]

import torch  # noqa: E402

from ubpl_amd.hourglass import StackedHourglass  # noqa: E402


class Snap:
    """Dispatch mode: after every op, clone each tensor it wrote (schema
    mutable args + outputs) on the current stream; records (net|op#|name, clone)."""

    def __init__(self, out, sid):
        self.out, self.sid = out, sid

    def __enter__(self):
        from torch.utils._python_dispatch import TorchDispatchMode
        out, sid = self.out, self.sid
        cnt = {}

        class M(TorchDispatchMode):
            def __torch_dispatch__(self, func, types, args=(), kwargs=None):
                r = func(*args, **(kwargs or {}))
                net = sid.get(torch.cuda.current_stream().cuda_stream, -1)
                cnt[net] = cnt.get(net, 0) + 1
                written = [a for sa, a in zip(func._schema.arguments, args)
                           if sa.alias_info is not None and sa.alias_info.is_write and torch.is_tensor(a)]
                rs = r if isinstance(r, (tuple, list)) else (r,)
                written += [t for t in rs if torch.is_tensor(t)]
                for j, t in enumerate(written):
                    if t.is_cuda and t.numel() > 0 and t.dtype in (torch.float32, torch.float64):
                        out.append(("net%d|op%d %s [%d]" % (net, cnt[net], func._schema.name, j), t.clone()))
                return r
        self.m = M()
        self.m.__enter__()
        return self

    def __exit__(self, *a):
        return self.m.__exit__(*a)


def flat_saved(ex, clone):
    """(name, tensor) of an executor's saved activations in execution order."""
    out = []
    for k, v in ex.saved.items():
        vs = v if isinstance(v, (tuple, list)) else (v,)
        for j, t in enumerate(vs):
            if torch.is_tensor(t):
                out.append(("%s[%d]" % (k, j), t.clone() if clone else t))
    return out


def main():
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 30
    B = int(sys.argv[2]) if len(sys.argv) > 2 else 4
    S = int(sys.argv[3]) if len(sys.argv) > 3 else 2
    one = len(sys.argv) > 4 and sys.argv[4] == "1"
    mode = sys.argv[5] if len(sys.argv) > 5 else ""
    eager = "eager" in mode              # "eager+locate": the eager forwards, first differing activation named
    locate = "locate" in mode
    trace = "trace" in mode
    anchor = [None]
    dev = torch.device("cuda")
    torch.manual_seed(0)
    nets = [StackedHourglass(16, S, "AvgPool").to(dev).train() for _ in range(4)]
    x = torch.rand(B, 3, 256, 256, device=dev)
    main_s = torch.cuda.Stream()
    side = [torch.cuda.Stream() for _ in range(4)]

    def work():
        for s in side:
            s.wait_stream(main_s)
        outs = []
        exs = []
        for i, m in enumerate(nets):
            with torch.cuda.stream(side[0 if one else i]):
                if locate:
                    p, f = m(x)
                    exs.append(p.grad_fn.ex)
                else:
                    with torch.no_grad():
                        p, f = m(x)
                outs.append(p)
                outs.append(f)
        anchor[0] = exs
        for s in side:
            main_s.wait_stream(s)
        return outs

    main_s.wait_stream(torch.cuda.current_stream())
    snaps_ref, snaps_g = [], []
    sid = {s.cuda_stream: i for i, s in enumerate(side)}
    with torch.cuda.stream(main_s):
        with (Snap(snaps_ref, sid) if trace else contextlib.nullcontext()):
            ref = [t.clone() for t in work()]
        ref_saved = [flat_saved(e, True) for e in anchor[0]] if locate else None
        work()
    torch.cuda.synchronize()
    if not eager:
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g, stream=main_s):
            with (Snap(snaps_g, sid) if trace else contextlib.nullcontext()):
                out = work()
    bad = 0
    for r in range(reps):
        if eager:
            with torch.cuda.stream(main_s):
                out = work()
        else:
            g.replay()
        torch.cuda.synchronize()
        ds = [float((a - b).abs().max()) for a, b in zip(out, ref)]
        if max(ds) != 0.0:
            bad += 1
            print("replay %d differs: %s" % (r, " ".join("%.3g" % d for d in ds)), flush=True)
            if trace:
                shown = {}
                for k, ((n1, a), (n2, b)) in enumerate(zip(snaps_ref, snaps_g)):
                    if a.shape != b.shape:
                        print("   snapshot lists diverge at %d: %s vs %s" % (k, n1, n2))
                        break
                    d = float((a - b).abs().max())
                    if d != 0.0 and shown.get(n1.split("|")[0], 0) < 3:
                        shown[n1.split("|")[0]] = shown.get(n1.split("|")[0], 0) + 1
                        print("   #%d %s  max |d| %.3g" % (k, n1, d), flush=True)
            if locate:
                for ni, (e, rs) in enumerate(zip(anchor[0], ref_saved)):
                    for (k, a), (_, b) in zip(flat_saved(e, False), rs):
                        d = float((a - b).abs().max())
                        if d != 0.0:
                            print("   net %d: first differing saved tensor %s (max |d| %.3g)" % (ni, k, d),
                                  flush=True)
                            break
    print("graph_fwd_probe B=%d S=%d %s %s precision=%s: %d of %d replays differ" %
          (B, S, "one side stream" if one else "4 side streams", "eager" if eager else "graph",
           os.environ.get("UBPL_CONV_PRECISION", "default"), bad, reps), flush=True)


if __name__ == "__main__":
    main()

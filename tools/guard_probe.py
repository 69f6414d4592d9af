"""GPU-box: out-of-bounds probe for every ubpl launch (graph-race hunt).

Every device-tensor argument of every C-ABI call (kernels.call) is moved into
a private copy with 64 KiB guard bands of 0xFF bytes (a NaN for f32 / bf16 /
f64) on both sides, the op runs on the copies, the guards are checked after a
synchronize, and the copies are written back.  A kernel that writes outside
its arguments' extents is named with the argument and the byte range it hit;
a kernel that READS outside and uses what it read propagates the NaN guards
into the results, which are compared with an unguarded run of the same pass.
Arguments that overlap are guarded as their union.

usage: python tools/guard_probe.py [B] [stacks] [mode] [res]
  (default 4 2 AvgPool 256: forward + backward of one StackedHourglass)
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "ubpl-poseestimation_amd"), ROOT]

import torch  # noqa: E402

from ubpl_amd import kernels as Kn  # noqa: E402
from ubpl_amd.hourglass import StackedHourglass  # noqa: E402

GUARD = 1 << 16
hits = []
ncalls = [0]


def guarded(real):
    def call(name, *args):
        ncalls[0] += 1
        ts = [(i, a) for i, a in enumerate(args) if torch.is_tensor(a) and a.is_cuda and a.numel() > 0]
        spans = []
        for i, a in ts:
            lo = a.data_ptr()
            # extent the kernel may legitimately touch: from data_ptr to the end of the view
            hi = lo + (sum((s - 1) * st for s, st in zip(a.shape, a.stride())) + 1) * a.element_size()
            spans.append([lo, hi, [i]])
        spans.sort()
        merged = []
        for s in spans:
            if merged and s[0] < merged[-1][1]:
                merged[-1][1] = max(merged[-1][1], s[1])
                merged[-1][2] += s[2]
            else:
                merged.append(s)
        new = list(args)
        keep = []
        for lo, hi, idx in merged:
            n = hi - lo
            mis = lo % 256
            buf = torch.full((GUARD + mis + n + GUARD,), 0xFF, dtype=torch.uint8, device=args[idx[0]].device)
            src = torch.empty(0, dtype=torch.uint8, device=buf.device)
            base = args[idx[0]]
            # raw byte view of the original span
            st = base.untyped_storage()
            off0 = lo - st.data_ptr()
            src.set_(st, off0, (n,), (1,))
            buf[GUARD + mis:GUARD + mis + n].copy_(src)
            for i in idx:
                a = args[i]
                o = GUARD + mis + (a.data_ptr() - lo)
                es = a.element_size()
                assert o % es == 0
                v = torch.empty(0, dtype=a.dtype, device=a.device)
                v.set_(buf.untyped_storage(), o // es, a.shape, a.stride())
                new[i] = v
            keep.append((lo, n, mis, idx, buf, src))
        real(name, *new)
        torch.cuda.synchronize()
        for lo, n, mis, idx, buf, src in keep:
            pre = buf[:GUARD + mis]
            post = buf[GUARD + mis + n:]
            bad_pre = (pre != 0xFF).nonzero()
            bad_post = (post != 0xFF).nonzero()
            if bad_pre.numel() or bad_post.numel():
                msg = "%s args %s (span %d B): " % (name, idx, n)
                if bad_pre.numel():
                    msg += "writes %d B BEFORE (from -%d)" % (bad_pre.numel(), GUARD + mis - int(bad_pre.min()))
                if bad_post.numel():
                    msg += " writes %d B AFTER (up to +%d)" % (bad_post.numel(), int(bad_post.max()) + 1)
                msg += " shapes %s" % [tuple(args[i].shape) for i in idx]
                hits.append(msg)
                print("OOB:", msg, flush=True)
            src.copy_(buf[GUARD + mis:GUARD + mis + n])
        torch.cuda.synchronize()
    return call


def run(B, S, mode, res, seed=0):
    torch.manual_seed(seed)
    dev = torch.device("cuda")
    m = StackedHourglass(16, S, mode).to(dev).train()
    x = torch.rand(B, 3, res, res, device=dev, generator=torch.Generator(dev).manual_seed(1))
    out = m(x)
    p, f = out if isinstance(out, tuple) else (out, None)
    loss = (p * p).sum() + ((f * f).sum() if f is not None else 0.0)
    loss.backward()
    torch.cuda.synchronize()
    return [p.detach().clone()] + ([f.detach().clone()] if f is not None else []) + [m.flat_grads.clone(),
                                                                                     m.flat_stats.clone()]


def main():
    B = int(sys.argv[1]) if len(sys.argv) > 1 else 4
    S = int(sys.argv[2]) if len(sys.argv) > 2 else 2
    mode = sys.argv[3] if len(sys.argv) > 3 else "AvgPool"
    res = int(sys.argv[4]) if len(sys.argv) > 4 else 256
    ref = run(B, S, mode, res)
    real = Kn.call
    Kn.call = guarded(real)
    try:
        got = run(B, S, mode, res)
    finally:
        Kn.call = real
    names = ["preds", "feats", "grads", "stats"] if len(ref) == 4 else ["preds", "grads", "stats"]
    for nm, a, b in zip(names, ref, got):
        nan = int(torch.isnan(b).sum())
        d = float((a - b).abs().nan_to_num(nan=float("inf")).max())
        print("%-5s max |guarded - plain| %.3g  NaNs %d" % (nm, d, nan), flush=True)
    print("guard_probe B=%d S=%d %s %d: %d launches, %d OOB writes" % (B, S, mode, res, ncalls[0], len(hits)),
          flush=True)


if __name__ == "__main__":
    main()

"""GPU-box: locate the first kernel whose output differs between repeats of
one eager MT_UBPL training step (tools/det_step.py runs the same step and only
says THAT it differs).  Every op's written tensors (outputs + mutated
arguments) get a checksum (float64 sum and abs-sum) computed in-stream right
after the op; the per-stream op sequences of each repeat are compared with the
first run and the first differing op of every stream is named, with the
checksums of the few ops before it.

    python tools/det_trace.py [case] [reps]
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "tools"), os.path.join(ROOT, "tests", "golden"), os.path.join(ROOT, "tests"),
                os.path.join(ROOT, "ubpl-poseestimation_amd"), ROOT]

import torch  # noqa: E402
from torch.utils._python_dispatch import TorchDispatchMode  # noqa: E402

import det_step  # noqa: E402
from ubpl_amd import train as T  # noqa: E402


class Sums(TorchDispatchMode):
    def __init__(self):
        super().__init__()
        self.rec = []          # (stream handle, op name, arg index, checksum tensor)

    def __torch_dispatch__(self, func, types, args=(), kwargs=None):
        name = func._schema.name
        if ONLY and not any(o in name for o in ONLY):
            return func(*args, **(kwargs or {}))
        st = torch.cuda.current_stream().cuda_stream
        if ONLY:
            # the selected ops' inputs too, checksummed before the op runs
            wr = [sa.alias_info is not None and sa.alias_info.is_write for sa in func._schema.arguments]
            for j, t in enumerate(args):
                if j < len(wr) and wr[j] and func._schema.arguments[j].name not in ("res",):
                    continue      # (output buffers: uninitialised before the op)
                if torch.is_tensor(t) and t.is_cuda and t.numel() > 0 and t.dtype == torch.float32:
                    with torch.no_grad():
                        c = torch.stack([t.sum(dtype=torch.float64), t.abs().sum(dtype=torch.float64)])
                    self.rec.append((st, name + " in", j, tuple(t.shape), c))
        r = func(*args, **(kwargs or {}))
        if name.startswith(("aten::sum", "aten::abs", "aten::stack", "aten::empty", "aten::new_empty")):
            return r          # (uninitialised allocations carry no result)
        written = [a for sa, a in zip(func._schema.arguments, args)
                   if sa.alias_info is not None and sa.alias_info.is_write and torch.is_tensor(a)]
        rs = r if isinstance(r, (tuple, list)) else (r,)
        # outputs that are views of an input (slice, view, ...) compute nothing
        written += [t for sr, t in zip(func._schema.returns, rs) if torch.is_tensor(t) and sr.alias_info is None]
        for j, t in enumerate(written):
            if t.is_cuda and t.numel() > 0 and t.dtype in (torch.float32, torch.float64):
                with torch.no_grad():
                    c = torch.stack([t.sum(dtype=torch.float64), t.abs().sum(dtype=torch.float64)])
                self.rec.append((st, name, j, tuple(t.shape), c))
        return r


# DET_OPS=a,b: checksum only ops whose name contains one of these (inputs and outputs), so the
# extra reductions perturb the step's timing less
ONLY = [o for o in os.environ.get("DET_OPS", "").split(",") if o]


def run(case):
    m = Sums()
    with m:
        final = det_step.run(case)
    torch.cuda.synchronize()
    out = {}
    for st, name, j, shp, c in m.rec:
        out.setdefault(st, []).append((name, j, shp, c.cpu().view(torch.int64).tolist(), c.cpu().tolist()))
    return out, final


def label(st):
    main = torch.cuda.current_stream().cuda_stream
    if st == main:
        return "main"
    for (M, _), ss in T._ModelStreams._cache.items():
        for i, s in enumerate(ss):
            if s.cuda_stream == st:
                return ("student%d" % i) if i < M else ("teacher%d" % (i - M))
    return "stream%x" % st


def main():
    case = sys.argv[1] if len(sys.argv) > 1 else "mt_ubpl_b32"
    reps = int(sys.argv[2]) if len(sys.argv) > 2 else 3
    det_step._record_forward()
    ref, rfin = run(case)
    print("ops per stream:", {label(k): len(v) for k, v in ref.items()}, flush=True)
    bad = 0
    for r in range(1, reps):
        cur, cfin = run(case)
        d = {k: max(float((x - y).abs().max()) for x, y in zip(rfin[k], cfin[k])) for k in ("grads", "params", "stats")}
        print("run %d final state vs run 0: %s" % (r, "  ".join("%s=%.3g" % kv for kv in d.items())), flush=True)
        diff = False
        for st, seq in ref.items():
            cs = cur.get(st, [])
            shown = 0
            for i, (a, b) in enumerate(zip(seq, cs)):
                if a[0] != b[0] or a[3] != b[3]:
                    diff = True
                    print("run %d: %-9s %s differing op #%d of %d: %s [%d] %s" % (
                        r, label(st), "first" if not shown else "next", i, len(seq), a[0], a[1], a[2]), flush=True)
                    lo = max(0, i - (6 if not shown else 0))
                    for k in range(lo, min(len(seq), i + 1)):
                        print("      #%d %s [%d] %s  ref %s  cur %s" % (k, seq[k][0], seq[k][1], seq[k][2],
                                                                    seq[k][4], cs[k][4] if k < len(cs) else None))
                    shown += 1
                    if not ONLY or shown >= 4:
                        break
            if len(seq) != len(cs):
                print("run %d: %s op count %d vs %d" % (r, label(st), len(seq), len(cs)), flush=True)
        bad += diff
    print("det_trace %s: %d of %d repeats differ" % (case, bad, reps - 1), flush=True)


if __name__ == "__main__":
    main()

"""GPU-box: read-before-write probe of one eager MT_UBPL training step
(VERDICT r3 item 1a).  Every fresh allocation is filled at allocation time
(torch.utils.deterministic.fill_uninitialized_memory: NaN for floats, the
type's maximum for integers — 0x7fff is a bf16 NaN, so a PSA image element
nothing wrote is NaN too).  After every op, in-stream, each tensor it wrote is
tested for NaN (float) / 0x7fff (int16); the first op of each stream whose
output carries one names a kernel that left part of its output unwritten or
read memory nothing wrote this step.  Nothing here depends on timing: the
fill happens at allocation, on the allocating stream.

    python tools/nan_probe.py [case]
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

SKIP = ("aten::empty", "aten::new_empty", "aten::empty_like", "aten::empty_strided", "aten::isnan",
        "aten::any", "aten::eq", "aten::view", "aten::_reshape_alias", "aten::as_strided", "aten::slice",
        "aten::select", "aten::detach", "aten::alias", "aten::t", "aten::transpose", "aten::expand",
        "aten::unsqueeze", "aten::squeeze", "aten::permute", "aten::split", "aten::unbind")


def _bad(t):
    if t.dtype in (torch.float32, torch.float64, torch.float16, torch.bfloat16):
        return torch.isnan(t).any()
    if t.dtype == torch.int16:
        return (t == 32767).any()
    return None


class Probe(TorchDispatchMode):
    def __init__(self):
        super().__init__()
        self.rec = []          # (stream, op, arg index, shape, device bool, inputs-bad device bool)

    def __torch_dispatch__(self, func, types, args=(), kwargs=None):
        name = func._schema.name
        if name.startswith(SKIP):
            return func(*args, **(kwargs or {}))
        st = torch.cuda.current_stream().cuda_stream
        sch = func._schema.arguments
        # inputs (read-only tensor arguments) before the op
        ins = []
        for sa, a in zip(sch, args):
            if torch.is_tensor(a) and a.is_cuda and a.numel() and not (sa.alias_info is not None and
                                                                       sa.alias_info.is_write):
                b = _bad(a)
                if b is not None:
                    ins.append(b)
        inb = torch.stack(ins).any() if ins else None
        r = func(*args, **(kwargs or {}))
        written = [(j, a) for j, (sa, a) in enumerate(zip(sch, args))
                   if sa.alias_info is not None and sa.alias_info.is_write and torch.is_tensor(a)]
        rs = r if isinstance(r, (tuple, list)) else (r,)
        written += [(100 + j, t) for j, (sr, t) in enumerate(zip(func._schema.returns, rs))
                    if torch.is_tensor(t) and sr.alias_info is None]
        for j, t in written:
            if t.is_cuda and t.numel() > 0:
                b = _bad(t)
                if b is not None:
                    self.rec.append((st, name, j, tuple(t.shape), b, inb))
        return r


def main():
    case = sys.argv[1] if len(sys.argv) > 1 else "mt_ubpl_b32"
    torch.use_deterministic_algorithms(True, warn_only=True)
    torch.utils.deterministic.fill_uninitialized_memory = True
    det_step._record_forward()
    p = Probe()
    with p:
        fin = det_step.run(case)
    torch.cuda.synchronize()
    main_st = torch.cuda.current_stream().cuda_stream

    def label(st):
        if st == main_st:
            return "main"
        for (M, _), ss in T._ModelStreams._cache.items():
            for i, s in enumerate(ss):
                if s.cuda_stream == st:
                    return ("student%d" % i) if i < M else ("teacher%d" % (i - M))
        return "stream%x" % st

    per = {}
    for st, name, j, shp, b, inb in p.rec:
        per.setdefault(st, []).append((name, j, shp, bool(b), None if inb is None else bool(inb)))
    nbad = 0
    for st, seq in per.items():
        flagged = [(i, e) for i, e in enumerate(seq) if e[3]]
        print("%-9s %d ops checked, %d with an unwritten element in an output" % (label(st), len(seq), len(flagged)),
              flush=True)
        shown = set()
        for i, (name, j, shp, _, inb) in flagged:
            key = (name, j, shp)
            if key in shown:
                continue
            shown.add(key)
            print("   op #%d %s arg %d %s  (inputs already bad: %s)" % (i, name, j, shp, inb), flush=True)
            if len(shown) >= 25:
                break
        nbad += len(flagged)
    fin_bad = sum(int(torch.isnan(t).any()) for k in ("grads", "params", "stats") for t in fin[k])
    print("nan_probe %s streams=%s: %d flagged op outputs; final state tensors with NaN: %d" % (
        case, os.environ.get("UBPL_MODEL_STREAMS", "1"), nbad, fin_bad), flush=True)


if __name__ == "__main__":
    main()

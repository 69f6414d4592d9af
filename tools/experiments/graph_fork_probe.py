"""Probe: HIP graph capture of work forked from a side stream onto a second-level side
stream and joined back (the weight-gradient side stream of hourglass._Exec.wg), bisecting
a capture_end segfault seen on the training step.  Each case runs in its own process.

    python tools/experiments/graph_fork_probe.py <case>
case: plain | nested | alloc | autograd | nested2
(round 6, ROCm 7.2 / torch 2.10: plain ok; nested, alloc, autograd segfault in capture_end)
"""
import sys

import torch


def body(case, s1, s2, x):
    cur = torch.cuda.current_stream()
    if case in ("nested", "alloc", "autograd", "nested2"):
        s1.wait_stream(cur)
        ctx = torch.cuda.stream(s1)
    else:
        ctx = torch.cuda.stream(cur)
    with ctx:
        inner = torch.cuda.current_stream()
        y = x * 2
        for _ in range(20):
            y = y + 1
            ev = torch.cuda.Event()
            ev.record(inner)
            s2.wait_event(ev)
            with torch.cuda.stream(s2):
                t = torch.empty_like(y) if case in ("alloc", "autograd") else None
                z = y * 3 if t is None else torch.mul(y, 3, out=t)
            keep.append((y, z, ev))
        if case != "nested2":
            ev = torch.cuda.Event()
            ev.record(s2)
            inner.wait_event(ev)
            keep.append(ev)
        out = y * 1
    if case in ("nested", "alloc", "autograd", "nested2"):
        cur.wait_stream(s1)
    if case == "nested2":
        cur.wait_stream(s2)            # the second-level stream joined by the origin directly
    return out


keep = []


class Fn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x):
        return x * 1

    @staticmethod
    def backward(ctx, g):
        return body("alloc", S1, S2, g)


def main():
    global S1, S2
    case = sys.argv[1]
    S1, S2 = torch.cuda.Stream(), torch.cuda.Stream()
    x = torch.randn(1 << 16, device="cuda", requires_grad=(case == "autograd"))

    def run():
        if case == "autograd":
            y = Fn.apply(x)
            y.sum().backward()
            return x.grad
        return body(case, S1, S2, x)

    side = torch.cuda.Stream()
    side.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(side):
        for _ in range(2):
            run()
    torch.cuda.current_stream().wait_stream(side)
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        out = run()
    g.replay()
    torch.cuda.synchronize()
    print(case, "ok", float(out.float().sum()))


if __name__ == "__main__":
    main()

"""GPU-box: does a captured graph with parallel stream branches keep each
branch's kernel order?  No ubpl kernels: torch elementwise chains only.

Four side streams each run a chain of dependent in-place updates on their own
tensor (x = x * a + b, L links), forked from and joined back to the capture
stream, then the main stream sums the four results.  The graph is replayed R
times and every replay is compared, bit for bit, with the same work run
eagerly on the same streams.

usage: python tools/graph_branch_probe.py [links] [replays] [numel]
"""
import sys

import torch


def work(xs, side, main, links):
    for s in side:
        s.wait_stream(main)
    outs = []
    for i, (x, s) in enumerate(zip(xs, side)):
        with torch.cuda.stream(s):
            y = x.clone()
            for k in range(links):
                y.mul_(1.0 + 1e-3 * ((k + i) % 7)).add_(0.25 * ((k * 3 + i) % 5) - 0.5)
            outs.append(y)
    for s in side:
        main.wait_stream(s)
    return torch.stack(outs).sum(0)


def main():
    links = int(sys.argv[1]) if len(sys.argv) > 1 else 200
    reps = int(sys.argv[2]) if len(sys.argv) > 2 else 50
    numel = int(sys.argv[3]) if len(sys.argv) > 3 else 1 << 20
    dev = torch.device("cuda")
    torch.manual_seed(0)
    xs = [torch.randn(numel, device=dev) for _ in range(4)]
    main_s = torch.cuda.Stream()
    side = [torch.cuda.Stream() for _ in range(4)]
    main_s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(main_s):
        ref = work(xs, side, main_s, links)
        for _ in range(2):
            work(xs, side, main_s, links)
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g, stream=main_s):
        out = work(xs, side, main_s, links)
    bad = 0
    for r in range(reps):
        g.replay()
        torch.cuda.synchronize()
        d = float((out - ref).abs().max())
        bad += d != 0.0
        if d != 0.0:
            print("replay %d differs: max |d| = %.3g" % (r, d), flush=True)
    print("graph_branch_probe links=%d numel=%d: %d of %d replays differ" % (links, numel, bad, reps), flush=True)


if __name__ == "__main__":
    main()

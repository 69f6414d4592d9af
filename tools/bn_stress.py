"""GPU-box: stress the one-launch BatchNorm statistics (last-arriver combine).

Many forward-statistics and backward launches over the hourglass's plane
shapes, on 4 streams at once (one scratch buffer per stream, as per network),
each case run twice: the outputs must repeat bit for bit, and the forward
mean / invstd must match a float64 torch reference.  A stale partial read
in the cross-workgroup combine shows up as a mismatch.
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "ubpl-poseestimation_amd"), ROOT]

import torch  # noqa: E402

from ubpl_amd import _lib  # noqa: E402
from ubpl_amd import kernels as Kn  # noqa: E402


def main():
    _lib.load()
    dev = torch.device("cuda", 0)
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 20
    g = torch.Generator(device=dev).manual_seed(0)
    shapes = [(B, C, R) for B in (32, 16) for C in (64, 128, 256) for R in (64, 32, 16, 8, 4)]
    streams = [torch.cuda.Stream(device=dev) for _ in range(4)]
    parts = [Kn.bn_part(32, 64, dev) for _ in streams]
    n = int(parts[0].numel())
    parts = [torch.zeros(max(n, int(_lib.lib().ubpl_bn_part_doubles(32, 256)) * 4), dtype=torch.float64,
                         device=dev) for _ in streams]
    coefs = [torch.empty(3 * 512, device=dev) for _ in streams]
    cases = []
    for (B, C, R) in shapes:
        x = torch.randn(B, C, R, R, device=dev, generator=g) * 3 + torch.randn(1, C, 1, 1, device=dev, generator=g)
        dz = torch.randn(B, C, R, R, device=dev, generator=g)
        cases.append((x, dz))
    torch.cuda.synchronize()

    def run_all():
        outs = []
        for rep in range(reps):
            for i, (x, dz) in enumerate(cases):
                si = (i + rep) % len(streams)
                s = streams[si]
                C = x.shape[1]
                with torch.cuda.stream(s):
                    gam = torch.ones(C, device=dev)
                    bet = torch.zeros(C, device=dev)
                    rm, rv = torch.zeros(C, device=dev), torch.ones(C, device=dev)
                    mu, istd, sc, sh = (torch.empty(C, device=dev) for _ in range(4))
                    Kn.bn_forward_stats(x, gam, bet, 1e-5, 0.1, rm, rv, parts[si], mu, istd, sc, sh)
                    dg, db = torch.zeros(C, device=dev), torch.zeros(C, device=dev)
                    dx = torch.empty_like(x)
                    Kn.bn_backward(dz, x, gam, mu, istd, sc, sh, 1, parts[si], coefs[si], dg, db, out=dx)
                    outs.append((i, mu, istd, dg, db, dx[:, :, :2, :2].clone()))
        torch.cuda.synchronize()
        return outs

    a = run_all()
    b = run_all()
    bad_rep = sum(1 for u, v in zip(a, b) if not all(torch.equal(p, q) for p, q in zip(u[1:], v[1:])))
    bad_ref = 0
    worst = 0.0
    for i, mu, istd, *_ in a:
        x = cases[i][0].double()
        m = x.mean((0, 2, 3))
        v = x.var((0, 2, 3), unbiased=False)
        e1 = float(((mu.double() - m).abs() / (v.sqrt() + 1e-12)).max())
        e2 = float(((istd.double() - 1 / (v + 1e-5).sqrt()) / (1 / (v + 1e-5).sqrt())).abs().max())
        worst = max(worst, e1, e2)
        if e1 > 1e-5 or e2 > 1e-5:
            bad_ref += 1
    print("launch pairs %d: non-repeating %d, off the f64 reference %d (worst rel %.3g)" %
          (len(a), bad_rep, bad_ref, worst), flush=True)
    sys.exit(1 if bad_rep or bad_ref else 0)


if __name__ == "__main__":
    main()

"""GPU-box: the 1x1 split-load conv (conv1x1_sol_kernel) under concurrency.
Four streams each run a chain of residual-shaped 1x1 convs (with prologue,
residual, in-place output) on their own inputs, all at once, ROUNDS times;
every round's outputs must equal, bit for bit, the same chain run alone on one
stream.  A difference reproduces the B=32 step's run-to-run drift
(tools/det_step.py) in isolation.

    python tools/sol_stress.py [rounds] [B] [plane]
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "ubpl-poseestimation_amd"), ROOT]

import torch  # noqa: E402

from ubpl_amd import kernels as Kn  # noqa: E402


def make_job(g, B, H, dev):
    def r(*s, scale=1.0):
        return (torch.randn(*s, generator=g) * scale).to(dev)
    job = {"x": r(B, 256, H, H)}
    for name, cin, cout in (("c1", 256, 128), ("c3", 128, 256), ("c4", 256, 256)):
        w = r(cout, cin, 1, 1, scale=cin ** -0.5)
        job[name] = (Kn.conv_weight_split(w, 0, 3), r(cout, scale=0.1), r(cin, scale=0.5).abs() + 0.5,
                     r(cin, scale=0.2))
    return job


def chain(job, extra):
    """x -> relu-prologue 256->128 -> 128->256 + x (new tensor) -> 256->256 + that (res aliasing out:
    in place over a copy of it, as the hourglass's skip-conv residuals run)."""
    ws, b, sc, sh = job["c1"]
    t1 = Kn.conv1x1_forward_split_load(job["x"], ws, b, sc, sh)
    if extra:
        t1 = Kn.bn_apply(t1, torch.ones_like(sc[:128]), torch.zeros_like(sh[:128]), relu=0)
    ws, b, sc, sh = job["c3"]
    t3 = Kn.conv1x1_forward_split_load(t1, ws, b, sc, sh, res=job["x"])
    ws, b, sc, sh = job["c4"]
    t4 = t3.clone()
    Kn.conv1x1_forward_split_load(t3, ws, b, sc, sh, res=t4, out=t4)
    return t1, t3, t4


def main():
    rounds = int(sys.argv[1]) if len(sys.argv) > 1 else 30
    B = int(sys.argv[2]) if len(sys.argv) > 2 else 32
    H = int(sys.argv[3]) if len(sys.argv) > 3 else 64
    extra = os.environ.get("STRESS_EXTRA", "1") == "1"
    dev = torch.device("cuda", 0)
    g = torch.Generator().manual_seed(7)
    jobs = [make_job(g, B, H, dev) for _ in range(4)]
    assert Kn.conv1x1_split_load_ok(jobs[0]["x"], jobs[0]["c1"][0])
    ref = []
    for j in jobs:
        ref.append([t.clone() for t in chain(j, extra)])
        torch.cuda.synchronize()
    streams = [torch.cuda.Stream(device=dev) for _ in jobs]
    main_s = torch.cuda.current_stream(dev)
    outs = []
    for _ in range(rounds):
        for s in streams:
            s.wait_stream(main_s)
        got = []
        for j, s in zip(jobs, streams):
            with torch.cuda.stream(s):
                got.append(chain(j, extra))
        for s, ts in zip(streams, got):
            main_s.wait_stream(s)
            for t in ts:
                t.record_stream(main_s)
        outs.append(got)
    torch.cuda.synchronize()
    bad = 0
    for rd, got in enumerate(outs):
        for ji, ts in enumerate(got):
            for k, (a, b) in enumerate(zip(ts, ref[ji])):
                if not torch.equal(a, b):
                    bad += 1
                    d = (a - b).abs()
                    print("round %d job %d out %d: %d elements differ, max |d| %.3g" % (
                        rd, ji, k, int((d != 0).sum()), float(d.max())), flush=True)
    print("sol_stress B=%d plane=%d rounds=%d extra=%d: %d differing outputs" % (B, H, rounds, extra, bad), flush=True)


if __name__ == "__main__":
    main()

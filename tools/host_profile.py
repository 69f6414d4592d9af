"""GPU-box: where the host time of the eager MT_UBPL step goes.

Builds the bench workload (bench.py: HG2, B=32, 256x256, 2 students + 2
teachers on per-network streams), warms up, then
  1. times the host side of N eager steps (the enqueue, no synchronize inside)
     against the same steps' wall time with a final synchronize;
  2. cProfiles N more eager steps and prints the top functions by own time.

    python tools/host_profile.py [steps]
"""
import cProfile
import os
import pstats
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "ubpl-poseestimation_amd"), ROOT]
os.environ.setdefault("UBPL_STEP_GRAPH", "0")

import torch  # noqa: E402

import bench  # noqa: E402


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 5
    from ubpl_amd import _lib
    from ubpl_amd.hourglass import StackedHourglass
    from ubpl_amd.optim import FlatAdamW
    from ubpl_amd import train as T
    _lib.load()
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    torch.manual_seed(1388)
    models, emas, optims = [], [], []
    for _ in range(2):
        m, e = StackedHourglass(16, 2, "AvgPool"), StackedHourglass(16, 2, "AvgPool")
        for p in e.parameters():
            p.detach_()
        models.append(m)
        emas.append(e)
        optims.append(FlatAdamW(m, lr=2.5e-4, weight_decay=0.0))
    args = bench.make_args(32)
    batches = bench.make_batches(2, 32, 16, dev, 1388, 256, False)
    T.train_mt_ubpl([batches[i % 2] for i in range(3)], models, emas, optims, args, verbose=False)
    torch.cuda.synchronize()
    steps = [batches[i % 2] for i in range(n)]
    t0 = time.perf_counter()
    T.train_mt_ubpl(steps, models, emas, optims, args, verbose=False)
    t1 = time.perf_counter()
    torch.cuda.synchronize()
    t2 = time.perf_counter()
    print("eager: host enqueue %.1f ms/step (incl. the lagged record reads), wall %.1f ms/step, %d steps" %
          ((t1 - t0) / n * 1e3, (t2 - t0) / n * 1e3, n), flush=True)
    pr = cProfile.Profile()
    pr.enable()
    T.train_mt_ubpl(steps, models, emas, optims, args, verbose=False)
    torch.cuda.synchronize()
    pr.disable()
    st = pstats.Stats(pr)
    st.sort_stats("tottime").print_stats(35)
    st.sort_stats("cumulative").print_stats(25)


if __name__ == "__main__":
    main()

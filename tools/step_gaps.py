"""GPU idle time at the step boundaries of the captured headline step: HIP events
on the main stream right before each step's static-input copies and right after
its graph replay (and the records' copy), the gap end(k) -> start(k+1) measured on
the device clock.  Unprofiled (rocprofv3 serialises dispatch).

    python tools/step_gaps.py [steps]
"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "ubpl-poseestimation_amd"))

import torch  # noqa: E402

import bench  # noqa: E402


def main():
    steps = int(sys.argv[1]) if len(sys.argv) > 1 else 10
    from ubpl_amd import _lib
    from ubpl_amd import train as T
    from ubpl_amd.hourglass import StackedHourglass
    from ubpl_amd.optim import FlatAdamW
    _lib.load()
    dev = torch.device("cuda", 0)
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
    batches = bench.make_batches(2, 32, 16, dev, 1388)
    T.train_mt_ubpl([batches[i % 2] for i in range(3)], models, emas, optims, args, verbose=False)
    torch.cuda.synchronize()
    ev = []
    orig = T._StepGraph.run

    def run(self, batch, d):
        s = torch.cuda.Event(enable_timing=True)
        s.record()
        out = orig(self, batch, d)
        e = torch.cuda.Event(enable_timing=True)
        e.record()
        ev.append((s, e, time.perf_counter()))
        return out
    T._StepGraph.run = run
    t0 = time.perf_counter()
    T.train_mt_ubpl([batches[i % 2] for i in range(steps)], models, emas, optims, args, verbose=False)
    torch.cuda.synchronize()
    wall = (time.perf_counter() - t0) / steps * 1e3
    spans = [s.elapsed_time(e) for s, e, _ in ev]
    gaps = [ev[i][1].elapsed_time(ev[i + 1][0]) for i in range(len(ev) - 1)]
    host = [(ev[i + 1][2] - ev[i][2]) * 1e3 for i in range(len(ev) - 1)]
    print("wall %.2f ms/step; device span per step (copies + replay) %.2f ms (min %.2f); "
          "gap end(k)->start(k+1) mean %.3f ms max %.3f; host loop per step %.2f ms"
          % (wall, sum(spans) / len(spans), min(spans), sum(gaps) / len(gaps), max(gaps), sum(host) / len(host)))


if __name__ == "__main__":
    main()

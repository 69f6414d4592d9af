"""Where the MT_UBPL step's time goes (eager, B=32): one network-view forward
alone, the forward phase (2 students x 2 views with saves + 2 teachers x 2 views
on the four model streams), one view's backward alone, and the full step.
A chain-bound phase takes about (passes per stream) x (one pass alone); a
throughput-bound one takes longer.

    python tools/phase_timing.py [reps]
"""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "ubpl-poseestimation_amd"))
import bench  # noqa: E402


def timed(fn, reps):
    fn()
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(reps):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t) / reps * 1e3


def main():
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 5
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    from ubpl_amd import _lib
    from ubpl_amd.hourglass import StackedHourglass
    from ubpl_amd.optim import FlatAdamW
    from ubpl_amd import train as T
    _lib.load()
    B, K = 32, 16
    torch.manual_seed(1388)
    models, emas, optims = [], [], []
    for _ in range(2):
        m = StackedHourglass(K, 2, "AvgPool")
        e = StackedHourglass(K, 2, "AvgPool")
        for p in e.parameters():
            p.detach_()
        models.append(m)
        emas.append(e)
        optims.append(FlatAdamW(m, lr=2.5e-4, weight_decay=0.0))
    args = bench.make_args(B)
    batches = bench.make_batches(2, B, K, dev, 1388)
    imgs = [x.to(dev).float().contiguous() for x in batches[0][0]]
    os.environ["UBPL_STEP_GRAPH"] = "0"

    def one_fwd():
        with torch.no_grad():
            emas[0](imgs[0])

    def one_fwd_grad():
        o, f = models[0](imgs[0])
        return o, f

    def one_fwd_bwd():
        o, f = models[0](imgs[0])
        (o.square().mean() + f.square().mean()).backward()

    def fwd_phase():
        ms = T._ModelStreams.make(2, dev)
        outs = []
        for mi in range(2):
            with ms.on(mi):
                for a in range(2):
                    outs.append(models[mi](imgs[a]))
            with ms.on_teacher(mi):
                with torch.no_grad():
                    for a in range(2):
                        outs.append(emas[mi](imgs[a]))
        ms.join()
        return outs

    def step():
        T.train_mt_ubpl(batches[:1], models, emas, optims, args, verbose=False)

    t1 = timed(one_fwd, reps)
    t1g = timed(one_fwd_grad, reps)
    t1b = timed(one_fwd_bwd, reps)
    tf = timed(fwd_phase, reps)
    ts = timed(step, reps)
    print("one forward (teacher, no grad) %.2f ms | with saves %.2f ms | fwd+bwd %.2f ms (bwd ~%.2f)" % (
        t1, t1g, t1b, t1b - t1g))
    print("forward phase (8 passes, 4 streams) %.2f ms  [2 passes per stream alone: %.2f ms]" % (tf, 2 * t1g))
    print("full step %.2f ms -> after the forward phase %.2f ms  [2 bwd per stream alone: %.2f ms]" % (
        ts, ts - tf, 2 * (t1b - t1g)))


if __name__ == "__main__":
    main()

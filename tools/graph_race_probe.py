"""GPU-box: repeat the MT_UBPL step with per-network streams in several modes
against the eager step on the null stream (tools/determinism.py's run) and
count the runs that differ.  Modes: graph (captured step), eager-side (eager
steps with a non-null stream as the step's main stream), graph-nosplit
(captured, second-view backward on the student's own stream)."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import determinism as D  # noqa: E402


STEPS = int(os.environ.get("PROBE_STEPS", "4"))


def one(mode):
    if mode == "eager-side":
        s = torch.cuda.Stream()
        s.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(s):
            r = D.run(False, True, STEPS)
        torch.cuda.synchronize()
        return r
    if mode == "graph-nosplit":
        return D.run(True, False, STEPS)
    return D.run(True, True, STEPS)


def main():
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 10
    modes = sys.argv[2].split(",") if len(sys.argv) > 2 else ["graph"]
    e = D.run(False, True, STEPS)
    e0 = D.run(False, False, STEPS)
    for mode in modes:
        ref = e0 if mode == "graph-nosplit" else e
        bad = 0
        for i in range(reps):
            g = one(mode)
            ds = {k: max(float((x - y).abs().max()) for x, y in zip(ref[k], g[k])) for k in ref}
            bad += max(ds.values()) != 0.0
            print("%s rep %d %s" % (mode, i, " ".join("%s=%.3g" % kv for kv in ds.items())), flush=True)
        print("%s (%d steps): %d of %d differ" % (mode, STEPS, bad, reps), flush=True)


if __name__ == "__main__":
    main()

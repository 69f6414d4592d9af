"""Calibrate bench.py's CPU baseline (the oracle's restatement of the MT_UBPL
step, oracle/step.py) against the reference's own train()
(projects/MT_UBPL.py:157-352) on the same inputs, same host, same threads.

Runs only in the build container (it imports /root/reference through the
golden generator's stub recipe).  Writes profiles/r03_cpu_calibration_b<B>.json.

    python tools/calibrate_cpu_baseline.py [B] [steps]
"""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "tests", "golden"), ROOT]
import torch  # noqa: E402
import gen_golden as GG  # noqa: E402
import seeds  # noqa: E402
from oracle import hourglass as OH  # noqa: E402
from oracle import render as OR  # noqa: E402
from oracle import step as OS  # noqa: E402


def timed(fn, steps):
    fn(1)                                       # warm-up step
    t = time.time()
    fn(steps)
    return (time.time() - t) / steps


def main(B=4, steps=2):
    threads = torch.get_num_threads()
    R = GG.import_reference()
    proj = GG._import_project("MT_UBPL")
    cfg = dict(seeds.step_cases()["mt_ubpl"], B=B, nlab=B // 2)

    def run(factory, train):
        models, emas, optims = seeds.step_models(factory, cfg)
        loader, args = seeds.step_batch(cfg, OR.kps_heatmap_torch)
        return lambda n: train(loader * n, models, emas, optims, args)

    import contextlib
    import io
    with contextlib.redirect_stdout(io.StringIO()):
        t_ref = timed(run(R["SH"], proj.train), steps)
        t_port = timed(run(OH.oracle_factory, OS.train_mt_ubpl), steps)
    rec = {"what": "MT_UBPL train step, 2-stack HG, K=16, 256x256, B=%d (half labeled); reference = "
                   "projects/MT_UBPL.py train() imported from /root/reference (stub recipe, CPU); port = "
                   "oracle/step.py train_mt_ubpl (bench.py cpu_baseline)" % B,
           "threads": threads, "cpus": os.cpu_count(), "steps_timed": steps,
           "reference_s_per_step": round(t_ref, 3), "port_s_per_step": round(t_port, 3),
           "reference_images_per_s": round(B / t_ref, 4), "port_images_per_s": round(B / t_port, 4),
           "port_over_reference": round(t_ref / t_port, 4),
           "survey_reference_images_per_s": {"B4": 0.92, "B32": 0.51}}
    out = os.path.join(ROOT, "profiles", "r03_cpu_calibration_b%d.json" % B)
    with open(out, "w") as f:
        json.dump(rec, f, indent=1)
    print(json.dumps(rec))


if __name__ == "__main__":
    main(*[int(v) for v in sys.argv[1:]])

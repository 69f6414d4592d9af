"""From a rocprofv3 kernel trace of `bench.py`: the roofline kernel's average
duration in situ (the warm-up + timed + recording steps, networks overlapping)
and in the back-to-back replays bench.py times with HIP events (the last
(1 + reps) * launches_per_step launches of that kernel).

    python tools/trace_roofline.py TRACE.csv [launches_per_step 60] [reps 10]
"""
import csv
import os
import json
import sys

# the 2xfp16 default instantiation (ROOF_KERNEL="conv_psah_kernel<64, 3, 128, 1, 1, 256" on 6xbf16)
KERNEL = os.environ.get("ROOF_KERNEL", "conv_psah_kernel<64, 2, 128, 1, 1, 256")


def main(path, n=60, reps=10):
    rows = [r for r in csv.DictReader(open(path)) if KERNEL in r["Kernel_Name"]]
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    d = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3 for r in rows]
    k = (1 + reps) * n
    situ, rep = d[:-k], d[-reps * n:]
    out = {"kernel": KERNEL + ">", "trace": path, "launches_total": len(d),
           "in_situ": {"launches": len(situ), "avg_us": round(sum(situ) / len(situ), 2)},
           "replayed": {"launches": len(rep), "avg_us": round(sum(rep) / len(rep), 2)}}
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main(sys.argv[1], *[int(v) for v in sys.argv[2:]])

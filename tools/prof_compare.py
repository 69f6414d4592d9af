"""Per-kernel time per step of two rocprofv3 kernel traces side by side (timed window:
steps delimited by the fused AdamW+EMA launches, 2 per step; warm-up steps skipped).

    python tools/prof_compare.py A/run_kernel_trace.csv B/run_kernel_trace.csv [warm] [steps] [labelA] [labelB]
"""
import collections
import csv
import re
import sys


def per_kernel(path, warm, steps):
    ks = []
    for r in csv.DictReader(open(path)):
        m = re.search(r"::(\w+)(<[^(]*>)?\(", r["Kernel_Name"])
        kn = (m.group(1) + (m.group(2) or "").replace(" ", "")) if m else r["Kernel_Name"][:40]
        ks.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), kn))
    ks.sort()
    ad = [k for k in ks if k[2].startswith("adamw_ema")]
    t0, t1 = ad[2 * warm - 1][1], ad[2 * (warm + steps) - 1][1]
    fam = collections.defaultdict(float)
    for s, e, kn in ks:
        if s >= t0 and e <= t1:
            fam[kn] += (e - s) / 1e6 / steps
    return fam, (t1 - t0) / 1e6 / steps


a, wa = per_kernel(sys.argv[1], int(sys.argv[3]) if len(sys.argv) > 3 else 2, int(sys.argv[4]) if len(sys.argv) > 4 else 3)
b, wb = per_kernel(sys.argv[2], int(sys.argv[3]) if len(sys.argv) > 3 else 2, int(sys.argv[4]) if len(sys.argv) > 4 else 3)
la, lb = (sys.argv[5], sys.argv[6]) if len(sys.argv) > 6 else ("A", "B")
print("step (profiled) ms: %s %.1f  %s %.1f;  kernel ms/step: %s %.1f  %s %.1f" % (
    la, wa, lb, wb, la, sum(a.values()), lb, sum(b.values())))
keys = sorted(set(a) | set(b), key=lambda k: -(a.get(k, 0) + b.get(k, 0)))
print("%-58s %9s %9s %7s" % ("kernel", la, lb, la + "/" + lb))
for k in keys[:32]:
    print("%-58s %9.2f %9.2f %7s" % (k[:58], a.get(k, 0), b.get(k, 0),
                                       "%.2f" % (a[k] / b[k]) if a.get(k) and b.get(k) else "-"))

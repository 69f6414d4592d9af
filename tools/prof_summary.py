"""Summarise a rocprofv3 kernel trace of bench.py: per-kernel totals per step and per-shape conv times.

    python tools/prof_summary.py <kernel_trace.csv> <timed steps> [top shapes] [bench.json]

With a bench.json (the same config benched WITHOUT the profiler) the window line
also carries the profiled / benched ms-per-step ratio: rocprofv3's kernel trace
serialises the captured graph's launches, so the profiled step is slower than
the benched one and the per-kernel times are to be read with that ratio.

bench.py launches a ~1-cycle spin_kernel (torch.cuda._sleep(1)) right before and
right after its timed region; only the kernels that START between those two
markers are counted (the timed steps alone: no warm-up, capture, roofline
replay or its 20M-cycle spin).  A trace without the markers (an older bench or
another program) is summarised whole, and the output says so."""
import collections
import csv
import json
import re
import sys


def kname(n):
    m = re.search(r"::(\w+)(<[^(]*>)?\(", n)
    return (m.group(1) if m else n[:40]), ((m.group(2) or "").replace(" ", "") if m else "")


def window(rows):
    """(start, end) timestamps between the bench's two spin-kernel markers, or None."""
    sp = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"])) for r in rows if "spin_kernel" in r["Kernel_Name"])
    if len(sp) < 2:
        return None
    return sp[0][1], sp[1][0]


def main():
    path = sys.argv[1]
    steps = int(sys.argv[2]) if len(sys.argv) > 2 else 1
    top = int(sys.argv[3]) if len(sys.argv) > 3 else 20
    benched = None
    if len(sys.argv) > 4:
        try:
            benched = float(json.load(open(sys.argv[4]))["ms_per_step"])
        except (OSError, ValueError, KeyError):
            benched = None
    rows = list(csv.DictReader(open(path)))
    w = window(rows)
    if w:
        rows = [r for r in rows if w[0] <= int(r["Start_Timestamp"]) < w[1] and "spin_kernel" not in r["Kernel_Name"]]
        print("window: %d kernels between the bench's markers, %.2f ms wall (%d timed steps: %.2f ms/step)"
              % (len(rows), (w[1] - w[0]) / 1e6, steps, (w[1] - w[0]) / 1e6 / steps))
        if benched:
            prof = (w[1] - w[0]) / 1e6 / steps
            print("profiled %.2f ms/step vs benched %.2f ms/step (%s): ratio %.3f"
                  % (prof, benched, sys.argv[4], prof / benched))
    else:
        print("window: no bench markers found - the WHOLE trace is summarised")
    g = collections.defaultdict(list)
    cat = collections.defaultdict(float)
    busy = []
    for r in rows:
        n = r["Kernel_Name"]
        t0, t1 = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        d = (t1 - t0) / 1e3
        kn, tmpl = kname(n)
        cat[kn] += d
        busy.append((t0, t1))
        if "conv" in kn or "wgrad" in kn:
            g[(kn, tmpl, int(r["Grid_Size_X"]) // 256, r["Grid_Size_Y"], r["Grid_Size_Z"])].append(d)
    # union of busy intervals (kernels of the four network streams overlap)
    union, cur = 0, None
    for a, b in sorted(busy):
        if cur is None or a > cur[1]:
            if cur:
                union += cur[1] - cur[0]
            cur = [a, b]
        else:
            cur[1] = max(cur[1], b)
    if cur:
        union += cur[1] - cur[0]
    tot = sum(cat.values())
    print("total kernel ms/step %.2f (summed over streams), busy union ms/step %.2f, launches/step %d"
          % (tot / steps / 1e3, union / steps / 1e6, len(rows) // steps))
    for k, v in sorted(cat.items(), key=lambda kv: -kv[1])[:20]:
        print("%5.1f%% %8.2f ms/step %s" % (100 * v / tot, v / steps / 1e3, k))
    ct = sum(sum(v) for v in g.values())
    for k, v in sorted(g.items(), key=lambda kv: -sum(kv[1]))[:top]:
        print("%5.1f%% n/step=%4d avg=%7.1fus %s" % (100 * sum(v) / ct, len(v) // steps, sum(v) / len(v), k))


if __name__ == "__main__":
    main()

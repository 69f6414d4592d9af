"""Summarise a rocprofv3 kernel trace: per-kernel totals per step and per-shape conv times."""
import collections
import csv
import re
import sys

path = sys.argv[1]
steps = int(sys.argv[2]) if len(sys.argv) > 2 else 1
rows = list(csv.DictReader(open(path)))
g = collections.defaultdict(list)
cat = collections.defaultdict(float)
for r in rows:
    n = r["Kernel_Name"]
    d = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
    m = re.search(r"::(\w+)(<[^(]*>)?\(", n)
    kn = m.group(1) if m else n[:40]
    cat[kn] += d
    if "conv" in kn:
        g[(kn, (m.group(2) or "").replace(" ", ""), int(r["Grid_Size_X"]) // 256, r["Grid_Size_Y"],
           r["Grid_Size_Z"])].append(d)
tot = sum(cat.values())
print("total kernel ms/step %.2f" % (tot / steps / 1e3))
for k, v in sorted(cat.items(), key=lambda kv: -kv[1])[:16]:
    print("%5.1f%% %8.2f ms/step %s" % (100 * v / tot, v / steps / 1e3, k))
ct = sum(sum(v) for v in g.values())
for k, v in sorted(g.items(), key=lambda kv: -sum(kv[1]))[:int(sys.argv[3]) if len(sys.argv) > 3 else 20]:
    print("%5.1f%% n/step=%4d avg=%7.1fus %s" % (100 * sum(v) / ct, len(v) // steps, sum(v) / len(v), k))

"""Per-pass kernel breakdown of a tools/pass_profile.py kernel trace: one
teacher forward and one student forward+backward, nothing overlapping.

    python tools/pass_summary.py gpurun_out/pp/pp_kernel_trace.csv
"""
import collections
import csv
import re
import sys


def main():
    rows = list(csv.DictReader(open(sys.argv[1])))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    idx = [i for i, r in enumerate(rows) if "stem_s2d_split_kernel" in r["Kernel_Name"] or
           "conv_fwd_kernel<64, 128, 7, 2" in r["Kernel_Name"]]
    # warm-up teacher fwd, warm-up student fwd+bwd, then REPS teacher fwds, then REPS student passes
    for lo, hi, label in ((idx[2], idx[3], "teacher forward"), (idx[5], idx[6], "student forward + backward")):
        cat, cnt, tot = collections.defaultdict(float), collections.Counter(), 0.0
        for r in rows[lo:hi]:
            m = re.search(r"(\w+)(<[^(]*>)?\(", r["Kernel_Name"])
            kn = m.group(1) if m else r["Kernel_Name"][:50]
            d = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
            cat[kn] += d
            cnt[kn] += 1
            tot += d
        span = (int(rows[hi - 1]["End_Timestamp"]) - int(rows[lo]["Start_Timestamp"])) / 1e3
        print("%s: %d launches, kernel sum %.2f ms, span %.2f ms" % (label, hi - lo, tot / 1e3, span / 1e3))
        for k, v in sorted(cat.items(), key=lambda kv: -kv[1])[:20]:
            print("   %6.3f ms %5.1f%% n=%4d %s" % (v / 1e3, 100 * v / tot, cnt[k], k))


if __name__ == "__main__":
    main()

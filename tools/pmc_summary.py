"""Summarise the rocprofv3 --pmc passes of tools/gpu_pmc.sh per kernel.

HBM traffic per launch follows MI355X_MICROARCH.md §HBM: FETCH_SIZE and
WRITE_SIZE are in KiB; on gfx950 FETCH_SIZE reports half the bytes of a wide
coalesced read, so it is doubled (fetch_bytes); the raw value is kept too.
SQ_* wave counters count quad-cycles; SQ_VALU_MFMA_BUSY_CYCLES counts cycles.

    python tools/pmc_summary.py gpurun_out/pmc profiles/r01_pmc_conv.json
"""
import collections
import csv
import json
import os
import sys


def load(path):
    per = collections.defaultdict(lambda: collections.defaultdict(list))
    dur = collections.defaultdict(dict)
    for r in csv.DictReader(open(path)):
        name = r["Kernel_Name"]
        if "conv" not in name:
            continue
        key = name.replace("void (anonymous namespace)::", "").split("(")[0]
        if BY_GRID:
            key += " grid=%d" % (int(r["Grid_Size"]) // 256)
        per[key][r["Counter_Name"]].append(float(r["Counter_Value"]))
        dur[key][r["Dispatch_Id"]] = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
    return per, dur


# PMC_BY_GRID=1: one entry per (kernel, workgroup count) — the shapes of one template apart
BY_GRID = os.environ.get("PMC_BY_GRID") == "1"


def main():
    d = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/pmc"
    out = sys.argv[2] if len(sys.argv) > 2 else None
    res = {}
    for pas in ("sq", "sq2", "fetch", "write"):
        f = os.path.join(d, pas + "_counter_collection.csv")
        if not os.path.exists(f):
            continue
        per, dur = load(f)
        for k, cs in per.items():
            e = res.setdefault(k, {})
            for c, v in cs.items():
                e[c] = sum(v) / len(v)
            e.setdefault("launches", len(dur[k]))
            e.setdefault("avg_us_profiled", sum(dur[k].values()) / max(1, len(dur[k])))
    for k, e in res.items():
        if "FETCH_SIZE" in e:
            e["fetch_bytes_raw"] = e["FETCH_SIZE"] * 1024
            e["fetch_bytes"] = 2 * e["FETCH_SIZE"] * 1024
        if "WRITE_SIZE" in e:
            e["write_bytes"] = e["WRITE_SIZE"] * 1024
        if "fetch_bytes" in e and "write_bytes" in e:
            e["hbm_bytes"] = e["fetch_bytes"] + e["write_bytes"]
        if "SQ_WAVE_CYCLES" in e:
            w = e["SQ_WAVE_CYCLES"]
            e["frac_wait_any"] = e.get("SQ_WAIT_ANY", 0) / w
            e["frac_wait_inst"] = e.get("SQ_WAIT_INST_ANY", 0) / w
            e["frac_active"] = e.get("SQ_ACTIVE_INST_ANY", 0) / w
        if "GRBM_GUI_ACTIVE" in e and "SQ_VALU_MFMA_BUSY_CYCLES" in e:
            # per-SIMD MFMA busy / kernel cycles (GRBM sums the 8 XCDs; 1024 SIMDs)
            e["mfma_pipe_util"] = (e["SQ_VALU_MFMA_BUSY_CYCLES"] / 1024) / (e["GRBM_GUI_ACTIVE"] / 8)
    txt = json.dumps(res, indent=1, sort_keys=True)
    print(txt)
    if out:
        with open(out, "w") as fh:
            fh.write(txt + "\n")


if __name__ == "__main__":
    main()

"""HBM traffic per launch of bench.py's roofline kernel, from rocprofv3 --pmc
passes over the bench command itself (tools/gpu_pmc.sh, mode "bench").

The roofline kernel is every 3x3 forward conv with the fused BN prologue
(conv_fwd_kernel<BM, 128, 3, 1, PRO=true, ...>, both tile heights), as in
bench.py's ConvTimer.  Bytes follow MI355X_MICROARCH.md §HBM: FETCH_SIZE and
WRITE_SIZE are KiB; gfx950's FETCH_SIZE counts half the bytes of wide reads,
so it is doubled.  Writes profiles/pmc_roofline.json for bench.py.

    python tools/pmc_roofline.py gpurun_out/pmc_bench profiles/pmc_roofline.json [source-tag] [f32|psa|psah]

With "psa" (conv precision 6xbf16) the roofline kernel is bench.py's:
conv_psa_kernel<128, 3, 3, 256, 2> on 512-workgroup grids (the 128 -> 128
3x3 convs on the 64x64 planes at B=32, forward and data gradient: rocprof
names cannot tell them apart, same shapes and traffic model).
"""
import csv
import json
import os
import re
import sys

PATS = {"f32": re.compile(r"conv_fwd_kernel<(\d+), 128, 3, 1, true, false"),
        "psa": re.compile(r"conv_psa_kernel<128, 3, 3, 256, 2(, false)?>"),
        "psah": re.compile(r"conv_psah_kernel<64, 3, 128, 1, 1(, 256(, false)*)?>"),
        "psah2": re.compile(r"conv_psah_kernel<64, 2, 128, 1, 1(, 256)?>")}
# psa / psah: only the 512-workgroup launches (grid size in work-items)
GRID = {"psa": 512 * 256, "psah": 512 * 256, "psah2": 512 * 256}
PAT = PATS["f32"]
KIND = "f32"


def per_launch(path, counter):
    vals = {}
    for r in csv.DictReader(open(path)):
        if r["Counter_Name"] != counter or not PAT.search(r["Kernel_Name"]):
            continue
        if GRID.get(KIND) and int(r["Grid_Size"]) != GRID[KIND]:
            continue
        vals[r["Dispatch_Id"]] = vals.get(r["Dispatch_Id"], 0.0) + float(r["Counter_Value"])
    return vals


def step_totals(path, counter, steps, scale):
    """Bytes per timed step by kernel family: the dispatches between bench.py's two
    spin-kernel markers (torch.cuda._sleep around the timed region), / steps."""
    rows = {}
    for r in csv.DictReader(open(path)):
        if r["Counter_Name"] != counter and "spin_kernel" not in r["Kernel_Name"]:
            continue
        i = int(r["Dispatch_Id"])
        name, v = r["Kernel_Name"], float(r["Counter_Value"]) if r["Counter_Name"] == counter else 0.0
        rows[i] = (name, rows.get(i, (name, 0.0))[1] + v)
    order = sorted(rows)
    marks = [i for i in order if "spin_kernel" in rows[i][0]]
    if len(marks) < 2:
        return None
    fam = {}
    for i in order:
        if marks[0] < i < marks[1]:
            m = re.search(r"(\w+)(<|\()", rows[i][0].split("::")[-1])
            k = m.group(1) if m else rows[i][0][:40]
            fam[k] = fam.get(k, 0.0) + scale * rows[i][1] / steps
    return fam


def main():
    d = sys.argv[1]
    out = sys.argv[2]
    tag = sys.argv[3] if len(sys.argv) > 3 else d
    kind = sys.argv[4] if len(sys.argv) > 4 else "f32"
    global PAT, KIND
    PAT, KIND = PATS[kind], kind
    fetch = per_launch(os.path.join(d, "fetch_counter_collection.csv"), "FETCH_SIZE")
    write = per_launch(os.path.join(d, "write_counter_collection.csv"), "WRITE_SIZE")
    nf, nw = len(fetch), len(write)
    fb = 2 * 1024 * sum(fetch.values()) / max(nf, 1)
    wb = 1024 * sum(write.values()) / max(nw, 1)
    res = {"kernel": {"f32": "conv_fwd_kernel<*,128,3,1,PRO> (all launches of the bench step)",
                      "psa": "conv_psa_kernel<128, 3, 3, 256, 2> on 512-workgroup grids (3x3 128->128 at 64x64, "
                             "B=32: forward + data gradient)",
                      "psah": "conv_psah_kernel<64, 3, 128, 1, 1, 256> on 512-workgroup grids (3x3 128->128 at "
                              "64x64, B=32: forward + data gradient)",
                      "psah2": "conv_psah_kernel<64, 2, 128, 1, 1, 256> on 512-workgroup grids (3x3 128->128 at "
                               "64x64, B=32, 2xfp16: forward + data gradient)"}[kind],
           "launches_fetch_pass": nf, "launches_write_pass": nw,
           "fetch_bytes_per_launch": fb, "write_bytes_per_launch": wb,
           "hbm_bytes_per_launch": fb + wb,
           "method": "rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE, separate passes over bench.py; FETCH_SIZE x2 (gfx950)",
           "source": tag}
    steps = int(os.environ.get("PMC_STEPS", "2"))
    ft = step_totals(os.path.join(d, "fetch_counter_collection.csv"), "FETCH_SIZE", steps, 2 * 1024)
    wt = step_totals(os.path.join(d, "write_counter_collection.csv"), "WRITE_SIZE", steps, 1024)
    if ft and wt:
        fams = sorted(set(ft) | set(wt), key=lambda k: -(ft.get(k, 0) + wt.get(k, 0)))
        res["step_bytes"] = {"fetch_gb": sum(ft.values()) / 1e9, "write_gb": sum(wt.values()) / 1e9,
                             "steps": steps, "note": "eager step: dispatches between the bench's timed-region markers",
                             "by_kernel_gb": {k: [round(ft.get(k, 0) / 1e9, 3), round(wt.get(k, 0) / 1e9, 3)]
                                              for k in fams[:30]}}
    print(json.dumps(res, indent=1))
    with open(out, "w") as fh:
        fh.write(json.dumps(res, indent=1) + "\n")


if __name__ == "__main__":
    main()

"""In-kernel shader clock of the two biggest split-path kernels (diagnostic; needs the
UBPL_CLOCK_STAMP=1 build of libubpl_hip.so, loaded with UBPL_LIB_DIR):

    make -C ubpl-poseestimation_amd/csrc OUT=../../abvar/CLK/libubpl_hip.so \\
         OPS=../../abvar/CLK/libubpl_ops.so OBJDIR=../../abvar/CLK/obj EXTRA=-DUBPL_CLOCK_STAMP=1
    UBPL_LIB_DIR=abvar/CLK python tools/clock_probe.py [seconds]

Each kernel runs back to back on random data for `seconds` (the chip settles its clock
under load: MI355X_MICROARCH.md 'DVFS give-back' item 6), then the last launch's per-
workgroup stamps give clock = d(s_memtime) / d(s_memrealtime) x 100 MHz; printed with the
launch time and the matrix-core rate it implies at 2.4 GHz and at the measured clock.

Other stamp builds: EXTRA=-DUBPL_CLOCK_STAMP=2 with UBPL_PROBE_TIMELINE=1 — the launch
timeline (workgroup entry / exit, by XCD and by dispatch half; profiles/r05_v10_timeline.txt);
EXTRA=-DUBPL_CLOCK_STAMP=3 with UBPL_PROBE_PHASES=1 — the 1x1 kernel's K-loop phases
(profiles/r05_v13_sol_phases.txt).
"""
import ctypes
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "ubpl-poseestimation_amd"))
from ubpl_amd import _lib  # noqa: E402
from ubpl_amd import kernels as Kn  # noqa: E402

SPLIT_PEAK = 2500.0 / 6          # f32-equivalent TF/s of 6 bf16 products at the dense bf16 peak
TIMELINE = os.environ.get("UBPL_PROBE_TIMELINE") == "1"   # with a UBPL_CLOCK_STAMP=2 build
PHASES = os.environ.get("UBPL_PROBE_PHASES") == "1"       # with a UBPL_CLOCK_STAMP=3 build


def stamps(lib, n):
    buf = (ctypes.c_ulonglong * (2 * n))()
    rc = lib.ubpl_debug_clock_stamps(buf, n)
    assert rc == 0, rc
    a = np.frombuffer(buf, dtype=np.uint64).astype(np.float64)
    return a[:n], a[n:]


def probe(name, fn, nwg, flops, seconds, lib):
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    t_end = time.time() + seconds
    n = 0
    while time.time() < t_end:
        for _ in range(20):
            fn()
        torch.cuda.synchronize()
        n += 20
    ev0.record()
    for _ in range(20):
        fn()
    ev1.record()
    torch.cuda.synchronize()
    ms = ev0.elapsed_time(ev1) / 20
    if PHASES:
        # UBPL_CLOCK_STAMP=3 build, 1x1 kernel only: per-workgroup K-loop phase sums (wave 0)
        if "sol" not in name:
            return
        buf = (ctypes.c_ulonglong * (4 * nwg))()
        assert lib.ubpl_debug_clock_stamps4(buf, nwg) == 0
        a = np.frombuffer(buf, dtype=np.uint64).astype(np.float64).reshape(4, nwg)
        med = np.median(a, axis=1)
        tot = med.sum()
        print("%-34s %.3f ms/launch; K-loop cycles per workgroup (median): wait+barrier %.0f (%.0f %%), DMA issue"
              " %.0f (%.0f %%), prologue+split %.0f (%.0f %%), MFMA rows %.0f (%.0f %%); sum %.0f"
              % (name, ms, med[0], 100 * med[0] / tot, med[1], 100 * med[1] / tot, med[2], 100 * med[2] / tot,
                 med[3], 100 * med[3] / tot, tot))
        ids = np.arange(nwg)
        for half, sel in (("first half", ids < nwg // 2), ("second half", ids >= nwg // 2)):
            m = np.median(a[:, sel], axis=1)
            print("    %s: %s" % (half, " ".join("%.0f" % v for v in m)))
        return
    dt, dr = stamps(lib, nwg)
    if TIMELINE:
        # UBPL_CLOCK_STAMP=2 build: absolute real-time (100 MHz) at workgroup entry / exit
        t0 = dt.min()
        st, en = (dt - t0) / 100.0, (dr - t0) / 100.0            # us
        print("%-34s %.3f ms/launch; last launch: span %.1f us, workgroup starts 0 .. %.1f us (median %.1f),"
              " lifetimes median %.1f us (p10 %.1f p90 %.1f), ends median %.1f us, last %.1f us"
              % (name, ms, en.max(), st.max(), np.median(st), np.median(en - st), np.percentile(en - st, 10),
                 np.percentile(en - st, 90), np.median(en), en.max()))
        # by XCD (dispatch order: linear workgroup id mod 8) and by tile (the kernels' XCD remap
        # gives XCD x the tiles x*n/8 .. (x+1)*n/8 - 1)
        lt = en - st
        ids = np.arange(nwg)
        print("    lifetime by XCD (id %% 8): " + " ".join("%.1f" % np.median(lt[ids % 8 == x]) for x in range(8)))
        print("    lifetime by 1/8 of the tile range: " + " ".join(
            "%.1f" % np.median(lt[(ids // max(1, nwg // 8)) == x]) for x in range(8)))
        print("    slowest 8 ids: %s" % list(np.argsort(lt)[-8:]))
        return
    ok = dr > 0
    clk = np.median(dt[ok] / dr[ok]) * 100.0          # MHz
    tf = flops / ms / 1e9
    print("%-34s %5d launches  %.3f ms  %6.1f TF/s  frac %.3f at 2.4 GHz  clock %6.0f MHz (p10 %.0f p90 %.0f)"
          "  frac %.3f at that clock  wg cycles median %.0f"
          % (name, n, ms, tf, tf / SPLIT_PEAK, clk, np.percentile(dt[ok] / dr[ok] * 100, 10),
             np.percentile(dt[ok] / dr[ok] * 100, 90), tf / (SPLIT_PEAK * clk / 2400.0), np.median(dt[ok])))


def main():
    seconds = float(sys.argv[1]) if len(sys.argv) > 1 else 3.0
    lib = _lib.lib()
    if not hasattr(lib, "ubpl_debug_clock_stamps"):
        raise SystemExit("not a UBPL_CLOCK_STAMP build (set UBPL_LIB_DIR)")
    lib.ubpl_debug_clock_stamps4.argtypes = [ctypes.c_void_p, ctypes.c_int]
    lib.ubpl_debug_clock_stamps4.restype = ctypes.c_int
    lib.ubpl_debug_clock_stamps.argtypes = [ctypes.c_void_p, ctypes.c_int]
    lib.ubpl_debug_clock_stamps.restype = ctypes.c_int
    dev = torch.device("cuda", 0)
    g = torch.Generator(device=dev).manual_seed(0)
    B, C, H = 32, 128, 64
    x = torch.randn(B, C, H, H, device=dev, generator=g)
    w = torch.randn(C, C, 3, 3, device=dev, generator=g) / 34.0
    b = torch.randn(C, device=dev, generator=g)
    xs, ws = Kn.split_activation(x, 3, 1), Kn.conv_weight_split(w, 0, 3)
    y = torch.empty(B, C, H, H, device=dev)
    probe("3x3 128->128 64x64 B=32 (psah)", lambda: Kn.conv2d_forward_psa(xs, ws, b, out=y),
          B * H * H // 256, 2.0 * B * C * C * 9 * H * H, seconds, lib)
    for cin, cout in ((256, 128), (128, 256)):
        x1 = torch.randn(B, cin, H, H, device=dev, generator=g)
        w1 = torch.randn(cout, cin, 1, 1, device=dev, generator=g) / 16.0
        b1 = torch.randn(cout, device=dev, generator=g)
        w1s = Kn.conv_weight_split(w1, 0, 3)
        y1 = torch.empty(B, cout, H, H, device=dev)
        probe("1x1 %d->%d 64x64 B=32 (sol)" % (cin, cout),
              lambda: Kn.conv1x1_forward_split_load(x1, w1s, b1, out=y1),
              (B * H * H // 256) * (cout // 128), 2.0 * B * cout * cin * H * H, seconds, lib)


if __name__ == "__main__":
    main()

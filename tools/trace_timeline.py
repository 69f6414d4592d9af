"""Step timeline of a rocprofv3 kernel trace: busy union, concurrency, grid-size buckets, per-kernel
totals over the timed window (steps delimited by the fused AdamW+EMA launches, 2 per step).

    python tools/trace_timeline.py run_kernel_trace.csv FIRST_STEP LAST_STEP
"""
import csv, re, sys, collections
rows = list(csv.DictReader(open(sys.argv[1])))
ks = []
for r in rows:
    n = r["Kernel_Name"]; m = re.search(r"::(\w+)(<[^(]*>)?\(", n); kn = m.group(1) if m else n[:40]
    ks.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), kn, int(r["Queue_Id"]), int(r["Grid_Size_X"])*int(r["Grid_Size_Y"])*int(r["Grid_Size_Z"])//max(1,int(r["Workgroup_Size_X"])*int(r["Workgroup_Size_Y"])*int(r["Workgroup_Size_Z"]))))
ks.sort()
ad = [k for k in ks if k[2].startswith("adamw_ema")]
print("adamw launches", len(ad))
w0, w1 = int(sys.argv[2]), int(sys.argv[3])     # step indices (adamw pairs)
t0 = ad[2*w0-1][1]; t1 = ad[2*w1-1][1]
win = [k for k in ks if k[0] >= t0 and k[1] <= t1]
nsteps = w1 - w0
print("window ms/step %.2f, kernels/step %d" % ((t1-t0)/1e6/nsteps, len(win)/nsteps))
# union busy
busy=0; cur_s=None; cur_e=None
for s,e,_,_,_ in win:
    if cur_e is None or s > cur_e:
        if cur_e is not None: busy += cur_e-cur_s
        cur_s, cur_e = s, e
    else: cur_e = max(cur_e, e)
busy += cur_e-cur_s
print("busy union ms/step %.2f (%.1f%%)" % (busy/1e6/nsteps, 100*busy/(t1-t0)))
tot = sum(e-s for s,e,_,_,_ in win)
print("sum kernel ms/step %.2f, avg concurrency %.2f" % (tot/1e6/nsteps, tot/busy))
# by grid size buckets
b = collections.defaultdict(float); bn = collections.defaultdict(int)
for s,e,kn,q,g in win:
    key = "<64" if g < 64 else "<256" if g < 256 else "<1024" if g < 1024 else ">=1024"
    b[key] += e-s; bn[key]+=1
for k in ["<64","<256","<1024",">=1024"]:
    print("grid %6s: %7.2f ms/step kernel time, %5d launches/step, avg %.1f us" % (k, b[k]/1e6/nsteps, bn[k]//nsteps, b[k]/max(1,bn[k])/1e3))
# per queue busy
qb = collections.defaultdict(float)
for s,e,kn,q,g in win: qb[q]+= e-s
print("per-queue kernel ms/step", {q: round(v/1e6/nsteps,1) for q,v in sorted(qb.items())})
# small-grid kernels by name
sm = collections.defaultdict(float); smn = collections.defaultdict(int)
for s,e,kn,q,g in win:
    if g < 256: sm[kn]+=e-s; smn[kn]+=1
for k,v in sorted(sm.items(), key=lambda kv:-kv[1])[:12]:
    print("  small-grid %-28s %6.2f ms/step %4d/step avg %.1f us" % (k, v/1e6/nsteps, smn[k]//nsteps, v/smn[k]/1e3))
fam = collections.defaultdict(float); famn = collections.defaultdict(int)
for s,e,kn,q,g in win: fam[kn]+=e-s; famn[kn]+=1
print("--- by kernel (timed window)")
for k,v in sorted(fam.items(), key=lambda kv:-kv[1])[:24]:
    print("  %-34s %6.2f ms/step %4d/step avg %6.1f us" % (k, v/1e6/nsteps, famn[k]//nsteps, v/famn[k]/1e3))

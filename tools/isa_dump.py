"""Disassemble the gfx950 code objects of libubpl_hip.so (or another HIP .so)
into one text file, and report per kernel its scratch (spill) instructions:

    python tools/isa_dump.py [lib.so] [out.s] [kernel-substring]
"""
import collections
import os
import re
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tests"))
sys.path.insert(0, os.path.join(ROOT, "tests", "golden"))
sys.path.insert(0, os.path.join(ROOT, "ubpl-poseestimation_amd"))


def main():
    from test_cpu_host import _gfx950_code_objects
    lib = sys.argv[1] if len(sys.argv) > 1 else os.path.join(ROOT, "ubpl-poseestimation_amd", "ubpl_amd",
                                                              "libubpl_hip.so")
    out = sys.argv[2] if len(sys.argv) > 2 else "/tmp/ubpl_isa.s"
    pat = sys.argv[3] if len(sys.argv) > 3 else ""
    with open(out, "w") as fo:
        for i, co in enumerate(_gfx950_code_objects(lib)):
            p = "/tmp/_co%d" % i
            open(p, "wb").write(co)
            fo.write(subprocess.run(["/opt/rocm/lib/llvm/bin/llvm-objdump", "-d", "--mcpu=gfx950", p],
                                    capture_output=True, text=True, check=True).stdout)
    c = collections.Counter()
    fn = None
    for line in open(out):
        m = re.match(r"^[0-9a-f]+ <(.*)>:$", line)
        if m:
            fn = m.group(1)
        elif "scratch_" in line and pat in (fn or ""):
            c[fn] += 1
    for f, n in c.most_common(40):
        dm = subprocess.run(["c++filt", f], capture_output=True, text=True).stdout.strip()
        print("%5d scratch ops  %s" % (n, dm[:150]))


if __name__ == "__main__":
    main()

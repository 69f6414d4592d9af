"""Do torch's RCCL gfx950 kernels use packed-FP32 VALU instructions?

The round-4 fault: v_pk_add_f32 mis-executed while other
queues ran bf16 matrix work beside it.  Our library is built without packed
FP32 (csrc/Makefile NOPK) and no PyTorch arithmetic runs beside the network
streams (train._backward_all); an RCCL reduce kernel enqueued on a student's
stream while other networks' backward runs (train._AR_OVERLAP) would break
that invariant if RCCL's reduce kernels carry the same instructions.

torch's librccl.so holds ONE compressed clang offload bundle (CCOB v2, zstd)
in .hip_fatbin; clang-offload-bundler decompresses it.  This script extracts
the gfx950 code object, disassembles it and counts v_pk_{add,mul,fma}_f32 per
kernel.  Output: a text record (profiles/r05_rccl_packed_fp32.txt).

    python tools/rccl_pk_check.py [librccl.so] > profiles/r05_rccl_packed_fp32.txt
"""
import collections
import os
import re
import struct
import subprocess
import sys
import tempfile

LLVM = "/opt/rocm/lib/llvm/bin"


def fatbin(path):
    d = open(path, "rb").read()
    shoff, = struct.unpack_from("<Q", d, 0x28)
    shentsize, shnum, shstrndx = struct.unpack_from("<HHH", d, 0x3A)
    secs = [struct.unpack_from("<IIQQQQ", d, shoff + i * shentsize) for i in range(shnum)]
    stroff = secs[shstrndx][4]
    for name, _, _, _, off, size in secs:
        if d[stroff + name:d.index(b"\0", stroff + name)] == b".hip_fatbin":
            return d[off:off + size]
    raise SystemExit("no .hip_fatbin in %s" % path)


def main():
    import torch
    path = sys.argv[1] if len(sys.argv) > 1 else os.path.join(os.path.dirname(torch.__file__), "lib", "librccl.so")
    fb = fatbin(path)
    with tempfile.TemporaryDirectory(dir="/tmp") as td:
        fbp = os.path.join(td, "fb.bin")
        open(fbp, "wb").write(fb)
        targets = subprocess.run([LLVM + "/clang-offload-bundler", "--list", "--type=o", "--input=" + fbp],
                                 capture_output=True, text=True, check=True).stdout.split()
        t950 = [t for t in targets if t.endswith("gfx950")]
        print("library: %s" % path)
        print("fatbin: %d bytes, CCOB (compressed) bundles: %d, plain bundles: %d"
              % (len(fb), fb.count(b"CCOB"), fb.count(b"__CLANG_OFFLOAD_BUNDLE__")))
        print("gfx950 targets: %s" % t950)
        per = collections.Counter()
        n_kernels = 0
        for t in t950:
            co = os.path.join(td, "co")
            subprocess.run([LLVM + "/clang-offload-bundler", "--unbundle", "--type=o", "--input=" + fbp,
                            "--output=" + co, "--targets=" + t], check=True)
            p = subprocess.Popen([LLVM + "/llvm-objdump", "-d", "--mcpu=gfx950", co], stdout=subprocess.PIPE,
                                 text=True)
            fn = None
            for line in p.stdout:
                m = re.match(r"^[0-9a-f]+ <(.*)>:$", line)
                if m:
                    fn = m.group(1)
                    continue
                if "s_endpgm" in line:
                    n_kernels += 1
                if re.search(r"v_pk_(?:add|mul|fma)_f32", line):
                    per[fn] += 1
            p.wait()
        print("s_endpgm: %d; packed-FP32 instructions: %d in %d functions" % (n_kernels, sum(per.values()), len(per)))
        for fn, c in per.most_common():
            dm = subprocess.run(["c++filt", fn], capture_output=True, text=True).stdout.strip()
            print("%5d  %s" % (c, dm[:160]))


if __name__ == "__main__":
    main()

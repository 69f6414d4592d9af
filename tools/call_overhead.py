"""Host cost of one C-ABI launch: through its torch op (the product path) vs
ctypes on the C entry (round 1's binding).  Small tensors: the GPU is idle,
the host is what is measured."""
import ctypes
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "ubpl-poseestimation_amd")]
import torch  # noqa: E402
from ubpl_amd import _lib  # noqa: E402

a = torch.ones(1024, device="cuda")
b = torch.ones(1024, device="cuda")
o = torch.empty(1024, device="cuda")
op = _lib.op("ubpl_add")
c = _lib.lib().ubpl_add
N = 20000
for name, f in (("torch op", lambda: op(a, b, 1024, o)),
                ("ctypes", lambda: c(a.data_ptr(), b.data_ptr(), 1024, o.data_ptr(),
                                     ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)))):
    for _ in range(200):
        f()
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(N):
        f()
    dt = time.perf_counter() - t
    torch.cuda.synchronize()
    print("%-9s %.2f us per launch (host)" % (name, dt / N * 1e6))

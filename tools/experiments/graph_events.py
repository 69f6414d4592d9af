"""Can timing events be recorded inside a captured HIP graph (torch)?"""
import torch

x = torch.randn(4096, 4096, device="cuda")
y = torch.empty_like(x)
s = torch.cuda.Stream()
s.wait_stream(torch.cuda.current_stream())
with torch.cuda.stream(s):
    for _ in range(2):
        torch.mm(x, x, out=y)
torch.cuda.current_stream().wait_stream(s)
g = torch.cuda.CUDAGraph()
evs = []
try:
    with torch.cuda.graph(g):
        for _ in range(3):
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record()
            torch.mm(x, x, out=y)
            b.record()
            evs.append((a, b))
    for _ in range(2):
        g.replay()
    torch.cuda.synchronize()
    print("captured events ok:", [round(a.elapsed_time(b), 4) for a, b in evs])
except Exception as e:  # noqa: BLE001
    print("captured events FAILED:", type(e).__name__, str(e)[:300])

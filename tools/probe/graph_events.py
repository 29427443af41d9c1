"""Probe: can timing events be recorded inside a captured HIP graph and read after replay?"""
import torch

x = torch.randn(4096, 4096, device="cuda")
y = torch.empty_like(x)
s = torch.cuda.Stream()
with torch.cuda.stream(s):
    torch.mm(x, x, out=y)
    torch.mm(y, x, out=y)
torch.cuda.synchronize()
res = {}
for ext in (True, False):
    try:
        evs = [torch.cuda.Event(enable_timing=True, external=ext) for _ in range(4)]
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g, stream=s):
            evs[0].record()
            torch.mm(x, x, out=y)
            evs[1].record()
            torch.mm(y, x, out=y)
            evs[2].record()
        g.replay()
        torch.cuda.synchronize()
        res[ext] = [evs[0].elapsed_time(evs[1]), evs[1].elapsed_time(evs[2])]
        g.replay(); torch.cuda.synchronize()
        res[str(ext) + "_2"] = [evs[0].elapsed_time(evs[1]), evs[1].elapsed_time(evs[2])]
    except Exception as e:
        res[ext] = f"{type(e).__name__}: {e}"
print(res)

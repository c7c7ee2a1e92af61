"""Probe: an external event recorded INSIDE a captured HIP graph gates work on another stream
issued after the replay (the trainer's bucketed gradient all-reduce overlap relies on it).
Prints whether the side-stream copy saw the in-graph producer's data and whether it finished
before the rest of the graph."""
import torch

dev = torch.device("cuda", 0)
a = torch.zeros(1 << 20, device=dev)
x = torch.randn(4096, 4096, device=dev)
ev = torch.cuda.Event(external=True)
side = torch.cuda.Stream(device=dev)
g = torch.cuda.CUDAGraph()
s = torch.cuda.Stream(device=dev)
s.wait_stream(torch.cuda.current_stream())
with torch.cuda.stream(s):
    y = x @ x
torch.cuda.current_stream().wait_stream(s)
with torch.cuda.graph(g):
    a.add_(1.0)            # producer of the "bucket"
    ev.record()
    for _ in range(20):    # the rest of the backward
        y = y @ x * 1e-3
for it in range(3):
    out = torch.empty_like(a)
    t0, t1, t2 = (torch.cuda.Event(enable_timing=True) for _ in range(3))
    t0.record()
    g.replay()
    t1.record()
    side.wait_event(ev)
    with torch.cuda.stream(side):
        out.copy_(a)
        ts = torch.cuda.Event(enable_timing=True)
        ts.record()
    torch.cuda.synchronize()
    print(f"replay {it}: side copy saw {out[0].item():.0f} (want {it + 1}), side done at "
          f"{t0.elapsed_time(ts):.3f} ms, graph done at {t0.elapsed_time(t1):.3f} ms")

"""When does the second branch of a captured two-branch graph start?  (GPU box, under
rocprofv3 --kernel-trace; tools/trace_path.py reads the per-queue start times)
    python tools/probe/graph_gate.py NA
Branch A: NA sleep kernels (~20 us each) forked onto a side stream first (the pipelined step's
encoder branch); branch B: 5 short sleep kernels on the capturing stream (the decoder branch).
The C3 step's decoder branch started after ~47-48 encoder kernels in rounds 4 and 5."""
import sys

import torch

NA = int(sys.argv[1]) if len(sys.argv) > 1 else 100
dev = torch.device("cuda:0")
side, cap = torch.cuda.Stream(), torch.cuda.Stream()
x = torch.zeros(1024, device=dev)
g = torch.cuda.CUDAGraph()
with torch.cuda.stream(cap):
    g.capture_begin()
    cur = torch.cuda.current_stream()
    x.add_(1)
    side.wait_stream(cur)
    with torch.cuda.stream(side):
        for _ in range(NA):
            torch.cuda._sleep(40_000)
    for _ in range(5):
        x.mul_(1.0001)
    cur.wait_stream(side)
    g.capture_end()
torch.cuda.synchronize()
for _ in range(5):
    g.replay()
torch.cuda.synchronize()
print("done", NA, flush=True)

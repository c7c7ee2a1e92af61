"""When does the second branch of a captured two-branch graph start?  (GPU box, under
rocprofv3 --kernel-trace; tools/trace_path.py reads the per-queue start times)
    python tools/probe/graph_gate.py NA
Branch A: NA sleep kernels (~20 us each) forked onto a side stream first (the pipelined step's
encoder branch); branch B: 5 short sleep kernels on the capturing stream (the decoder branch).
The C3 step's decoder branch started after ~47-48 encoder kernels in rounds 4 and 5."""
import sys

import torch

NA = int(sys.argv[1]) if len(sys.argv) > 1 else 100
KIND = sys.argv[2] if len(sys.argv) > 2 else "sleep"  # "sleep": one block each; "wide": grid-filling
dev = torch.device("cuda:0")
big = torch.ones(64 << 20, device=dev)  # 256 MB: a grid-filling elementwise kernel of ~60 us
side, cap = torch.cuda.Stream(), torch.cuda.Stream()
x = torch.zeros(1024, device=dev)
g = torch.cuda.CUDAGraph()
with torch.cuda.stream(cap):
    g.capture_begin()
    cur = torch.cuda.current_stream()
    x.add_(1)
    side.wait_stream(cur)
    ORDER = sys.argv[3] if len(sys.argv) > 3 else "afirst"

    def branch_a():
        with torch.cuda.stream(side):
            for _ in range(NA):
                if KIND == "sleep":
                    torch.cuda._sleep(40_000)
                else:
                    big.mul_(1.0000001)

    def branch_b():
        for _ in range(5):
            x.mul_(1.0001)
    if ORDER == "afirst":
        branch_a()
        branch_b()
    else:
        branch_b()
        branch_a()
    cur.wait_stream(side)
    g.capture_end()
torch.cuda.synchronize()
for _ in range(5):
    g.replay()
torch.cuda.synchronize()
print("done", NA, flush=True)

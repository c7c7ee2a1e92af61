"""Host-side cost of one pipelined C3 step (graph replay): time of trainer.step() on the host
without synchronising, against the device time per step.  If the host time per step is close
to the device's, the replay is host-bound (GPU box):  python tools/probe/host_replay.py [C3]"""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import bench  # noqa: E402
from imagecaptioningconvnext_amd.train_step import TeacherForcedTrainer  # noqa: E402

cfg = dict(bench.CONFIGS[sys.argv[1] if len(sys.argv) > 1 else "C3"])
dev = torch.device("cuda:0")
enc, dec = bench.build(cfg, dev)
tr = TeacherForcedTrainer(enc, dec, lstm=cfg["decoder"] == "lstm", graph=True, pipeline=True)
B = cfg["batch"]
batches = [bench.synthetic_batch(B, 0, i, dev) for i in range(4)]
for i in range(8):
    tr.step(*batches[i % 4][:3], max_caplen=batches[i % 4][3])
torch.cuda.synchronize()
n = 30
host = []
t0 = time.perf_counter()
for i in range(n):
    h0 = time.perf_counter()
    tr.step(*batches[i % 4][:3], max_caplen=batches[i % 4][3])
    host.append(time.perf_counter() - h0)
torch.cuda.synchronize()
wall = (time.perf_counter() - t0) / n
host.sort()
print(f"per step: wall {wall * 1e3:.3f} ms, host step() median {host[n // 2] * 1e3:.3f} ms "
      f"(min {host[0] * 1e3:.3f}, max {host[-1] * 1e3:.3f})", flush=True)
g = tr._pipe["sets"][next(iter(tr._pipe["sets"]))]["graphs"][0]
torch.cuda.synchronize()
r = []
for i in range(10):
    h0 = time.perf_counter()
    g.replay()
    r.append(time.perf_counter() - h0)
    torch.cuda.synchronize()
r.sort()
print(f"bare graph.replay() host time: median {r[5] * 1e3:.3f} ms", flush=True)

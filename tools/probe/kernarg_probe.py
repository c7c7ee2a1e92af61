"""Do captured graphs keep their kernel arguments intact across replays?  (GPU box; never faults:
the probe kernels only compare their by-value argument words and count mismatches.)

    hipcc --offload-arch=gfx950 -O2 -shared -fPIC tools/probe/kernarg_probe.hip -o tools/probe/kernarg_probe.so
    python tools/probe/kernarg_probe.py

Schedules, each replayed 6 times in order, ids distinct per node:
  split    g1 = 80 canary nodes, g2 = ONE big node (3.3 KB argument), g1 and g2 sharing a pool
           (the captured DDP decoder split: g2 = imgcap_colsum_multi alone)
  split1k  the same with a 1 KB big node
  whole    one graph: 80 canaries + the big node last
  split_ft g1 = 80 canaries + big node last, g2 = 40 canaries (the fine-tuned split)
"""
import ctypes
import os

import torch

HERE = os.path.dirname(os.path.abspath(__file__))
lib = ctypes.CDLL(os.path.join(HERE, "kernarg_probe.so"))
lib.probe_canary.argtypes = [ctypes.c_uint, ctypes.c_void_p]
lib.probe_big.argtypes = [ctypes.c_uint, ctypes.c_int, ctypes.c_void_p]
lib.probe_read.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int]

dev = torch.device("cuda:0")
torch.zeros(1, device=dev)
NID = 4096


def canaries(ids):
    st = torch.cuda.current_stream().cuda_stream
    for i in ids:
        assert lib.probe_canary(i, st) == 0


def big(i, words):
    assert lib.probe_big(i, words, torch.cuda.current_stream().cuda_stream) == 0


def read():
    torch.cuda.synchronize()
    bad = (ctypes.c_uint * NID)()
    runs = (ctypes.c_uint * NID)()
    assert lib.probe_read(bad, runs, NID) == 0
    return list(bad), list(runs)


def capture(fn, pool=None):
    g = torch.cuda.CUDAGraph()
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        g.capture_begin(pool=pool)
        fn()
        g.capture_end()
    torch.cuda.current_stream().wait_stream(s)
    return g


def run(name, graphs, ids, reps=6):
    b0, r0 = read()
    for _ in range(reps):
        for g in graphs:
            g.replay()
        torch.cuda.synchronize()
        torch.empty(64 << 20, device=dev).fill_(1.0)  # eager work between replays
    b1, r1 = read()
    bad = {i: b1[i] - b0[i] for i in ids if b1[i] != b0[i]}
    runs = {r1[i] - r0[i] for i in ids}
    print(f"{name}: nodes {len(ids)}, runs per node {sorted(runs)}, corrupted argument words "
          f"{sum(bad.values())} in {len(bad)} nodes {sorted(bad)[:12]}", flush=True)


base = 0
# split: g1 = 80 canaries, g2 = one 3.3 KB node
ids1 = list(range(base, base + 80))
g1 = capture(lambda: canaries(ids1))
g2 = capture(lambda: big(base + 80, 840), pool=g1.pool())
run("split", [g1, g2], ids1 + [base + 80])
base += 100
ids1 = list(range(base, base + 80))
h1 = capture(lambda: canaries(ids1))
h2 = capture(lambda: big(base + 80, 256), pool=h1.pool())
run("split1k", [h1, h2], ids1 + [base + 80])
base += 100
ids1 = list(range(base, base + 80))
w = capture(lambda: (canaries(ids1), big(base + 80, 840)))
run("whole", [w], ids1 + [base + 80])
base += 100
ids1 = list(range(base, base + 80))
ids2 = list(range(base + 81, base + 121))
f1 = capture(lambda: (canaries(ids1), big(base + 80, 840)))
f2 = capture(lambda: canaries(ids2), pool=f1.pool())
run("split_ft", [f1, f2], ids1 + [base + 80] + ids2)
base += 200
ids1 = list(range(base, base + 80))
k1 = capture(lambda: canaries(ids1))
k2 = capture(lambda: big(base + 80, 920), pool=k1.pool())
run("split_3.6k", [k1, k2], ids1 + [base + 80])
print("kernarg probe done", flush=True)

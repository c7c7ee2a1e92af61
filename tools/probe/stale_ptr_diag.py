"""Which device pointers does a captured train step hand to the library that are NOT live
allocations when the capture ends (GPU box, no replay, nothing faults):
    python tools/probe/stale_ptr_diag.py C4
Every imgcap_* call made during the sequential-schedule capture is recorded with every pointer
it passes (plain arguments and the fields of ctypes descriptors / arrays); after the capture each
pointer is looked up in torch.cuda.memory_snapshot(): a pointer inside an inactive block (freed,
or never allocated) is a stale argument baked into the graph."""
import ctypes
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
import bench  # noqa: E402
from imagecaptioningconvnext_amd import _abi  # noqa: E402
from imagecaptioningconvnext_amd import kernels as K  # noqa: E402
from imagecaptioningconvnext_amd.train_step import TeacherForcedTrainer  # noqa: E402

name = sys.argv[1] if len(sys.argv) > 1 else "C4"
cfg = bench.CONFIGS[name]
dev = torch.device("cuda:0")
torch.manual_seed(42)
enc, dec = bench.build(cfg, dev)
tr = TeacherForcedTrainer(enc, dec, lstm=cfg["decoder"] == "lstm", graph=True)
imgs, caps, lens = bench.synthetic_batch(cfg["batch"], 0, 0, dev)[:3]

rec = []
orig = _abi.call


def ptrs_of(a, depth=0):
    out = []
    if isinstance(a, int):
        if a > (1 << 32):
            out.append(a)
    elif isinstance(a, ctypes.c_void_p):
        if a.value and a.value > (1 << 32):
            out.append(a.value)
    elif hasattr(a, "_obj"):  # byref(...)
        out += ptrs_of(a._obj, depth + 1)
    elif isinstance(a, ctypes.Array) and depth < 3:
        for e in a:
            out += ptrs_of(e, depth + 1)
    elif isinstance(a, ctypes.Structure) and depth < 3:
        for f, _ in a._fields_:
            out += ptrs_of(getattr(a, f), depth + 1)
    return out


capturing = [False]


def call(fn, *args):
    if capturing[0]:
        ps = []
        for a in args:
            ps += ptrs_of(a)
        if fn in ("imgcap_colsum_multi", "imgcap_gemm_grouped"):  # array passed as a cast pointer
            ps = ps[:-1] if ps else ps
        rec.append((fn, ps))
    return orig(fn, *args)


_abi.call = call
tr._seed_ctr = torch.zeros(1, dtype=torch.int64, device=dev)
K.set_seed_counter(tr._seed_ctr)
tr._inputs = (imgs.clone(), caps.clone(), lens.clone())
side = torch.cuda.Stream(device=dev)
side.wait_stream(torch.cuda.current_stream(dev))
with torch.cuda.stream(side):
    for i in range(2):
        tr._fwd_bwd(*tr._inputs)
torch.cuda.current_stream(dev).wait_stream(side)
torch.cuda.synchronize()
g = torch.cuda.CUDAGraph()
with torch.cuda.graph(g):
    capturing[0] = True
    tr._seed_ctr.add_(1)
    m = tr._fwd_bwd(*tr._inputs)
    capturing[0] = False
torch.cuda.synchronize()
snap = torch.cuda.memory_snapshot()
blocks = []
for seg in snap:
    a = seg["address"]
    for b in seg["blocks"]:
        blocks.append((a, a + b["size"], b["state"], str(seg.get("segment_pool_id")), seg.get("stream")))
        a += b["size"]
blocks.sort()
import bisect  # noqa: E402
starts = [b[0] for b in blocks]
bad = {}
unknown = {}
for fn, ps in rec:
    for p in ps:
        i = bisect.bisect_right(starts, p) - 1
        if i < 0 or p >= blocks[i][1]:
            unknown.setdefault(fn, set()).add(hex(p))
            continue
        if blocks[i][2] != "active_allocated" and blocks[i][3] != str(g.pool()):
            bad.setdefault(fn, []).append((hex(p), blocks[i][2], blocks[i][3]))
print(f"{len(rec)} calls recorded during the capture; graph pool {g.pool()}")
print("pointers in NON-live blocks (stale):")
for fn, v in bad.items():
    print(" ", fn, v[:6])
print("pointers outside every torch segment (library-owned or foreign):")
for fn, v in unknown.items():
    print(" ", fn, sorted(v)[:6])
print("diag done")

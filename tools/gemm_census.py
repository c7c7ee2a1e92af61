"""Every GEMM of one train step at a bench config, timed in isolation (GPU box):
    python tools/gemm_census.py [C2|C3|C4|C5]
Prints one line per call (shape, operand layout, epilogue, plan, us, TFLOP/s) sorted by time."""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402
from imagecaptioningconvnext_amd import kernels as K  # noqa: E402
from tools.microbench import time_launch  # noqa: E402
from imagecaptioningconvnext_amd.train_step import TeacherForcedTrainer  # noqa: E402

cfgname = sys.argv[1] if len(sys.argv) > 1 else "C2"
cfg = bench.CONFIGS[cfgname]
dev = torch.device("cuda:0")
enc, dec = bench.build(cfg, dev)
tr = TeacherForcedTrainer(enc, dec, lstm=cfg["decoder"] == "lstm", graph=False)
batch = bench.synthetic_batch(cfg["batch"], 0, 0, dev)[:3]
tr.step(*batch)
rec = []
K.record_gemms(rec)
tr._fwd_bwd(*batch)
K.record_gemms(None)
torch.cuda.synchronize()
def torch_time(c, reps=20):
    """hipBLASLt (torch.matmul) on the same shape / operand layout, bf16 out, no epilogue:
    a calibration column only (the product never calls it)."""
    M, N, Kd = c["M"], c["N"], c["K"]
    a = torch.randn((M, Kd) if c["ak"] else (Kd, M), device=dev, dtype=torch.bfloat16)
    b = torch.randn((N, Kd) if c["bk"] else (Kd, N), device=dev, dtype=torch.bfloat16)
    aa = a if c["ak"] else a.t()
    bb = b.t() if c["bk"] else b
    out = torch.matmul(aa, bb)
    side = torch.cuda.Stream()
    side.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(side):  # warm hipBLASLt's heuristics / workspace outside the capture
        for _ in range(3):
            torch.matmul(aa, bb, out=out)
    torch.cuda.current_stream().wait_stream(side)
    g = torch.cuda.CUDAGraph()  # replayed, so the host launch cost (~18 us per eager call) is out
    with torch.cuda.graph(g):
        for _ in range(reps):
            torch.matmul(aa, bb, out=out)
    g.replay()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    g.replay()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps * 1e-3


rows = []
for c in rec:
    kind, sp = K.gemm_plan(c["dtype"], c["ak"], c["bk"], c["M"], c["N"], c["K"], c["lda"], c["ldb"], 1, c["split_k"])
    ep = c["keep"][-1]
    t = time_launch(c["call"], reps=20, warm=2)
    rows.append((t, c, kind, sp, ep, torch_time(c)))
tot = sum(r[0] for r in rows)
print(f"{cfgname}: {len(rows)} GEMM calls, {tot * 1e6:.1f} us in isolation")
print(f"hipBLASLt (torch.matmul, same shapes, no epilogue): {sum(r[5] for r in rows) * 1e6:.1f} us")
for t, c, kind, sp, ep, tt in sorted(rows, key=lambda r: -r[0]):
    f = 2.0 * c["M"] * c["N"] * c["K"]
    print(f"{t * 1e6:8.1f} us {f / t / 1e12:7.1f} TF  M={c['M']:6d} N={c['N']:5d} K={c['K']:5d} "
          f"ak={c['ak']} bk={c['bk']} act={ep.act} c={'f32' if ep.c_dtype == 0 else 'bf16'} "
          f"bias={int(bool(ep.bias))} res={int(bool(ep.res))} beta={ep.beta:g} kind={kind} split={sp} "
          f"| blaslt {tt * 1e6:6.1f} us {f / tt / 1e12:6.1f} TF")

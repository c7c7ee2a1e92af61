"""Every GEMM one training step issues, timed under each imgcap_gemm_set_pt mode (GPU box):
    python tools/gemm_census.py [C3|C4|C2|C5] [reps]
Runs one eager (ungraphed, unpipelined) step of the bench's configuration with kernels.gemm
wrapped to record each call (operands, layout, epilogue), then replays every distinct call
back-to-back in a HIP graph under each mode (PT_MODES env, default the LDS-staged plan 0, the
stream-tile configs 4..7 and the by-shape plan -1).  Prints per call: count per step, layout,
epilogue kind, µs per mode; and per mode the step's GEMM total (count-weighted) -- the number a
plan change moves."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
from imagecaptioningconvnext_amd import kernels as K  # noqa: E402
from tools.microbench import time_launch  # noqa: E402

cfg_name = sys.argv[1] if len(sys.argv) > 1 else "C3"
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 10
MODES = [int(m) for m in os.environ.get("PT_MODES", "0 4 5 6 7 -1").split()]
dev = torch.device("cuda:0")

cfg = dict(bench.CONFIGS[cfg_name])
torch.manual_seed(42)
enc, dec = bench.build(cfg, dev)
from imagecaptioningconvnext_amd.train_step import TeacherForcedTrainer  # noqa: E402
tr = TeacherForcedTrainer(enc, dec, lstm=cfg["decoder"] == "lstm", graph=False, pipeline=False)
B = cfg["batch"]
batch = bench.synthetic_batch(B, 0, 0, dev)
tr.step(*batch[:3], max_caplen=batch[3])  # warm: workspaces, packs
torch.cuda.synchronize()

orig = K.gemm
calls = {}


def _key(a, b, kw):
    ep = "+".join(sorted(k for k, v in kw.items() if v is not None and k not in ("out", "out_dtype")
                         and not (k == "act" and v == K.ACT_NONE)))
    return (tuple(a.shape), tuple(a.stride()), tuple(b.shape), tuple(b.stride()), kw.get("trans_a", False),
            kw.get("trans_b", False), ep, kw.get("K"), kw.get("N"))


def rec(a, b, **kw):
    k = _key(a, b, kw)
    if k in calls:
        calls[k][2] += 1
    else:
        calls[k] = [a, b, 1, dict(kw)]
    return orig(a, b, **kw)


K.gemm = rec
tr.step(*batch[:3], max_caplen=batch[3])
torch.cuda.synchronize()
K.gemm = orig
tr.flush() if hasattr(tr, "flush") else None

tot = {m: 0.0 for m in MODES}
best_tot = 0.0
print(f"{cfg_name}: {len(calls)} distinct GEMM calls, {sum(c[2] for c in calls.values())} per step", flush=True)
print(f"{'M':>6s} {'N':>5s} {'K':>5s} {'ta':>2s}{'tb':>3s} {'n':>3s} {'epilogue':24s} | "
      + " ".join(f"{m:>7d}" for m in MODES) + " | us", flush=True)
for k, (a, b, n, kw) in sorted(calls.items(), key=lambda kv: -kv[1][2] * kv[1][0].numel() * kv[1][1].shape[0]):
    ta, tb = kw.get("trans_a", False), kw.get("trans_b", False)
    M = a.shape[1] if ta else a.shape[0]
    Kd = a.shape[0] if ta else a.shape[1]
    N = b.shape[0] if tb else b.shape[1]
    if kw.get("N") is not None:
        N = kw["N"]
    kw2 = dict(kw)
    if kw2.get("out") is None:  # one output for all replays (no allocation per launch)
        kw2["out"] = orig(a, b, **kw)
    row = []
    for m in MODES:
        with K.gemm_pt_mode(m):
            row.append(time_launch(lambda: orig(a, b, **kw2), reps=reps))
    for m, t in zip(MODES, row):
        tot[m] += n * t
    best_tot += n * min(row)
    print(f"{M:6d} {N:5d} {Kd:5d} {int(ta):2d}{int(tb):3d} {n:3d} {k[6][:24]:24s} | "
          + " ".join(f"{t * 1e6:7.1f}" for t in row), flush=True)
print("step GEMM total (us): " + "  ".join(f"mode {m}: {tot[m] * 1e6:.0f}" for m in MODES)
      + f"  best-of: {best_tot * 1e6:.0f}", flush=True)

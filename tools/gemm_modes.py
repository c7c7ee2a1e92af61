"""LDS-staged GEMM tile plans at the step's widest-gap shapes (GPU box):
    python tools/gemm_modes.py
One row per shape: us per launch for the plan by shape (-1), the 256x256 tile (1: BK 64 x 2
stages, 2: BK 32 x 4, 3: BK 32 x 3), 128x128 (4), 64x64 (6), 128x64 (7), and torch.matmul (hipBLASLt, no epilogue; calibration only)."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from imagecaptioningconvnext_amd import kernels as K  # noqa: E402
from tools.microbench import time_launch  # noqa: E402

dev = torch.device("cuda:0")
bf = torch.bfloat16
SHAPES = [(12544, 384, 1536, "res"), (12544, 1536, 384, "gelu"), (3136, 3072, 768, "gelu"), (3136, 768, 3072, "res"),
          (12544, 384, 768, "bias"), (3136, 768, 1536, "bias"),
          (6272, 2048, 512, "gelu"), (6272, 512, 2048, "res"), (25088, 1024, 256, "gelu"), (3328, 9490, 512, "bias"),
          (3328, 512, 512, "bias"), (3328, 1536, 512, "bias")]
MODES = tuple(int(m) for m in os.environ.get("MODES", "-1,1,2,3,4,6,7").split(","))
print(f"{'M':>6s} {'N':>5s} {'K':>5s} | " + " ".join(f"{m:>7d}" for m in MODES) + " | blaslt  (us)", flush=True)
for M, N, Kd, form in SHAPES:
    a = torch.randn(M, Kd, device=dev).to(bf)
    b = torch.randn(N, Kd, device=dev).to(bf)
    out = torch.empty(M, (N + 7) // 8 * 8, device=dev, dtype=bf)[:, :N]  # 16-byte rows, as the engines allocate
    bias = torch.randn(N, device=dev)
    kw = dict(bias=bias)
    if form == "gelu":
        kw["act"] = K.ACT_GELU
    elif form == "res":
        kw.update(colscale=torch.rand(N, device=dev), res=torch.randn(M, N, device=dev).to(bf))
    row = []
    for m in MODES:
        K.gemm_set_policy(m)
        try:
            row.append(time_launch(lambda: K.gemm(a, b, trans_b=True, out=out, **kw), reps=20))
        finally:
            K.gemm_set_policy(-1)
    tt = time_launch(lambda: torch.matmul(a, b.t()), reps=20)
    print(f"{M:6d} {N:5d} {Kd:5d} | " + " ".join(f"{t * 1e6:7.1f}" for t in row) + f" | {tt * 1e6:6.1f}", flush=True)

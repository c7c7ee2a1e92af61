"""Stream-tile GEMM vs the LDS-staged kernels vs hipBLASLt at the step's shapes (GPU box):
    python tools/pt_bench.py [reps]
Each row: one shape (forward nn.Linear form unless marked), µs per launch (graph replay of
back-to-back launches, random bf16 operands) for the LDS-staged plan (pt=0), the persistent
kernel with each tile config (2: 256x128, 3: 128x256, 4: 128x128, 5: 128x192), its cost-model pick (1) and 7: 128x128 with 128-deep k-steps, and
torch.matmul (hipBLASLt, no epilogue: a calibration column only)."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from imagecaptioningconvnext_amd import kernels as K  # noqa: E402
from tools.microbench import time_launch  # noqa: E402

dev = torch.device("cuda:0")
bf = torch.bfloat16
reps = int(sys.argv[1]) if len(sys.argv) > 1 else 20
# IMGCAP_GEMM_PT modes: 0 the LDS-staged plan, c + 1 stream-tile config c, 1 the cost-model pick (last)
NAMES = {0: "old", 2: "256x128", 3: "128x256", 4: "128x128", 5: "128x192", 6: "128x128b2", 7: "128x128k",
         8: "256x128w", 9: "256x256w", 10: "128x256w", 1: "auto"}
# (modes 2 / 3 need the diagnostic library: IMGCAP_LIB=build/libimgcap_hip_diag.so)
MODES = [int(m) for m in os.environ.get("PT_MODES", "0 4 5 6 7 1").split()]

SHAPES = [
    # C3 (Tiny, B=64) encoder
    ("C3 s3 pw1 +GELU", 12544, 1536, 384, "gelu"),
    ("C3 s3 pw2 +res", 12544, 384, 1536, "res"),
    ("C3 s4 pw1 +GELU", 3136, 3072, 768, "gelu"),
    ("C3 s4 pw2 +res", 3136, 768, 3072, "res"),
    ("C3 down2", 12544, 384, 768, "bias"),
    ("C3 down3", 3136, 768, 1536, "bias"),
    ("C3 enc_proj", 3136, 512, 768, "bias"),
    # C3 Transformer decoder (B*L = 3328)
    ("C3 in_proj", 3328, 1536, 512, "bias"),
    ("C3 ffn/out", 3328, 512, 512, "bias"),
    ("C3 mem kv", 3136, 1024, 512, "bias"),
    ("C3 vocab", 3328, 9490, 512, "bias"),
    # C4 (Base, B=32)
    ("C4 s3 pw1 +GELU", 6272, 2048, 512, "gelu"),
    ("C4 s3 pw2 +res", 6272, 512, 2048, "res"),
    ("C4 s4 pw1 +GELU", 1568, 4096, 1024, "gelu"),
    ("C4 s4 pw2 +res", 1568, 1024, 4096, "res"),
    ("C4 vocab", 1664, 9490, 512, "bias"),
    ("square 4096", 4096, 4096, 4096, "plain"),
]


def case(name, M, N, Kd, form):
    r8 = lambda x: (x + 7) // 8 * 8  # noqa: E731
    a = torch.randn(M, Kd, device=dev).to(bf)
    b = torch.randn(N, Kd, device=dev).to(bf)
    out = torch.empty(M, r8(N), device=dev, dtype=bf)[:, :N]
    bias = torch.randn(N, device=dev)
    cs = torch.rand(N, device=dev)
    res = torch.randn(M, r8(N), device=dev).to(bf)[:, :N]
    rs = torch.ones(M // 49 + 1, device=dev)
    kw = {}
    if form == "gelu":
        kw = dict(bias=bias, act=K.ACT_GELU)
    elif form == "res":
        kw = dict(bias=bias, colscale=cs, rowscale=rs, rows_per_scale=49, res=res)
    elif form == "bias":
        kw = dict(bias=bias)
    row = []
    for mode in MODES:
        K.gemm_set_pt(mode)
        try:
            t = time_launch(lambda: K.gemm(a, b, trans_b=True, out=out, **kw), reps=reps)
        finally:
            K.gemm_set_pt(-1)
        row.append(t)
    tt = time_launch(lambda: torch.matmul(a, b.t()), reps=reps)
    f = 2.0 * M * N * Kd
    cells = " ".join(f"{t * 1e6:7.1f}" for t in row)
    best = min(row[1:-1]) if len(row) > 2 else row[-1]
    print(f"{name:18s} {M:6d} {N:5d} {Kd:5d} | {cells} | blaslt {tt * 1e6:7.1f} | "
          f"old {f / row[0] / 1e12:6.0f} TF  st-best {f / best / 1e12:6.0f} TF  st-auto {f / row[-1] / 1e12:6.0f} TF "
          f"({row[0] / row[-1]:.2f}x)", flush=True)


print(f"{'shape':18s} {'M':>6s} {'N':>5s} {'K':>5s} | " + " ".join(f"{NAMES[m]:>7s}" for m in MODES) + " | us",
      flush=True)
for s in SHAPES:
    case(*s)

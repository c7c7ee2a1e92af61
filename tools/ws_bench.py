"""Weight-stationary short-K GEMM (imgcap_gemm_set_ws 1 / 2) vs the library's plan without it (ws 0)
at the C3 / C4 short-K shapes (GPU box): python tools/ws_bench.py [reps]
µs per launch (graph replay of back-to-back launches, random bf16 operands) and TFLOP/s."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from imagecaptioningconvnext_amd import kernels as K  # noqa: E402
from tools.microbench import time_launch  # noqa: E402

dev = torch.device("cuda:0")
bf = torch.bfloat16
reps = int(sys.argv[1]) if len(sys.argv) > 1 else 20
SHAPES = [
    ("C3 s3 pw1 +GELU", 12544, 1536, 384, "gelu"),
    ("C3 down1", 50176, 192, 384, "bias"),
    ("C3 in_proj", 3328, 1536, 512, "bias"),
    ("C3 d512 +ReLU", 3328, 512, 512, "relu"),
    ("C3 d512", 3328, 512, 512, "bias"),
    ("C3 mem kv x6", 3136, 6144, 512, "bias"),
    ("C3 vocab", 3328, 9490, 512, "bias"),
    ("C4 s3 pw1 +GELU", 6272, 2048, 512, "gelu"),
    ("C4 in_proj", 1664, 1536, 512, "bias"),
    ("C4 d512", 1664, 512, 512, "bias"),
    ("C2 s3 pw1 +GELU", 6272, 1536, 384, "gelu"),
]
if os.environ.get("WS_SHAPES"):  # "M,N,K,form;..."
    SHAPES = [("custom", *[int(x) for x in s.split(",")[:3]], s.split(",")[3]) for s in os.environ["WS_SHAPES"].split(";")]
for name, M, N, Kd, form in SHAPES:
    a = torch.randn(M, Kd, device=dev).to(bf)
    b = (torch.randn(N, Kd, device=dev) / Kd ** 0.5).to(bf)
    out = torch.empty(M, (N + 7) // 8 * 8, device=dev, dtype=bf)[:, :N]
    bias = torch.randn(N, device=dev)
    kw = dict(bias=bias)
    if form == "gelu":
        kw["act"] = K.ACT_GELU
    elif form == "relu":
        kw["act"] = K.ACT_RELU
    row = []
    for m in (0, 1, 2):
        with K.gemm_ws_mode(m):
            row.append(time_launch(lambda: K.gemm(a, b, trans_b=True, out=out, **kw), reps=reps))
    f = 2.0 * M * N * Kd
    print(f"{name:18s} {M:6d} {N:5d} {Kd:4d} | " + " ".join(f"{t * 1e6:7.1f}" for t in row) + " us | " +
          " ".join(f"{f / t / 1e12:5.0f}" for t in row) + " TF", flush=True)

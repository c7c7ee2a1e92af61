"""The Transformer decoder's dX products (dY W, transformerDecoder.py's Linears backward) with the
weight read as stored ([out][in], n-major for this product) vs a transposed copy (k-major), µs per
launch, C3 shapes (GPU box):  python tools/dx_layout_bench.py"""
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
from imagecaptioningconvnext_amd import kernels as K  # noqa: E402
from tools.microbench import time_launch  # noqa: E402

dev = torch.device("cuda:0")
bf = torch.bfloat16
M = 64 * 52
for (n_in, n_out) in ((512, 512), (512, 1536), (512, 2048)):
    dy = torch.randn(M, n_out, device=dev).to(bf)
    w = torch.randn(n_out, n_in, device=dev).to(bf)      # nn.Linear weight [out][in]
    wt = w.t().contiguous()                               # [in][out]: k-major for dX = dY W
    res = torch.randn(M, n_in, device=dev).to(bf)
    a = time_launch(lambda: K.gemm(dy, w), reps=40) * 1e6                     # B = W (k = out rows): n-major
    b = time_launch(lambda: K.gemm(dy, wt, trans_b=True), reps=40) * 1e6      # B = W^T rows: k-major
    c = time_launch(lambda: K.gemm(dy, w, out=res, beta=1.0), reps=40) * 1e6
    d = time_launch(lambda: K.gemm(dy, wt, trans_b=True, out=res, beta=1.0), reps=40) * 1e6
    print(f"M={M} N={n_in} K={n_out}: W as stored {a:6.2f} us, W^T copy {b:6.2f} us | +res: {c:6.2f} vs {d:6.2f}", flush=True)

# split-K on the long-K dX products (the default plan splits only past K = 2048 on small grids);
# fp32 out (split-K's form)
for (n_in, n_out) in ((512, 1536), (512, 2048), (512, 512)):
    dy = torch.randn(M, n_out, device=dev).to(bf)
    w = torch.randn(n_out, n_in, device=dev).to(bf)
    row = []
    for sk in (1, 2, 3, 4):
        t = time_launch(lambda: K.gemm(dy, w, split_k=sk, out_dtype=torch.float32), reps=40) * 1e6
        row.append(f"split {sk}: {t:6.2f}")
    print(f"M={M} N={n_in} K={n_out}: " + ", ".join(row), flush=True)

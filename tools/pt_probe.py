"""Persistent-tile GEMM probe (GPU box): µs per launch of tile configs 2/3/4 (and the LDS-staged
plan, pt=0) at a few step shapes; run under IMGCAP_PT_DBG (1: no MFMA, 2: no operand DMA) and
IMGCAP_PT_GRID=1 (one block per tile) to split its time."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from imagecaptioningconvnext_amd import kernels as K  # noqa: E402
from tools.microbench import time_launch  # noqa: E402

dev = torch.device("cuda:0")
bf = torch.bfloat16
tag = sys.argv[1] if len(sys.argv) > 1 else ""
for (M, N, Kd) in [(12544, 1536, 384), (12544, 384, 1536), (3136, 768, 3072), (4096, 4096, 4096)]:
    a = torch.randn(M, Kd, device=dev).to(bf)
    b = torch.randn(N, Kd, device=dev).to(bf)
    out = torch.empty(M, N, device=dev, dtype=bf)
    row = []
    for mode in (0, 2, 3, 4):
        with K.gemm_pt_mode(mode):
            row.append(time_launch(lambda: K.gemm(a, b, trans_b=True, out=out), reps=10))
    f = 2.0 * M * N * Kd
    print(f"{tag:10s} {M:6d} {N:5d} {Kd:5d} | " + " ".join(f"{t * 1e6:7.1f}" for t in row) + " us | " +
          " ".join(f"{f / t / 1e12:5.0f}" for t in row) + " TF", flush=True)

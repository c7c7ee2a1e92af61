"""LayerNorm2d + 2x2 patchify (imgcap_ln_patchify2) at the downsample shapes (GPU box):
    python tools/lnp_bench.py
us per launch and algorithmic HBM rate (read x once, write the patch rows once)."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from imagecaptioningconvnext_amd import kernels as K  # noqa: E402
from tools.microbench import time_launch  # noqa: E402

dev = torch.device("cuda:0")
for B, H, C in [(64, 56, 96), (64, 28, 192), (64, 14, 384), (32, 56, 128), (64, 56, 192), (64, 28, 384)]:
    x = torch.randn(B, H, H, C, device=dev).bfloat16()
    lw, lb = torch.rand(C, device=dev), torch.rand(C, device=dev)
    out = torch.empty(B * (H // 2) ** 2, 4 * C, device=dev, dtype=torch.bfloat16)
    for cm in (False, True):
        t = time_launch(lambda: K.ln_patchify2(x, lw, lb, out, cmajor=cm), reps=50)
        byt = 2 * x.numel() * 2
        print(f"B={B:3d} H={H:3d} C={C:4d} cmajor={int(cm)}  {t * 1e6:7.1f} us  {byt / t / 1e12:5.2f} TB/s", flush=True)

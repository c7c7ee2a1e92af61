"""ConvNeXt stem (4x4/4 patch conv + LayerNorm, imgcap_convnext_stem) at the bench batches, µs per
launch, and its output checksum (GPU box; IMGCAP_STEM_PX=2/4 overrides the patches per thread,
by default 4 for C0 >= 128):  python tools/stem_bench.py"""
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
from imagecaptioningconvnext_amd import kernels as K  # noqa: E402
from tools.microbench import time_launch  # noqa: E402

dev = torch.device("cuda:0")
g = torch.Generator().manual_seed(0)
rows = []
for B, C0 in ((64, 96), (32, 96), (32, 128), (64, 192)):
    img = torch.randn(B, 3, 224, 224, generator=g).to(dev)
    w = (torch.randn(C0, 3, 4, 4, generator=g) * 0.1).to(dev)
    b, lw, lb = (torch.randn(C0, generator=g).to(dev) for _ in range(3))
    out = torch.empty(B, 56, 56, C0, device=dev, dtype=torch.bfloat16)
    t = time_launch(lambda: K.convnext_stem(img, w, b, lw, lb, out), reps=40) * 1e6
    rows.append(f"B={B} C0={C0}: {t:6.2f} us (sum {out.float().sum().item():.6e})")
print(f"PX={os.environ.get('IMGCAP_STEM_PX', 'default')}: " + " | ".join(rows), flush=True)

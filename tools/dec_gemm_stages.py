"""The decoder chain's GEMM shapes at C3 (B*L = 3328 rows, d = 512, ff = 2048) on the plan by
shape, one line per shape (GPU box); run under IMGCAP_GLDS64_STAGES=2/3/4 to compare the 64x64
tile's pipeline depth on these small grids:
    IMGCAP_GLDS64_STAGES=4 python tools/dec_gemm_stages.py"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from imagecaptioningconvnext_amd import kernels as K  # noqa: E402
from tools.microbench import time_launch  # noqa: E402

dev = torch.device("cuda:0")
bf = torch.bfloat16
BL, d, ff = 3328, 512, 2048
# (M, N, K, B stored [N, K] (x W^T) or [K, N], epilogue)
SHAPES = [(BL, d, d, True, "bias"), (BL, 3 * d, d, True, "bias"), (BL, ff, d, True, "relu"),
          (BL, d, ff, True, "bias"), (BL, d, d, False, "beta"), (BL, d, d, False, ""), (BL, d, 3 * d, False, "beta"),
          (BL, ff, d, False, "aux")]
tot = 0.0
for M, N, Kd, tb, form in SHAPES:
    a = torch.randn(M, Kd, device=dev).to(bf)
    b = (torch.randn(N, Kd, device=dev) if tb else torch.randn(Kd, N, device=dev)).to(bf)
    kw = {}
    if form in ("bias", "relu"):
        kw["bias"] = torch.randn(N, device=dev)
    if form == "relu":
        kw["act"] = K.ACT_RELU
    if form == "beta":
        kw.update(out=torch.randn(M, N, device=dev), beta=1.0)
    if form == "aux":
        kw.update(aux=torch.randn(M, N, device=dev).to(bf), aux_scale=1.0 / 0.9)
    try:
        t = time_launch(lambda: K.gemm(a, b, trans_b=tb, **kw), reps=30) * 1e6
    except Exception as e:  # noqa: BLE001
        print(f"{M:5d} {N:5d} {Kd:5d} tb={int(tb)} {form:5s}: {e}", flush=True)
        continue
    tot += t
    print(f"{M:5d} {N:5d} {Kd:5d} tb={int(tb)} {form:5s}: {t:6.2f} us", flush=True)
print(f"stages={os.environ.get('IMGCAP_GLDS64_STAGES', '2')} total {tot:.1f} us", flush=True)

"""Launch one short-K GEMM shape a few times (rocprofv3 counter passes):
    python tools/ws_one.py M N K WS_MODE [reps] [gelu]   WS_MODE: imgcap_gemm_set_ws (0 = without)"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from imagecaptioningconvnext_amd import kernels as K  # noqa: E402

M, N, Kd, mode = (int(x) for x in sys.argv[1:5])
reps = int(sys.argv[5]) if len(sys.argv) > 5 else 5
act = K.ACT_GELU if len(sys.argv) > 6 and sys.argv[6] == "gelu" else K.ACT_NONE
dev = torch.device("cuda:0")
a = torch.randn(M, Kd, device=dev).to(torch.bfloat16)
b = (torch.randn(N, Kd, device=dev) / Kd ** 0.5).to(torch.bfloat16)
bias = torch.randn(N, device=dev)
out = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
K.gemm_set_ws(mode)
for _ in range(reps):
    K.gemm(a, b, trans_b=True, out=out, bias=bias, act=act)
torch.cuda.synchronize()

"""Launch one GEMM shape a few times (for rocprofv3 counter passes):
    python tools/pt_one.py M N K MODE [reps]     MODE: imgcap_gemm_set_pt mode (0 = the LDS-staged plan)"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from imagecaptioningconvnext_amd import kernels as K  # noqa: E402

M, N, Kd, mode = (int(x) for x in sys.argv[1:5])
reps = int(sys.argv[5]) if len(sys.argv) > 5 else 5
dev = torch.device("cuda:0")
a = torch.randn(M, Kd, device=dev).to(torch.bfloat16)
b = torch.randn(N, Kd, device=dev).to(torch.bfloat16)
out = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
K.gemm_set_pt(mode)
for _ in range(reps):
    K.gemm(a, b, trans_b=True, out=out)
torch.cuda.synchronize()

"""Debug: attention probabilities (desc.probs) and output of imgcap_mha_fwd vs torch (GPU box)."""
import ctypes
import math
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from imagecaptioningconvnext_amd import _abi  # noqa: E402
from imagecaptioningconvnext_amd import kernels as K  # noqa: E402

dev = torch.device("cuda:0")
torch.manual_seed(0)
B, H, d, L = 1, 1, 64, 8
q, k, v = (torch.randn(B, L, d) for _ in range(3))
qd, kd, vd = (t.to(dev, torch.bfloat16).contiguous() for t in (q, k, v))
qf, kf, vf = (t.to(torch.bfloat16).float() for t in (q, k, v))
s = qf[0] @ kf[0].t() / 8.0
P = torch.softmax(s, -1)
O = P @ vf[0]
o = torch.empty(B, L, d, device=dev, dtype=torch.bfloat16)
lse = torch.empty(B, H, L, device=dev)
probs = torch.zeros(B, H, L, L, device=dev)
m = _abi.MhaDesc()
m.dtype, m.B, m.H, m.Lq, m.Lk, m.dh, m.causal = K.dt(qd), B, H, L, L, 64, 0
m.ldq = m.ldk = m.ldv = m.ldo = d
m.q, m.k, m.v, m.o, m.lse = qd.data_ptr(), kd.data_ptr(), vd.data_ptr(), o.data_ptr(), lse.data_ptr()
m.scale = 1 / 8.0
m.probs = probs.data_ptr()
_abi.call("imgcap_mha_fwd", ctypes.byref(m), K.stream())
torch.cuda.synchronize()
torch.set_printoptions(precision=3, linewidth=200)
print("P err", (probs[0, 0].cpu() - P).abs().max().item())
print("O err", (o[0].float().cpu() - O).abs().max().item())
print("O rows err", (o[0].float().cpu() - O).abs().max(1).values)
# which V combination matches row 1?
print("got O[1,:8]", o[0, 1, :8].float().cpu())
print("ref O[1,:8]", O[1, :8])
print("V[:4,:8]", vf[0, :4, :8])
print("P[1]", P[1])
Wf = o[0].float().cpu() @ torch.linalg.pinv(vf[0])
print("effective P (got O = W V):")
print(Wf)
print("ref P:")
print(P)

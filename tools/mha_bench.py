"""imgcap_mha_fwd / _bwd at the C3 shapes (B=64, H=8, L=52 self-attention causal with key
padding; cross-attention over 49 pixels), dropout 0 and 0.1, µs per launch (GPU box):
    python tools/mha_bench.py [reps]"""
import ctypes
import math
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from imagecaptioningconvnext_amd import _abi  # noqa: E402
from imagecaptioningconvnext_amd import kernels as K  # noqa: E402
from tools.microbench import time_launch  # noqa: E402

reps = int(sys.argv[1]) if len(sys.argv) > 1 else 20
dev = torch.device("cuda:0")
bf = torch.bfloat16
B, H, L, P, d = 64, 8, 52, 49, 512


def desc(Lq, Lk, q, ldq, k, ldk, v, ldv, causal, key_ids, p, bwd_bufs=None):
    m = _abi.MhaDesc()
    m.dtype, m.B, m.H, m.Lq, m.Lk, m.dh, m.causal = K.dt(q), B, H, Lq, Lk, 64, int(causal)
    m.pad_id = 0
    m.ldq, m.ldk, m.ldv, m.ldo = ldq, ldk, ldv, d
    o = torch.empty(B * Lq, d, device=dev, dtype=bf)
    lse = torch.empty(B, H, Lq, device=dev)
    m.q, m.k, m.v, m.o, m.lse = q.data_ptr(), k.data_ptr(), v.data_ptr(), o.data_ptr(), lse.data_ptr()
    m.key_ids = K.ptr(key_ids)
    m.scale = 1.0 / math.sqrt(64.0)
    m.drop_p, m.seed, m.drop_stream = p, 11, 3
    keep = [o, lse]
    if bwd_bufs:
        dout, dq, dk, dv, lddk = bwd_bufs
        m.dout, m.lddo = dout.data_ptr(), d
        m.dq, m.dk, m.dv = dq.data_ptr(), dk.data_ptr(), dv.data_ptr()
        m.lddq, m.lddk, m.lddv = d, lddk, lddk
    return m, keep


qkv = torch.randn(B * L, 3 * d, device=dev).to(bf)
ids = torch.randint(1, 100, (B, L), device=dev)
ids[:, 40:] = 0
q2 = torch.randn(B * L, d, device=dev).to(bf)
kv = torch.randn(B * P, 2 * d, device=dev).to(bf)
dout = torch.randn(B * L, d, device=dev).to(bf)
dqkv = torch.empty(B * L, 3 * d, device=dev, dtype=bf)
dq2 = torch.empty(B * L, d, device=dev, dtype=bf)
dkv = torch.empty(B * P, 2 * d, device=dev, dtype=bf)
for p in (0.0, 0.1):
    ms, k1 = desc(L, L, qkv, 3 * d, qkv[:, d:], 3 * d, qkv[:, 2 * d:], 3 * d, True, ids, p,
                  (dout, dqkv, dqkv[:, d:], dqkv[:, 2 * d:], 3 * d))
    mc, k2 = desc(L, P, q2, d, kv, 2 * d, kv[:, d:], 2 * d, False, None, p, (dout, dq2, dkv, dkv[:, d:], 2 * d))
    _abi.call("imgcap_mha_fwd", ctypes.byref(ms), K.stream())
    _abi.call("imgcap_mha_fwd", ctypes.byref(mc), K.stream())
    r = []
    for m in (ms, mc):
        r.append(time_launch(lambda: _abi.call("imgcap_mha_fwd", ctypes.byref(m), K.stream()), reps=reps) * 1e6)
        r.append(time_launch(lambda: _abi.call("imgcap_mha_bwd", ctypes.byref(m), K.stream()), reps=reps) * 1e6)
    print(f"p={p}: self fwd {r[0]:.2f} bwd {r[1]:.2f} | cross fwd {r[2]:.2f} bwd {r[3]:.2f} us", flush=True)

"""Time the wide fused CNBlock MLP against the LayerNorm + two-GEMM path it replaces, at the
encoder's stage shapes, random operands, interleaved rounds in one process (GPU box):

    python tools/mlp_wide_bench.py [--reps 20] [--rounds 5]

Per shape: us per CNBlock MLP (LN + Linear + GELU + Linear + scale + residual), min / median over
rounds, and TFLOP/s at 16*M*C^2."""
import argparse
import math
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
from imagecaptioningconvnext_amd import kernels as K  # noqa: E402

SHAPES = [  # (label, M, C)
    ("C2 Tiny s3 B32", 32 * 196, 384), ("C3 Tiny s3 B64", 64 * 196, 384), ("C4 Base s3 B32", 32 * 196, 512),
    ("C3 Base s3 B64", 64 * 196, 512),
]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--only", default="", help="comma-separated shape indices")
    ap.add_argument("--fused-only", action="store_true")
    a = ap.parse_args()
    dev = torch.device("cuda:0")
    torch.manual_seed(0)
    sel = [int(i) for i in a.only.split(",")] if a.only else range(len(SHAPES))
    for label, M, C in [SHAPES[i] for i in sel]:
        y = (torch.randn(M, C, device=dev) * 2).bfloat16()
        x = torch.randn(M, C, device=dev).bfloat16()
        w1 = (torch.randn(4 * C, C, device=dev) / math.sqrt(C)).bfloat16()
        w2 = (torch.randn(C, 4 * C, device=dev) / math.sqrt(4 * C)).bfloat16()
        b1, b2, g, lw, lb = (torch.randn(n, device=dev) for n in (4 * C, C, C, C, C))
        img = K.cnblock_mlp_wide_pack(w1, w2)
        scratch = K.cnblock_mlp_wide_scratch(M, C, dev)
        zn = torch.empty(M, C, device=dev, dtype=torch.bfloat16)
        hid = torch.empty(M, 4 * C, device=dev, dtype=torch.bfloat16)

        def fused():
            K.cnblock_mlp_wide(y, img, b1, b2, g, x, scratch, ln_w=lw, ln_b=lb)

        def gemms():
            K.add_layernorm(y, None, lw, lb, 1e-6, y=zn)
            K.gemm(zn, w1, trans_b=True, bias=b1, act=K.ACT_GELU, out=hid)
            K.gemm(hid, w2, trans_b=True, bias=b2, colscale=g, res=x, out=x)

        times = {"fused": []} if a.fused_only else {"fused": [], "ln+2gemm": []}
        for fn in (fused, gemms):
            for _ in range(5):
                fn()
        torch.cuda.synchronize()
        for _ in range(a.rounds):
            for name, fn in (("fused", fused),) + ((("ln+2gemm", gemms),) if not a.fused_only else ()):
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                for _ in range(a.reps):
                    fn()
                e1.record()
                e1.synchronize()
                times[name].append(e0.elapsed_time(e1) * 1e3 / a.reps)
        fl = 16.0 * M * C * C
        line = f"{label:16s} M={M:6d} C={C:4d} split={'yes' if scratch[0] is not None else 'no ':3s}"
        for name, ts in times.items():
            ts = sorted(ts)
            line += f" | {name} min {ts[0]:7.1f} med {ts[len(ts) // 2]:7.1f} us ({fl / ts[0] / 1e6:6.0f} TF/s)"
        print(line, flush=True)


if __name__ == "__main__":
    main()

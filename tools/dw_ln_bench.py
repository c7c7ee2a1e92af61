"""Depthwise 7x7 + LayerNorm at the encoder's narrow stages: the fused row kernel
(imgcap_dwconv7_ln) against the channel-tiled depthwise kernel + add_layernorm the stages run
(GPU box; random operands, interleaved rounds, us per CNBlock head):

    python tools/dw_ln_bench.py"""
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
from imagecaptioningconvnext_amd import kernels as K  # noqa: E402

SHAPES = [("Tiny s3 B32", 32, 14, 384), ("Tiny s3 B64", 64, 14, 384), ("Base s3 B32", 32, 14, 512),
          ("Tiny s4 B64", 64, 7, 768), ("Base s4 B32", 32, 7, 1024), ("Large s3 B32", 32, 14, 768),
          ("Large s3 B64", 64, 14, 768)]


def main():
    dev = torch.device("cuda:0")
    torch.manual_seed(0)
    for label, B, H, C in SHAPES:
        x = torch.randn(B, H, H, C, device=dev).bfloat16()
        w49 = torch.randn(49, C, device=dev) * 0.1
        b, lw, lb = (torch.randn(C, device=dev) for _ in range(3))
        y = torch.empty_like(x)
        z = torch.empty_like(x)
        zf = torch.empty_like(x)
        M = B * H * H

        def cp_ln():
            os.environ["IMGCAP_DW_CP_R"] = "1"
            K.dwconv7_ln(x, w49, b, lw, lb, zf)

        def cp_dw():
            os.environ["IMGCAP_DW_CP_R"] = "1"
            K.dwconv7(x, w49, b, y)

        def cp2_ln():
            os.environ["IMGCAP_DW_CP_R"] = "2"
            K.dwconv7_ln(x, w49, b, lw, lb, zf)

        def cp2_dw():
            os.environ["IMGCAP_DW_CP_R"] = "2"
            K.dwconv7(x, w49, b, y)

        def old_dw_ln():
            os.environ["IMGCAP_DW_CP"] = "0"
            K.dwconv7(x, w49, b, y)
            K.add_layernorm(y.view(M, C), None, lw, lb, 1e-6, y=z.view(M, C))
            del os.environ["IMGCAP_DW_CP"]

        def old_dw():
            os.environ["IMGCAP_DW_CP"] = "0"
            K.dwconv7(x, w49, b, y)
            del os.environ["IMGCAP_DW_CP"]

        fns = (("cp+ln", cp_ln), ("cp2+ln", cp2_ln), ("old dw+ln", old_dw_ln), ("cp dw", cp_dw), ("cp2 dw", cp2_dw),
               ("old dw", old_dw))
        for _, fn in fns:
            fn()
        torch.cuda.synchronize()
        cp_ln()
        torch.cuda.synchronize()
        err = float((zf.float() - z.float()).norm() / z.float().norm())
        res = {n: [] for n, _ in fns}
        for _ in range(5):
            for name, fn in fns:
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                for _ in range(20):
                    fn()
                e1.record()
                e1.synchronize()
                res[name].append(e0.elapsed_time(e1) * 1e3 / 20)
        mb = 2 * M * C * 2 / 1e6
        print(f"{label:14s} B={B} H={H} C={C}: " + ", ".join(f"{n} {min(t):6.1f} us" for n, t in res.items())
              + f" | cp+ln {mb / min(res['cp+ln']):.2f} TB/s (2 x {mb / 2:.1f} MB), LN'd rel diff {err:.2e}", flush=True)


if __name__ == "__main__":
    main()

"""Depthwise 7x7 at the encoder's wide stages (W = 56 / 28): the column-segment kernel against
the channel-tiled kernel (IMGCAP_DW_SEG=0), random operands, interleaved rounds (GPU box):

    python tools/dw_wide_bench.py"""
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
from imagecaptioningconvnext_amd import kernels as K  # noqa: E402

SHAPES = [("Tiny s1 B32", 32, 56, 96), ("Tiny s1 B64", 64, 56, 96), ("Tiny s2 B64", 64, 28, 192),
          ("Base s1 B32", 32, 56, 128), ("Base s2 B32", 32, 28, 256), ("Large s1 B64", 64, 56, 192),
          ("Large s2 B64", 64, 28, 384)]


def main():
    dev = torch.device("cuda:0")
    torch.manual_seed(0)
    for label, B, H, C in SHAPES:
        x = torch.randn(B, H, H, C, device=dev).bfloat16()
        w49 = torch.randn(49, C, device=dev) * 0.1
        b = torch.randn(C, device=dev)
        y = torch.empty_like(x)

        def seg():
            os.environ["IMGCAP_DW_SEG"] = "1"
            K.dwconv7(x, w49, b, y)

        def tiled():
            os.environ["IMGCAP_DW_SEG"] = "0"
            K.dwconv7(x, w49, b, y)

        fns = (("seg", seg), ("tiled", tiled))
        for _, fn in fns:
            fn()
        torch.cuda.synchronize()
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
        mb = 2 * x.numel() * 2 / 1e6
        print(f"{label:13s} B={B} W={H} C={C}: " + ", ".join(f"{n} {min(t):6.1f} us ({mb / min(t):.2f} TB/s)"
                                                          for n, t in res.items()), flush=True)


if __name__ == "__main__":
    main()

"""imgcap_dwconv7_ln / imgcap_dwconv7 on the channel-pair kernel (dwconv7_cp_kernel) at the narrow
encoder stages, µs per launch (GPU box):  python tools/dw_cp_bench.py
(Round 6 timed a 2- and 3-rows-ahead load variant with it, IMGCAP_DW_CP_PF, since removed: DESIGN §7.)"""
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
from imagecaptioningconvnext_amd import kernels as K  # noqa: E402
from tools.microbench import time_launch  # noqa: E402

SHAPES = [("Tiny s3 B64", 64, 14, 384), ("Tiny s4 B64", 64, 7, 768), ("Base s3 B32", 32, 14, 512),
          ("Large s3 B64", 64, 14, 768), ("Tiny s3 B32", 32, 14, 384)]


def main():
    dev = torch.device("cuda:0")
    torch.manual_seed(0)
    out = []
    for label, B, H, C in SHAPES:
        x = torch.randn(B, H, H, C, device=dev).bfloat16()
        w = torch.randn(49, C, device=dev) * 0.1
        b, lw, lb = (torch.randn(C, device=dev) for _ in range(3))
        y = torch.empty_like(x)
        t_ln = time_launch(lambda: K.dwconv7_ln(x, w, b, lw, lb, y), reps=40) * 1e6
        t = time_launch(lambda: K.dwconv7(x, w, b, y), reps=40) * 1e6
        out.append(f"{label}: ln {t_ln:6.2f}  plain {t:6.2f}")
    print(" | ".join(out), flush=True)


if __name__ == "__main__":
    main()

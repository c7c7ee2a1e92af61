"""Time the batched bias-gradient column sums at the decoders' dlogits shapes (GPU box):

    python tools/colsum_bench.py"""
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
from imagecaptioningconvnext_amd import kernels as K  # noqa: E402


def main():
    dev = torch.device("cuda:0")
    for rows, cols in ((1632, 9490), (3264, 9490), (3264, 2048)):
        x = torch.randn(rows, cols, device=dev).bfloat16()
        out = torch.empty(cols, device=dev)

        def run():
            cb = K.ColsumBatch()
            cb.add(x, out)
            cb.run()
        for _ in range(5):
            run()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(50):
            run()
        e1.record()
        e1.synchronize()
        us = e0.elapsed_time(e1) * 1e3 / 50
        print(f"colsum_multi {rows}x{cols} bf16: {us:6.1f} us, {rows * cols * 2 / us / 1e6:5.2f} TB/s", flush=True)


if __name__ == "__main__":
    main()

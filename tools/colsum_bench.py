"""The C3 Transformer backward's bias-gradient column sums (one ColsumBatch: dlogits, six
layers' dY / dpre / dQ / dK|dV / dQKV and LayerNorm partials, dmem), single-pass vs two-pass
(GPU box):  python tools/colsum_bench.py [reps]"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from imagecaptioningconvnext_amd import kernels as K  # noqa: E402
from tools.microbench import time_launch  # noqa: E402

reps = int(sys.argv[1]) if len(sys.argv) > 1 else 10
dev = torch.device("cuda:0")
bf = torch.bfloat16
BL, BP, d, V, layers = 3328, 3136, 512, 9490, 6
items = [(torch.randn(BL, 9496, device=dev).to(bf), V)]
dkv_all = torch.randn(BP, 2 * d * layers, device=dev).to(bf)
for i in range(layers):
    items += [(torch.randn(BL, d, device=dev).to(bf), None) for _ in range(5)]  # dy3 dpre dy2 dq2 dy
    items.append((torch.randn(BL, 3 * d, device=dev).to(bf), None))              # dqkv
    items.append((dkv_all[:, 2 * d * i:2 * d * (i + 1)], None))                     # dK|dV
    part = torch.randn(416, 2, d, device=dev)
    items += [(part[:, 0], None), (part[:, 1], None)] * 3                           # LN partials
items.append((torch.randn(BP, d, device=dev), None))                                # dmem (fp32)
outs = [torch.zeros(c or x.shape[1], device=dev) for x, c in items]
mb = sum(x.shape[0] * (c or x.shape[1]) * x.element_size() for x, c in items) / 1e6


def run(two):
    K.ColsumBatch.TWO_PASS = two
    cb = K.ColsumBatch()
    for (x, c), o in zip(items, outs):
        cb.add(x, o, cols=c)
    cb.run()


for two in (False, True):
    t = time_launch(lambda: run(two), reps=reps)
    print(f"{'two-pass' if two else 'single-pass'}: {t * 1e6:.1f} us for {len(items)} items, {mb:.0f} MB "
          f"-> {mb / 1e6 / t:.2f} TB/s", flush=True)
run(False)
a = [o.clone() for o in outs]
for o in outs:
    o.zero_()
run(True)
print("max rel diff single vs two-pass:", max(((x - y).abs().max() / (y.abs().max() + 1e-9)).item() for x, y in zip(outs, a)))

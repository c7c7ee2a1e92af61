"""bf16 noise floor of the Transformer decoder's gradients (CPU only; test infrastructure).

Runs the bf16-emulating oracle (oracle/decoders.py numerics="bf16": the HIP build's rounding
points) in fp32 and in fp64 on the headline test's inputs and prints, per tensor, the relative
norm difference -- what two correct implementations of the same rounding points that accumulate in
different fp32 orders differ by -- and the emulating oracle's distance from the plain fp32 oracle
(what bf16 storage itself costs).  Usage: python tools/decoder_noise_floor.py [B] [E] [layers]."""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tests")]

from golden_util import make_captions, make_features, make_params  # noqa: E402
from oracle import decoders, shapes, train_step  # noqa: E402

V, L, D, H = 9490, 52, 512, 8


def grads(p, feats, caps, lens, layers, numerics, dtype):
    rb = lambda t: t.to(torch.bfloat16).to(dtype)  # noqa: E731
    # the engine's operands: bf16 GEMM weight matrices, fp32 biases / norms / embedding table
    pr = {k: (rb(v) if v.dim() == 2 and k != "embedding.weight" else v.to(dtype)).clone().requires_grad_(True)
          for k, v in p.items()}
    preds, cs, dls = decoders.transformer_tf_forward(pr, rb(feats), caps, lens, caps == 0, H, layers,
                                                     numerics=numerics)
    loss, _, _ = train_step.transformer_loss(preds, cs, dls)
    loss.backward()
    return {k: v.grad.double() for k, v in pr.items()}


def main():
    B = int(sys.argv[1]) if len(sys.argv) > 1 else 64
    E = int(sys.argv[2]) if len(sys.argv) > 2 else 768
    layers = int(sys.argv[3]) if len(sys.argv) > 3 else 6
    p = make_params(shapes.transformer_decoder_shapes(E, D, D, V, layers), 71)
    feats = make_features((B, 7, 7, E), 72)
    g = torch.Generator().manual_seed(74)
    pool = torch.tensor([L, L, L, 40, 40, 23, 17, 17, 9])
    caps, lens = make_captions(B, L, pool[torch.randint(0, len(pool), (B,), generator=g)].tolist(), V, 75)
    e64 = grads(p, feats, caps, lens, layers, "bf16", torch.float64)
    e32 = grads(p, feats, caps, lens, layers, "bf16", torch.float32)
    f32 = grads(p, feats, caps, lens, layers, "fp32", torch.float32)
    rel = lambda a, b: ((a - b).norm() / b.norm()).item()  # noqa: E731
    rows = sorted(((rel(e32[k], e64[k]), rel(e64[k], f32[k]), k) for k in e64), reverse=True)
    print(f"B={B} E={E} layers={layers}: emu32-vs-emu64 | emu64-vs-fp32 oracle")
    for a, b, k in rows:
        print(f"  {a:.4f} | {b:.4f}  {k}")


if __name__ == "__main__":
    main()

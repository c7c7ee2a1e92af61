"""Would the Transformer decoder's latency-bound chain run faster as two half-batch chains on two
streams?  (GPU box; probe for DESIGN §7.)

Captures the C3 decoder's forward + backward (B = 64, E = 768, d = 512, 6 layers, V = 9490, bf16,
dropout 0.5) into HIP graphs and times the replays:
  one64   : one chain at B = 64 (the shipped form)
  one32   : one chain at B = 32
  two32   : two B = 32 chains on two streams in one graph (own gradient buffers, scratch slot 1
            for the second chain)
usage: python tools/probe/dec_split.py [reps]"""
import faulthandler
import os
import sys

faulthandler.enable()

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from imagecaptioningconvnext_amd import kernels as K  # noqa: E402
from imagecaptioningconvnext_amd import transformer_engine as TE  # noqa: E402
from imagecaptioningconvnext_amd.models.transformerDecoder import TransformerDecoder  # noqa: E402

reps = int(sys.argv[1]) if len(sys.argv) > 1 else 20
dev = torch.device("cuda:0")
V, L, E = 9490, 52, 768
dec = TransformerDecoder(embed_dim=512, decoder_dim=512, vocab_size=V, maxLen=L, device=dev, wordMap=None,
                         pretrained_embeddings_path=None, fine_tune_embeddings=True, dropout=0.5, encoder_dim=E,
                         compute_dtype=torch.bfloat16).to(dev)
dec.train()
eng = dec.engine()


def batch(B, seed):
    g = torch.Generator(device="cpu").manual_seed(seed)
    feats = torch.randn(B, 7, 7, E, generator=g).to(dev)
    caps = torch.randint(1, V, (B, L), generator=g).to(dev)
    lens = torch.full((B, 1), L, dtype=torch.int64).to(dev)
    return feats, caps, lens


def chain(b, gbuf):
    s = eng.forward(*b)
    eng.backward(s, gbuf=gbuf)


def timed(fn):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    print("eager ok", flush=True)
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        fn()
    for _ in range(3):
        g.replay()
    torch.cuda.synchronize()
    a, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(reps):
        g.replay()
    e.record()
    e.synchronize()
    return a.elapsed_time(e) / reps * 1e3


b64, b32a, b32b = batch(64, 1), batch(32, 2), batch(32, 3)
g2 = torch.zeros_like(eng.fp.grad)
side = torch.cuda.Stream(device=dev)


def two():
    main = torch.cuda.current_stream(dev)
    print("two: fork", flush=True)
    K.fork(side, main)
    with torch.cuda.stream(side), K.workspace_slot(1):
        chain(b32b, g2)
    print("two: side chain issued", flush=True)
    chain(b32a, None)
    print("two: main chain issued", flush=True)
    K.join(main, side)


t64 = timed(lambda: chain(b64, None))
print(f"one64: {t64:8.1f} us", flush=True)
t32 = timed(lambda: chain(b32a, None))
print(f"one32: {t32:8.1f} us  ({t32 / t64:.2f} of one64)", flush=True)
# (the engine's tail side stream stays off here: one stream forked from two different capturing
# streams of one capture crashed hipStreamEndCapture -- tools/probe/capture_refork.py)
TE.TAIL_FORK = False
t1 = timed(lambda: chain(b64, None))
print(f"one64 without the tail fork: {t1:8.1f} us", flush=True)
t2 = timed(two)
print(f"two32: {t2:8.1f} us  ({t2 / t64:.2f} of one64)", flush=True)

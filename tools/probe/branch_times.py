"""The two branches of the pipelined C3 step timed alone (GPU box; probe for DESIGN §7): the frozen
ConvNeXt-Tiny forward at B = 64 (bf16, 224x224) and the Transformer decoder's forward + backward
(B = 64, E = 768, bf16, dropout 0.5), each captured as a HIP graph and replayed; then both in one
graph on two streams (the pipelined step without the update).  usage: python tools/probe/branch_times.py"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from imagecaptioningconvnext_amd import kernels as K  # noqa: E402
from imagecaptioningconvnext_amd.models.encoder import Encoder  # noqa: E402
from imagecaptioningconvnext_amd.models.transformerDecoder import TransformerDecoder  # noqa: E402

dev = torch.device("cuda:0")
V, L, E, B = 9490, 52, 768, 64
enc = Encoder(variant="tiny").to(dev).eval()
dec = TransformerDecoder(embed_dim=512, decoder_dim=512, vocab_size=V, maxLen=L, device=dev, wordMap=None,
                         pretrained_embeddings_path=None, fine_tune_embeddings=True, dropout=0.5, encoder_dim=E,
                         compute_dtype=torch.bfloat16).to(dev)
dec.train()
eng = dec.engine()
g = torch.Generator(device="cpu").manual_seed(0)
img = torch.randn(B, 3, 224, 224, generator=g).to(dev)
feats = torch.randn(B, 7, 7, E, generator=g).to(dev)
caps = torch.randint(1, V, (B, L), generator=g).to(dev)
lens = torch.full((B, 1), L, dtype=torch.int64).to(dev)
out = torch.empty(B, 7, 7, E, device=dev)


def encode():
    with torch.no_grad(), K.workspace_slot(1):
        out.copy_(enc(img))


def decode():
    s = eng.forward(feats, caps, lens)
    eng.backward(s)


side = torch.cuda.Stream(device=dev)


def both():
    main = torch.cuda.current_stream(dev)
    K.fork(side, main)
    with torch.cuda.stream(side):
        encode()
    decode()
    K.join(main, side)


def timed(fn, reps=20):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    gr = torch.cuda.CUDAGraph()
    with torch.cuda.graph(gr):
        fn()
    for _ in range(3):
        gr.replay()
    torch.cuda.synchronize()
    a, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(reps):
        gr.replay()
    e.record()
    e.synchronize()
    return a.elapsed_time(e) / reps * 1e3


te = timed(encode)
print(f"encoder alone (Tiny, B=64, bf16):        {te:8.1f} us", flush=True)
td = timed(decode)
print(f"decoder fwd+bwd alone (B=64, bf16):      {td:8.1f} us", flush=True)
tb = timed(both)
print(f"both branches in one graph:              {tb:8.1f} us  (sum {te + td:.1f}, max {max(te, td):.1f})", flush=True)

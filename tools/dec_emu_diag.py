"""Where does the bf16 Transformer engine leave the bf16-emulating oracle?  (GPU box; diagnostics.)

Runs one eager forward + backward of the engine (bf16, dropout 0) and the emulating oracle
(oracle/decoders.py numerics="bf16", fp64) on the same inputs and compares every stored activation
in forward order: relative norm difference and the fraction of elements whose bf16 bits differ.
A storage point the oracle emulates faithfully differs only by fp32 accumulation-order flips
(~1e-3 of the elements); the first tensor with many more is where the rounding points part.
Usage: python tools/dec_emu_diag.py [B] [E] [layers]."""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tests")]

from golden_util import make_captions, make_features, make_params  # noqa: E402
from oracle import decoders, shapes, train_step  # noqa: E402

V, L, D, H = 9490, 52, 512, 8


def main():
    B = int(sys.argv[1]) if len(sys.argv) > 1 else 64
    E = int(sys.argv[2]) if len(sys.argv) > 2 else 768
    layers = int(sys.argv[3]) if len(sys.argv) > 3 else 1
    dev = torch.device("cuda:0")
    from imagecaptioningconvnext_amd.models.transformerDecoder import TransformerDecoder
    p = make_params(shapes.transformer_decoder_shapes(E, D, D, V, layers), 71)
    feats = make_features((B, 7, 7, E), 72).to(torch.bfloat16).float()
    g = torch.Generator().manual_seed(74)
    pool = torch.tensor([L, L, L, 40, 40, 23, 17, 17, 9])
    caps, lens = make_captions(B, L, pool[torch.randint(0, len(pool), (B,), generator=g)].tolist(), V, 75)
    dec = TransformerDecoder(embed_dim=D, decoder_dim=D, vocab_size=V, maxLen=L, device=dev, wordMap=None,
                             pretrained_embeddings_path=None, fine_tune_embeddings=True, dropout=0.0, encoder_dim=E,
                             num_heads=H, num_layers=layers, compute_dtype=torch.bfloat16)
    p["pos_encoding.pe"] = dec.pos_encoding.pe.clone()
    dec.load_state_dict(p)
    dec = dec.to(dev)
    eng = dec.engine()
    s = eng.forward(feats.to(dev), caps.to(dev), lens.to(dev))
    eng.backward(s)
    torch.cuda.synchronize()

    # oracle, recording every bf16 storage point in call order
    rec = []
    orig_both = decoders._Bf16.both

    def both(t):
        out = orig_both(t)
        rec.append(out)
        out.retain_grad()
        return out
    decoders._Bf16.both = staticmethod(both)
    try:
        dt = torch.float64
        # the engine's operands: bf16 GEMM weight matrices, fp32 biases / norms / embedding table
        pr = {k: (v.to(torch.bfloat16).to(dt) if v.dim() == 2 and k != "embedding.weight" else v.to(dt)).clone()
              .requires_grad_(k != "pos_encoding.pe") for k, v in p.items()}
        preds, cs, dls = decoders.transformer_tf_forward(pr, feats.to(dt), caps, lens, caps == 0, H, layers,
                                                         pe=pr["pos_encoding.pe"], numerics="bf16")
        loss, _, _ = train_step.transformer_loss(preds, cs, dls)
        loss.backward()
    finally:
        decoders._Bf16.both = staticmethod(orig_both)
    names = ["x0", "kv_all"]
    for i in range(layers):
        names += [f"L{i}.{n}" for n in ("qkv", "o", "y1", "s1", "x1", "q2", "o2", "y2", "s2", "x2", "hdn", "y3",
                                        "s3", "x3")]
    names += ["logits"]
    assert len(names) == len(rec), (len(names), len(rec))
    o = dict(zip(names, rec))
    hip = {"x0": s["x0"], "kv_all": s["kv_all"], "logits": s["logits"][:, :V]}
    for i, st in enumerate(s["layers"]):
        for n in ("qkv", "o", "s1", "x1", "q2", "o2", "s2", "x2", "hdn", "s3"):
            hip[f"L{i}.{n}"] = st[n]
        hip[f"L{i}.x3"] = s["layers"][i + 1]["x"] if i + 1 < layers else s["xL"]

    def cmp(name, a, b):
        a = a.detach().float().cpu().reshape(b.shape).to(torch.bfloat16)
        b = b.detach().to(torch.bfloat16)
        diff = (a != b).float().mean().item()
        rel = ((a.double() - b.double()).norm() / (b.double().norm() + 1e-30)).item()
        print(f"  {name:12s} rel {rel:.2e}  bits differ {100 * diff:6.3f} %", flush=True)

    print(f"forward (B={B} E={E} layers={layers}): engine vs emulating oracle")
    for n in names:
        if n in hip:
            cmp(n, hip[n], o[n])
    print("backward: dlogits")
    cmp("dlogits", s["dlogits"][:, :V], o["logits"].grad.reshape(-1, V))
    print("gradients")
    for k in sorted(pr):
        if pr[k].grad is None:
            continue
        a = eng.fp.g(k).double().cpu()
        b = pr[k].grad
        print(f"  {k}: {((a - b).norm() / b.norm()).item():.2e}")


if __name__ == "__main__":
    main()

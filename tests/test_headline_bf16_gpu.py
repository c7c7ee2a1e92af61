"""The bench's exact decoder configuration, in its own precision and schedule, against the CPU oracle
(VERDICT r4 "What's weak" 2, VERDICT r5 "Next round" 1): bf16 compute with fp32 master weights,
B = 64 / E = 768 (C3) and B = 32 / E = 1024 (C4's width), V = 9490, L = 52, d = 512, 8 heads, the
step captured as HIP graphs and run through the two-stream pipelined schedule
(TeacherForcedTrainer(graph=True, pipeline=True): batch 1 is decoded by the first replay of the
captured pipelined graph while batch 2 is encoded beside it).  The reference's step
(train.py:262-291: packed CE, backward, clamp +-5, Adam) is the oracle's restatement on the same
weights and batch.  Dropout is 0 (the oracle cannot draw the HIP kernels' counter-based masks;
dropout has its own tests).  The encoder is a pass-through (the batch is encoder features).

Gradients are checked against the bf16-EMULATING oracle (oracle/decoders.py numerics="bf16": every
tensor the engine stores in bf16 is rounded there too, forward value and backward gradient; the
oracle gets the engine's operands: bf16 GEMM weight matrices, fp32 biases, LayerNorm parameters
and embedding table), evaluated in fp64, so the comparison measures the engine, not bf16.  What is
left between any two correct fp32-accumulating implementations of the same rounding points is
chaotic: a one-ulp difference in one stored element (a different fp32 summation order) moves later
roundings and flips ReLU masks of hidden units within rounding of zero, and each flip is a
full-size term in linear1's weight gradient; the spread grows ~3x per layer.  So each case computes
that floor for its own inputs -- the same emulating oracle in fp32 against the fp64 one -- and
gates the engine per tensor at FLOOR_X times the floor of that tensor (at least ABS_MIN), and its
worst tensor at FLOOR_X times the worst floor.  At one layer every tensor, linear1 included, must
also be within 1e-2 of the emulating oracle.  The fp32 step (last case) holds every tensor to 1e-2
of the plain fp32 oracle.

Measured on MI355X (round 6, tools/gpu/r6_c.sh; engine-vs-emu64 | floor):
  1 layer:  linear1.weight 0.0051 | 0.0064, encoder_proj.weight 0.0035 | 0.0037, the rest <= 0.0022
  2 layers: linear1.weight 0.0193 | 0.0195, embedding 0.0076 | 0.0076
  6 layers, B = 64 / E = 768:  linear1.weight 0.0397 | 0.0388, embedding 0.0265 | 0.0265
  6 layers, B = 32 / E = 1024: linear1.weight 0.0495 | 0.0460, embedding 0.0280 | 0.0265
i.e. the engine sits ON the floor (ratio 0.8-1.2 per tensor).  Against the plain fp32 oracle the
engine and the emulating oracle are equally far (embedding 0.038 both at 6 layers): that distance
is bf16 storage itself, which is why round 5's fixed 3e-2 gate against fp32 could not hold.
(Round 5 also fed that oracle bf16-rounded biases / embedding table, which the engine reads in
fp32; tools/dec_emu_diag.py compares every stored activation and located it: x0 6.8 % of its bf16
bits apart before, 0 % after.)"""
import pytest
import torch

from golden_util import make_captions, make_features, make_params
from oracle import decoders, shapes, train_step

pytestmark = pytest.mark.gpu

V, L, D, H = 9490, 52, 512, 8
FLOOR_X = 1.6   # engine error / (fp32-vs-fp64 spread of the emulating oracle), per tensor (measured <= 1.22)
ABS_MIN = 3e-3  # a tensor whose floor is ~0 still gets a few bf16 ulps


class PassThrough(torch.nn.Module):
    def forward(self, x):
        return x


def _rel(a, b):
    a, b = a.detach().double().cpu(), b.detach().double().cpu()
    return ((a - b).norm() / (b.norm() + 1e-30)).item()


def _lengths(B, seed):
    # full-length captions (the bench's synthetic default) mixed with shorter, tied ones
    g = torch.Generator().manual_seed(seed)
    pool = torch.tensor([L, L, L, 40, 40, 23, 17, 17, 9])
    return pool[torch.randint(0, len(pool), (B,), generator=g)].tolist()


def engine_operand(k, v):
    """The engine multiplies bf16 shadows of the GEMM weight matrices (FlatParams.w); biases,
    LayerNorm parameters and the embedding table it reads in fp32 (FlatParams.f32)."""
    return v.dim() == 2 and k != "embedding.weight"


def _oracle(p, feats, caps, lens, layers, numerics, dtype, bf16_operands):
    """The reference's step on the oracle: (loss, top-5 %, grads, tokens)."""
    rb = (lambda t: t.to(torch.bfloat16).to(dtype)) if bf16_operands else (lambda t: t.to(dtype))
    pr = {k: (rb(v) if engine_operand(k, v) else v.to(dtype)).clone().requires_grad_(k != "pos_encoding.pe")
          for k, v in p.items()}
    preds, cs, dls = decoders.transformer_tf_forward(pr, rb(feats), caps, lens, caps == 0, H, layers,
                                                     pe=pr["pos_encoding.pe"], numerics=numerics)
    loss, scores, targets = train_step.transformer_loss(preds, cs, dls)
    loss.backward()
    top5 = train_step.top5_correct(scores, targets) / len(targets) * 100
    return loss.item(), top5, {k: v.grad for k, v in pr.items() if v.requires_grad}, sum(dls)


@pytest.mark.parametrize("B,E,layers,dt", [(64, 768, 6, "bf16"), (32, 1024, 6, "bf16"), (64, 768, 1, "bf16"),
                                           (64, 768, 2, "bf16"), (64, 768, 6, "fp32")])
def test_bf16_pipelined_graph_step_vs_oracle(hip_device, B, E, layers, dt):
    from imagecaptioningconvnext_amd.models.transformerDecoder import TransformerDecoder
    from imagecaptioningconvnext_amd.train_step import TeacherForcedTrainer
    dev = hip_device
    lr = 1e-4
    bf = dt == "bf16"
    p = make_params(shapes.transformer_decoder_shapes(E, D, D, V, layers), 71)
    feats1, feats2 = make_features((B, 7, 7, E), 72), make_features((B, 7, 7, E), 73)
    caps1, lens1 = make_captions(B, L, _lengths(B, 74), V, 75)
    caps2, lens2 = make_captions(B, L, _lengths(B, 76), V, 77)
    dec = TransformerDecoder(embed_dim=D, decoder_dim=D, vocab_size=V, maxLen=L, device=dev, wordMap=None,
                             pretrained_embeddings_path=None, fine_tune_embeddings=True, dropout=0.0, encoder_dim=E,
                             num_heads=H, num_layers=layers, compute_dtype=torch.bfloat16 if bf else torch.float32)
    p["pos_encoding.pe"] = dec.pos_encoding.pe.clone()
    dec.load_state_dict(p)
    dec = dec.to(dev)

    # oracles on batch 1, on the operands the engine multiplies (its bf16 weight copies / features;
    # the fp32 masters are what Adam updates, below)
    loss32, top5, grads32, tokens = _oracle(p, feats1, caps1, lens1, layers, "fp32", torch.float32, bf)
    if bf:
        _, _, emu64, _ = _oracle(p, feats1, caps1, lens1, layers, "bf16", torch.float64, True)
        _, _, emu32, _ = _oracle(p, feats1, caps1, lens1, layers, "bf16", torch.float32, True)

    tr = TeacherForcedTrainer(PassThrough(), dec, lstm=False, decoder_lr=lr, grad_clip=5.0, graph=True,
                              pipeline=True)
    feats1_dev = feats1.to(torch.bfloat16).float() if bf else feats1
    assert tr.step(feats1_dev.to(dev), caps1.to(dev), lens1.to(dev)) is None  # batch 1 encoded
    tr.step(feats2.to(dev), caps2.to(dev), lens2.to(dev))  # captured graph: decode 1 || encode 2
    torch.cuda.synchronize()
    (g_loss, g_tok, g_top5), = tr.drain_metrics()
    assert abs(g_loss - loss32) <= 1e-2 * loss32, (g_loss, loss32)
    assert g_tok == tokens
    assert abs(g_top5 - top5) <= 0.5, (g_top5, top5)

    # the batch-1 gradients the replay left in the flat buffer, per tensor
    hip = {k: tr.eng.fp.g(k).detach().double().cpu() for k in grads32}
    if not bf:
        errs = sorted(((_rel(hip[k], grads32[k]), k) for k in grads32), reverse=True)
        assert errs[0][0] <= 1e-2, errs[:6]
    else:
        rows = []
        for k in grads32:
            rows.append((k, _rel(hip[k], emu64[k]), _rel(emu32[k], emu64[k]), _rel(hip[k], grads32[k]),
                         _rel(emu64[k], grads32[k])))
        rows.sort(key=lambda r: -r[1])
        print(f"\n[B={B} E={E} layers={layers}] tensor: engine-vs-emu64 | floor emu32-vs-emu64 | engine-vs-fp32 | "
              f"emu64-vs-fp32")
        for k, e, f, e32, f32 in rows[:12]:
            print(f"  {k}: {e:.4f} | {f:.4f} | {e32:.4f} | {f32:.4f}")
        if layers == 1:
            assert rows[0][1] <= 1e-2, rows[:4]
        worst_floor = max(r[2] for r in rows)
        assert rows[0][1] <= FLOOR_X * max(worst_floor, ABS_MIN), (rows[:4], worst_floor)
        bad = [r for r in rows if r[1] > FLOOR_X * max(r[2], ABS_MIN)]
        assert not bad, bad[:4]

    # post-Adam parameters: Adam's first step moves an entry by lr * g / (|g| + eps)
    grads = {k: (emu64[k].float() if bf else grads32[k]) for k in grads32}
    clip = train_step.clip_gradient(grads, 5.0)
    want = train_step.adam_step({k: p[k] for k in grads}, clip, {}, lr, 1)
    named = dict(dec.named_parameters())
    for k, w in want.items():
        got = named[k].detach().float().cpu()
        hg = hip[k].float()
        sure = (grads[k].abs() > 1e-5) & ((hg - grads[k]).abs() < 0.5 * grads[k].abs())
        if sure.any():
            assert (got - w)[sure].abs().max().item() <= 2e-3 * lr + 1e-7, k
        # (+ fp32 rounding of the parameter itself: entries near 1, e.g. LayerNorm gammas)
        assert ((got - w).abs() <= 2 * lr * 1.0001 + 4e-7 * w.abs().clamp(min=1.0)).all(), k
    tr.flush()  # batch 2 (eager), leaves the trainer drained
    torch.cuda.synchronize()

"""Teacher-forced decoder forwards restated with explicit torch-CPU tensor math (autograd on).

``p`` is a {state-dict key: tensor} dict with the reference's key names.

lstm_tf_forward        models/decoder.py:69-113 (+ Attention 25-31, init_hidden_state 63-67)
transformer_tf_forward models/transformerDecoder.py:88-108 (+ PositionalEncoding 14-27) and
                       torch.nn.TransformerDecoderLayer's post-norm (norm_first=False) math
                       with ReLU FFN, as constructed at transformerDecoder.py:82-83.
Dropout is the identity here (parity runs use p=0 / eval, SURVEY.md §7 hard part iv).

``numerics="bf16"`` (transformer_tf_forward) emulates the HIP bf16 build's storage points, so the
bf16 gates measure the engine rather than bf16 itself (as oracle/convnext.py's mode does for the
encoder).  Every tensor the engine keeps in bf16 is rounded to bf16 here, in the forward (value)
and in the backward (its gradient), at the same place: GEMM outputs after bias / ReLU, the
embedding + positional sum, each residual sum s = x + y the LayerNorm reads and the LayerNorm
output, the attention probabilities before P V, the score gradient dS before dQ = dS K /
dK = dS^T Q, the logits and dlogits.  Sums the engine forms in fp32 stay fp32 (softmax, LayerNorm
statistics, the memory gradient over the six layers' K/V products, weight-gradient products,
bias column sums); the encoder_proj weight gradient reads the memory gradient rounded to bf16,
its bias gradient the fp32 one (transformer_engine.py backward).  Weights are given already
rounded (the engine multiplies its bf16 shadow copies).
"""
import math

import torch
import torch.nn.functional as F


def _lin(x, p, name):
    return x @ p[name + ".weight"].t() + p[name + ".bias"]


def _bf(t):
    return t.to(torch.bfloat16).to(t.dtype)


class _RoundBoth(torch.autograd.Function):
    """bf16 storage point: the value rounded in the forward, its gradient in the backward."""

    @staticmethod
    def forward(ctx, x):
        return _bf(x)

    @staticmethod
    def backward(ctx, g):
        return _bf(g)


class _RoundValue(torch.autograd.Function):
    """An MFMA operand rounded to bf16 whose gradient stays fp32 (the attention probabilities)."""

    @staticmethod
    def forward(ctx, x):
        return _bf(x)

    @staticmethod
    def backward(ctx, g):
        return g


class _RoundGrad(torch.autograd.Function):
    """Identity forward; the gradient rounded to bf16 (dS before the dQ / dK products)."""

    @staticmethod
    def forward(ctx, x):
        return x

    @staticmethod
    def backward(ctx, g):
        return _bf(g)


class _ProjBf16(torch.autograd.Function):
    """memory = enc W^T + b with the engine's gradients: dW from the fp32 memory gradient rounded
    to bf16 (dmem_c), db from the fp32 one, d enc = bf16(dmem) W."""

    @staticmethod
    def forward(ctx, x, w, b):
        ctx.save_for_backward(x, w)
        return _bf(x @ w.t() + b)

    @staticmethod
    def backward(ctx, g):
        x, w = ctx.saved_tensors
        gc = _bf(g)
        gx = gc @ w
        gw = gc.reshape(-1, gc.shape[-1]).t() @ x.reshape(-1, x.shape[-1])
        gb = g.reshape(-1, g.shape[-1]).sum(0)
        return gx, gw, gb


_IDENT = staticmethod(lambda t: t)


class _Fp32:
    both = value = grad = _IDENT


class _Bf16:
    both = staticmethod(_RoundBoth.apply)
    value = staticmethod(_RoundValue.apply)
    grad = staticmethod(_RoundGrad.apply)


def lstm_tf_forward(p, encoder_out, encoded_captions, caption_lengths):
    """Returns (predictions[B,Tmax,V], caps_sorted, decode_lengths(list), alphas[B,Tmax,P], sort_ind)."""
    B = encoder_out.size(0)
    E = encoder_out.size(-1)
    enc = encoder_out.reshape(B, -1, E)                                      # decoder.py:75
    P = enc.size(1)
    lens, sort_ind = caption_lengths.squeeze(1).sort(dim=0, descending=True)  # decoder.py:79
    enc = enc[sort_ind]
    caps = encoded_captions[sort_ind]
    emb = p["embedding.weight"][caps]                                        # decoder.py:84
    mean = enc.mean(dim=1)                                                   # decoder.py:64
    h = _lin(mean, p, "init_h")
    c = _lin(mean, p, "init_c")
    dls = (lens - 1).tolist()                                                # decoder.py:91
    T = max(dls)
    V = p["fc.weight"].shape[0]
    D = h.shape[1]
    preds = torch.zeros(B, T, V, dtype=enc.dtype)
    alphas = torch.zeros(B, T, P, dtype=enc.dtype)
    att1_full = _lin(enc, p, "attention.encoder_att")                        # decoder.py:26
    w_ih, w_hh = p["decode_step.weight_ih"], p["decode_step.weight_hh"]
    b_ih, b_hh = p["decode_step.bias_ih"], p["decode_step.bias_hh"]
    for t in range(T):                                                       # decoder.py:100
        bt = sum(int(l > t) for l in dls)
        ht, ct = h[:bt], c[:bt]
        att2 = _lin(ht, p, "attention.decoder_att")                          # decoder.py:27
        e = _lin(torch.relu(att1_full[:bt] + att2.unsqueeze(1)), p, "attention.full_att").squeeze(2)
        alpha = torch.softmax(e, dim=1)                                      # decoder.py:29
        awe = (enc[:bt] * alpha.unsqueeze(2)).sum(dim=1)                     # decoder.py:30
        gate = torch.sigmoid(_lin(ht, p, "f_beta"))                          # decoder.py:104
        x = torch.cat([emb[:bt, t, :], gate * awe], dim=1)                   # decoder.py:107
        gates = x @ w_ih.t() + b_ih + ht @ w_hh.t() + b_hh                   # torch LSTMCell
        i, f, g, o = gates.split(D, dim=1)
        c = torch.sigmoid(f) * ct + torch.sigmoid(i) * torch.tanh(g)
        h = torch.sigmoid(o) * torch.tanh(c)
        preds_t = _lin(h, p, "fc")                                           # decoder.py:109
        preds = preds.index_put((torch.arange(bt), torch.full((bt,), t)), preds_t)
        alphas = alphas.index_put((torch.arange(bt), torch.full((bt,), t)), alpha)
    return preds, caps, dls, alphas, sort_ind


def positional_encoding(embed_dim, max_len, dtype=torch.float32):
    """PositionalEncoding buffer (transformerDecoder.py:17-22), shape [1, max_len, embed_dim]."""
    pe = torch.zeros(max_len, embed_dim)
    pos = torch.arange(0, max_len, dtype=torch.float).unsqueeze(1)
    div = torch.exp(torch.arange(0, embed_dim, 2).float() * (-math.log(10000.0) / embed_dim))
    pe[:, 0::2] = torch.sin(pos * div)
    pe[:, 1::2] = torch.cos(pos * div)
    return pe.unsqueeze(0).to(dtype)


def _mha(xq, xkv, p, pre, nhead, attn_mask=None, key_pad=None, nm=_Fp32, kv=None):
    """torch MultiheadAttention (batch-first restatement): packed in_proj [3d, d], out_proj.
    ``kv`` (bf16 mode): the cross-attention K | V already projected (the engine's one GEMM over
    every layer's stacked W_kv, a storage point of its own)."""
    B, Lq, d = xq.shape
    Lk = xkv.shape[1]
    W, bias = p[pre + ".in_proj_weight"], p[pre + ".in_proj_bias"]
    if nm is _Fp32:
        q = xq @ W[:d].t() + bias[:d]
        k = xkv @ W[d:2 * d].t() + bias[d:2 * d]
        v = xkv @ W[2 * d:].t() + bias[2 * d:]
    elif xq is xkv:  # self-attention: one qkv GEMM
        qkv = nm.both(xq @ W.t() + bias)
        q, k, v = qkv[..., :d], qkv[..., d:2 * d], qkv[..., 2 * d:]
    else:
        q = nm.both(xq @ W[:d].t() + bias[:d])
        if kv is None:
            kv = nm.both(xkv @ W[d:].t() + bias[d:])
        k, v = kv[..., :d], kv[..., d:]
    dh = d // nhead
    q = q.reshape(B, Lq, nhead, dh).transpose(1, 2)
    k = k.reshape(B, Lk, nhead, dh).transpose(1, 2)
    v = v.reshape(B, Lk, nhead, dh).transpose(1, 2)
    s = nm.grad(q @ k.transpose(-1, -2)) / math.sqrt(dh)
    if attn_mask is not None:
        s = s.masked_fill(attn_mask.view(1, 1, Lq, Lk), float("-inf"))
    if key_pad is not None:
        s = s.masked_fill(key_pad.view(B, 1, 1, Lk), float("-inf"))
    a = torch.softmax(s, dim=-1)
    o = nm.both((nm.value(a) @ v).transpose(1, 2).reshape(B, Lq, d))
    return o @ p[pre + ".out_proj.weight"].t() + p[pre + ".out_proj.bias"]


def transformer_tf_forward(p, encoder_out, encoded_captions, caption_lengths, tgt_key_padding_mask,
                           nhead, num_layers, pe=None, numerics="fp32"):
    """Returns (predictions[B,L,V], encoded_captions, decode_lengths).  ``numerics``: "fp32", or
    "bf16" (the HIP bf16 build's storage points, module docstring)."""
    nm = {"fp32": _Fp32, "bf16": _Bf16}[numerics]
    B = encoder_out.size(0)
    E = encoder_out.size(-1)
    dls = (caption_lengths.squeeze(1) - 1).tolist()                          # transformerDecoder.py:92
    enc = encoder_out.reshape(B, -1, E)
    if "encoder_proj.weight" in p:                                           # transformerDecoder.py:95
        if nm is _Fp32:
            mem = _lin(enc, p, "encoder_proj")
        else:
            mem = _ProjBf16.apply(enc, p["encoder_proj.weight"], p["encoder_proj.bias"])
    else:
        mem = enc
    x = p["embedding.weight"][encoded_captions]                              # :97
    L, d = x.shape[1], x.shape[2]
    if pe is None:
        pe = positional_encoding(d, L)
    x = nm.both(x + pe[:, :L].to(x.dtype))                                   # :98 (dropout = id)
    causal = torch.triu(torch.ones(L, L, dtype=torch.bool), diagonal=1)     # :102
    kv_all = None
    if nm is not _Fp32:  # the engine's stacked cross-attention K | V GEMM (one storage point)
        pl = [f"transformer_decoder.layers.{li}.multihead_attn." for li in range(num_layers)]
        wkv = torch.cat([p[q + "in_proj_weight"][d:] for q in pl])
        bkv = torch.cat([p[q + "in_proj_bias"][d:] for q in pl])
        kv_all = nm.both(mem @ wkv.t() + bkv)

    def add_ln(x, y, pre, k):
        s = nm.both(x + nm.both(y))
        return nm.both(F.layer_norm(s, (d,), p[pre + f"norm{k}.weight"], p[pre + f"norm{k}.bias"], 1e-5))

    for li in range(num_layers):                                             # :104
        pre = f"transformer_decoder.layers.{li}."
        x = add_ln(x, _mha(x, x, p, pre + "self_attn", nhead, causal, tgt_key_padding_mask, nm), pre, 1)
        kv = None if kv_all is None else kv_all[..., 2 * d * li:2 * d * (li + 1)]
        x = add_ln(x, _mha(x, mem, p, pre + "multihead_attn", nhead, nm=nm, kv=kv), pre, 2)
        ff = _lin(nm.both(torch.relu(_lin(x, p, pre + "linear1"))), p, pre + "linear2")
        x = add_ln(x, ff, pre, 3)
    preds = nm.both(_lin(x, p, "fc_out"))                                    # :106
    return preds, encoded_captions, dls

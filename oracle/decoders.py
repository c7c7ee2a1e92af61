"""Teacher-forced decoder forwards restated with explicit torch-CPU tensor math (autograd on).

``p`` is a {state-dict key: tensor} dict with the reference's key names.

lstm_tf_forward        models/decoder.py:69-113 (+ Attention 25-31, init_hidden_state 63-67)
transformer_tf_forward models/transformerDecoder.py:88-108 (+ PositionalEncoding 14-27) and
                       torch.nn.TransformerDecoderLayer's post-norm (norm_first=False) math
                       with ReLU FFN, as constructed at transformerDecoder.py:82-83.
Dropout is the identity here (parity runs use p=0 / eval, SURVEY.md §7 hard part iv).
"""
import math

import torch
import torch.nn.functional as F


def _lin(x, p, name):
    return x @ p[name + ".weight"].t() + p[name + ".bias"]


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


def _mha(xq, xkv, p, pre, nhead, attn_mask=None, key_pad=None):
    """torch MultiheadAttention (batch-first restatement): packed in_proj [3d, d], out_proj."""
    B, Lq, d = xq.shape
    Lk = xkv.shape[1]
    W, bias = p[pre + ".in_proj_weight"], p[pre + ".in_proj_bias"]
    q = xq @ W[:d].t() + bias[:d]
    k = xkv @ W[d:2 * d].t() + bias[d:2 * d]
    v = xkv @ W[2 * d:].t() + bias[2 * d:]
    dh = d // nhead
    q = q.view(B, Lq, nhead, dh).transpose(1, 2)
    k = k.view(B, Lk, nhead, dh).transpose(1, 2)
    v = v.view(B, Lk, nhead, dh).transpose(1, 2)
    s = (q @ k.transpose(-1, -2)) / math.sqrt(dh)
    if attn_mask is not None:
        s = s.masked_fill(attn_mask.view(1, 1, Lq, Lk), float("-inf"))
    if key_pad is not None:
        s = s.masked_fill(key_pad.view(B, 1, 1, Lk), float("-inf"))
    a = torch.softmax(s, dim=-1)
    o = (a @ v).transpose(1, 2).reshape(B, Lq, d)
    return o @ p[pre + ".out_proj.weight"].t() + p[pre + ".out_proj.bias"]


def transformer_tf_forward(p, encoder_out, encoded_captions, caption_lengths, tgt_key_padding_mask,
                           nhead, num_layers, pe=None):
    """Returns (predictions[B,L,V], encoded_captions, decode_lengths)."""
    B = encoder_out.size(0)
    E = encoder_out.size(-1)
    dls = (caption_lengths.squeeze(1) - 1).tolist()                          # transformerDecoder.py:92
    enc = encoder_out.reshape(B, -1, E)
    if "encoder_proj.weight" in p:
        mem = _lin(enc, p, "encoder_proj")                                   # transformerDecoder.py:95
    else:
        mem = enc
    x = p["embedding.weight"][encoded_captions]                              # :97
    L, d = x.shape[1], x.shape[2]
    if pe is None:
        pe = positional_encoding(d, L)
    x = x + pe[:, :L].to(x.dtype)                                            # :98 (dropout = id)
    causal = torch.triu(torch.ones(L, L, dtype=torch.bool), diagonal=1)     # :102
    for li in range(num_layers):                                             # :104
        pre = f"transformer_decoder.layers.{li}."
        x = F.layer_norm(x + _mha(x, x, p, pre + "self_attn", nhead, causal, tgt_key_padding_mask),
                         (d,), p[pre + "norm1.weight"], p[pre + "norm1.bias"], 1e-5)
        x = F.layer_norm(x + _mha(x, mem, p, pre + "multihead_attn", nhead),
                         (d,), p[pre + "norm2.weight"], p[pre + "norm2.bias"], 1e-5)
        ff = _lin(torch.relu(_lin(x, p, pre + "linear1")), p, pre + "linear2")
        x = F.layer_norm(x + ff, (d,), p[pre + "norm3.weight"], p[pre + "norm3.bias"], 1e-5)
    preds = _lin(x, p, "fc_out")                                             # :106
    return preds, encoded_captions, dls

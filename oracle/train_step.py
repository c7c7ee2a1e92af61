"""Loss assembly, top-5, clip and Adam of the teacher-forced step, restated on torch CPU.

pack_time_major  torch.nn.utils.rnn.pack_padded_sequence(...).data semantics used at
                 train.py:266-267 / 274-275 (time-major packing; enforce_sorted=False sorts
                 rows by length, descending, stable)
lstm_loss        train.py:265-269   (CE mean over packed tokens + alphaC * mean((1-sum_t a)^2))
transformer_loss train.py:271-276
top5_correct     utils/utils.py:239-254 (topk(5) hit count)
clip_gradient    utils/utils.py:183-192 (element-wise clamp to +-gradClip)
adam_step        torch.optim.Adam defaults (betas .9/.999, eps 1e-8, no weight decay) as
                 created at train.py:110 and stepped at train.py:291
"""
import math

import torch
import torch.nn.functional as F


def pack_time_major(x, lengths, enforce_sorted=True):
    """Rows ordered t-major then by (sorted) batch index, keeping [:, :len_b] per row."""
    lengths = torch.as_tensor(lengths)
    if enforce_sorted:
        order = torch.arange(len(lengths))
    else:
        order = torch.sort(lengths, descending=True, stable=True).indices
    idx_b, idx_t = [], []
    for t in range(int(lengths.max())):
        for b in order.tolist():
            if lengths[b] > t:
                idx_b.append(b)
                idx_t.append(t)
    return x[torch.tensor(idx_b), torch.tensor(idx_t)]


def lstm_loss(predictions, caps_sorted, decode_lengths, alphas, alphaC=1.0):
    scores = pack_time_major(predictions, decode_lengths)
    targets = pack_time_major(caps_sorted[:, 1:], decode_lengths)
    ce = F.cross_entropy(scores, targets)
    return ce + alphaC * ((1.0 - alphas.sum(dim=1)) ** 2).mean(), scores, targets


def transformer_loss(predictions, caps, decode_lengths):
    scores = pack_time_major(predictions, decode_lengths, enforce_sorted=False)
    targets = pack_time_major(caps[:, 1:], decode_lengths, enforce_sorted=False)
    return F.cross_entropy(scores, targets), scores, targets


def top5_correct(scores, targets, k=5):
    _, ind = scores.topk(k, 1, True, True)
    return float(ind.eq(targets.view(-1, 1).expand_as(ind)).float().sum())


def clip_gradient(grads, clip):
    return {k: g.clamp(-clip, clip) for k, g in grads.items()}


def adam_step(params, grads, state, lr, step, betas=(0.9, 0.999), eps=1e-8):
    """Returns new params; ``state`` {name: (m, v)} is updated in place."""
    b1, b2 = betas
    out = {}
    for k, p in params.items():
        g = grads[k]
        m, v = state.get(k, (torch.zeros_like(p), torch.zeros_like(p)))
        m = b1 * m + (1 - b1) * g
        v = b2 * v + (1 - b2) * g * g
        state[k] = (m, v)
        bc1 = 1 - b1 ** step
        bc2 = 1 - b2 ** step
        denom = v.sqrt() / math.sqrt(bc2) + eps
        out[k] = p - (lr / bc1) * m / denom
    return out

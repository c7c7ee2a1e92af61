"""Validation without teacher forcing: train.py:367-441 ``validate`` on
device, ``preprocessDecoderOutputForMetrics`` (utils.py:261-296) and corpus BLEU.

* The greedy predictions stay on the GPU: the decode lengths (first <end> + 1, else
  maxDecodeLen) and the ignore-mask (t >= length or target = <pad>) become a target row per
  (sample, step) with -1 for dropped rows, so the cross-entropy / top-5 kernels of the training
  loss (imgcap_ce_fwd + imgcap_loss_finalize) evaluate exactly the rows the reference's
  filtering keeps, and the LSTM's attention regulariser is imgcap_attn_reg over all steps.
* BLEU: nltk is not part of this image, so ``corpus_bleu`` restates
  ``nltk.translate.bleu_score.corpus_bleu`` (nltk 3.x defaults: clipped n-gram counts summed
  over the corpus, closest-reference-length brevity penalty, smoothing method0 -- a zero
  numerator at n makes log p_n = log(sys.float_info.min), and no unigram match gives 0), pinned
  by nltk's documented examples (tests/test_metrics_cpu.py).
"""
import math
import sys
from collections import Counter
from fractions import Fraction

import torch

from . import _abi
from . import kernels as K


# ---- BLEU (nltk.translate.bleu_score.corpus_bleu restated) -----------------------------------
def _ngrams(seq, n):
    return [tuple(seq[i:i + n]) for i in range(len(seq) - n + 1)]


def _modified_precision(references, hypothesis, n):
    counts = Counter(_ngrams(hypothesis, n))
    if not counts:  # nltk: numerator 0 over max(1, 0) -- a too-short hypothesis still counts once
        return 0, 1
    max_ref = {}
    for ref in references:
        rc = Counter(_ngrams(ref, n))
        for g in counts:
            max_ref[g] = max(max_ref.get(g, 0), rc[g])
    clipped = sum(min(c, max_ref[g]) for g, c in counts.items())
    return clipped, max(1, sum(counts.values()))


def _closest_ref_length(references, hyp_len):
    return min((len(r) for r in references), key=lambda rl: (abs(rl - hyp_len), rl))


def corpus_bleu(list_of_references, hypotheses, weights=(0.25, 0.25, 0.25, 0.25)):
    assert len(list_of_references) == len(hypotheses)
    num, den = Counter(), Counter()
    hyp_len = ref_len = 0
    for refs, hyp in zip(list_of_references, hypotheses):
        for i in range(1, len(weights) + 1):
            a, b = _modified_precision(refs, hyp, i)
            num[i] += a
            den[i] += b
        hyp_len += len(hyp)
        ref_len += _closest_ref_length(refs, len(hyp))
    bp = 1.0 if hyp_len > ref_len else (0.0 if hyp_len == 0 else math.exp(1 - ref_len / hyp_len))
    if num[1] == 0:
        return 0.0
    p_n = [Fraction(num[i], den[i], _normalize=False) if den[i] else Fraction(0) for i in range(1, len(weights) + 1)]
    logs = []
    for w, p in zip(weights, p_n):
        pv = float(p) if p.numerator else sys.float_info.min  # smoothing method0
        logs.append(w * math.log(pv))
    return bp * math.exp(math.fsum(logs))


# ---- preprocessDecoderOutputForMetrics on device ------------------------------------------
def decode_lengths(sequences, end_id, maxlen):
    """utils.py:268-275: first <end> index + 1, else maxDecodeLen (device int64 [B])."""
    is_end = sequences == end_id
    first = torch.where(is_end.any(dim=1), is_end.int().argmax(dim=1) + 1,
                        torch.full_like(sequences[:, 0], maxlen))
    return first


def metric_targets(sequences, captions, end_id, pad_id, maxlen):
    """Target id per (sample, step) of the greedy predictions, -1 where the reference's filtering
    drops the row (t >= decode length, or the ground truth there is <pad>): utils.py:277-282."""
    B = sequences.shape[0]
    n = decode_lengths(sequences, end_id, maxlen)
    L = captions.shape[1]
    gt = torch.full((B, maxlen), pad_id, device=captions.device, dtype=torch.int64)
    m = min(maxlen, L - 1)
    gt[:, :m] = captions[:, 1:1 + m]
    t = torch.arange(maxlen, device=captions.device).view(1, maxlen)
    keep = (t < n.view(B, 1)) & (gt != pad_id)
    return torch.where(keep, gt, torch.full_like(gt, -1)), n


def greedy_loss(predictions, sequences, captions, wordMap, maxlen, alphas=None, alphaC=1.0):
    """train.py:396-407 on device: (metrics [loss, tokens, top-5 hits, 1/tokens] fp32 device
    tensor, decode lengths).  loss = CE over the kept rows (+ alphaC * mean((1 - sum_t alpha)^2)
    for the LSTM); one host read per batch is the caller's choice."""
    B, T, V = predictions.shape
    targets, n = metric_targets(sequences, captions, wordMap['<end>'], wordMap['<pad>'], maxlen)
    dev = predictions.device
    f32 = dict(device=dev, dtype=torch.float32)
    lse, lrow, hit = (torch.empty(B * T, **f32) for _ in range(3))
    logits = predictions.reshape(B * T, V)
    tg = targets.reshape(-1).contiguous()
    K.ce_fwd(logits, tg, V, lse, lrow, hit)
    reg = None
    if alphas is not None:
        P = alphas.shape[2]
        reg = torch.empty(1, **f32)
        dalpha = torch.empty(B, T, P, **f32)
        dl = torch.full((B,), T, device=dev, dtype=torch.int32)
        _abi.call("imgcap_attn_reg", B, T, P, alphas.contiguous().data_ptr(), dl.data_ptr(), alphaC,
                  dalpha.data_ptr(), reg.data_ptr(), None, K.stream())
    metrics = torch.empty(4, **f32)
    K.loss_finalize(lrow, hit, tg, reg, metrics)
    return metrics, n


def validate(valDataLoader, encoder, decoder, wordMap, lstm, device, maxDecodeLen=51, alphaC=1.0, log=print,
             label="Validation"):
    """train.py:367-441: greedy decoding over the VAL split -> (loss avg, top-5 avg, BLEU-1..4).
    test.py:144-215 is the same loop over the TEST split (``label="Test"``)."""
    decoder.eval()
    if encoder is not None:
        encoder.eval()
    start_pad = {wordMap['<start>'], wordMap['<pad>']}
    references, hypotheses = [], []
    tot_loss = tot_tok = tot_hit = 0.0
    with torch.no_grad():
        for i, (imgs, caps, caplens, allcaps) in enumerate(valDataLoader):
            if i % 100 == 0:
                log(f"No TF, {label} Batch {i + 1}", flush=True)
            imgs, caps = imgs.to(device), caps.to(device)
            feats = encoder(imgs) if encoder is not None else imgs
            out = decoder(teacherForcing=False, encoder_out=feats, wordMap=wordMap, maxDecodeLen=maxDecodeLen)
            scores, seqs = out[0], out[-1]
            metrics, n = greedy_loss(scores, seqs, caps, wordMap, maxDecodeLen, alphas=out[1] if lstm else None,
                                     alphaC=alphaC)
            m = metrics.cpu()
            tot_loss += float(m[0]) * float(m[1])
            tot_tok += float(m[1])
            tot_hit += float(m[2])
            for imgCaps in allcaps.tolist():
                references.append([[w for w in c if w not in start_pad] for c in imgCaps])
            for seq, L in zip(seqs.cpu().tolist(), n.cpu().tolist()):
                hypotheses.append(seq[:L])
    loss = tot_loss / max(tot_tok, 1.0)
    top5 = tot_hit / max(tot_tok, 1.0) * 100.0
    bleu = [corpus_bleu(references, hypotheses, weights=w) for w in
            ((1.0, 0.0, 0.0, 0.0), (0.5, 0.5, 0.0, 0.0), (0.33, 0.33, 0.33, 0.0), (0.25, 0.25, 0.25, 0.25))]
    log(f"No TF, {label} Loss = {loss:.4f}, Top-5 Accuracy = {top5:.4f}, Bleu-1 = {bleu[0]:.4f}, "
        f"Bleu-2 = {bleu[1]:.4f}, Bleu-3 = {bleu[2]:.4f}, Bleu-4 = {bleu[3]:.4f}", flush=True)
    return (loss, top5, *bleu)

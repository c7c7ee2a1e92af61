"""corpus BLEU restated from nltk.translate.bleu_score (nltk absent here: parity pinned by the
known answers in nltk's own documentation) and the greedy-metric target construction vs the
reference's preprocessDecoderOutputForMetrics (utils.py:261-296, restated in torch below)."""
import pytest
import torch

H1 = ['It', 'is', 'a', 'guide', 'to', 'action', 'which', 'ensures', 'that', 'the', 'military', 'always', 'obeys',
      'the', 'commands', 'of', 'the', 'party']
R1A = ['It', 'is', 'a', 'guide', 'to', 'action', 'that', 'ensures', 'that', 'the', 'military', 'will', 'forever',
       'heed', 'Party', 'commands']
R1B = ['It', 'is', 'the', 'guiding', 'principle', 'which', 'guarantees', 'the', 'military', 'forces', 'always',
       'being', 'under', 'the', 'command', 'of', 'the', 'Party']
R1C = ['It', 'is', 'the', 'practical', 'guide', 'for', 'the', 'army', 'always', 'to', 'heed', 'the', 'directions',
       'of', 'the', 'party']
H2 = ['he', 'read', 'the', 'book', 'because', 'he', 'was', 'interested', 'in', 'world', 'history']
R2A = ['he', 'was', 'interested', 'in', 'world', 'history', 'because', 'he', 'read', 'the', 'book']


def test_corpus_bleu_known_answers():
    from imagecaptioningconvnext_amd.metrics import corpus_bleu
    # nltk documentation (bleu_score.corpus_bleu / sentence_bleu docstrings)
    assert corpus_bleu([[R1A, R1B, R1C], [R2A]], [H1, H2]) == pytest.approx(0.5920778868801042, abs=1e-12)
    assert corpus_bleu([[R1A, R1B, R1C]], [H1]) == pytest.approx(0.5045666840058485, abs=1e-12)
    assert corpus_bleu([[R1A, R1B, R1C], [R2A]], [H1, H2], weights=(0.5, 0.5)) == pytest.approx(
        corpus_bleu([[R1A, R1B, R1C], [R2A]], [H1, H2], weights=(0.5, 0.5, 0.0, 0.0)), abs=1e-12)
    assert corpus_bleu([[['a', 'b']]], [['c', 'd']]) == 0.0  # no unigram match


def test_corpus_bleu_short_hypothesis_counts_in_denominator():
    """nltk's modified_precision divides by max(1, #hyp n-grams): a hypothesis shorter than n
    adds 0/1.  Worked by hand: p1 = 6/6, p2 = (4+0)/(4+1), hyp_len 6 vs ref_len 11, so
    BLEU-2 = exp(1 - 11/6) * sqrt(4/5)."""
    import math
    from imagecaptioningconvnext_amd.metrics import corpus_bleu
    refs = [[[1, 2, 3, 4, 5]], [[1, 2, 3, 4, 5, 6]]]
    hyps = [[1, 2, 3, 4, 5], [1]]
    want = math.exp(1 - 11 / 6) * math.sqrt(0.8)
    assert corpus_bleu(refs, hyps, weights=(0.5, 0.5)) == pytest.approx(want, abs=1e-12)
    assert want == pytest.approx(0.3887, abs=1e-4)


def _ref_preprocess(predictions, sequences, encodedCaptions, end, pad, maxlen):
    """utils.py:261-296 (the reference function, restated verbatim in behaviour)."""
    outs, tgts, lens = [], [], []
    for i in range(predictions.size(0)):
        if (sequences[i] == end).any():
            n = (sequences[i] == end).nonzero(as_tuple=True)[0][0].item() + 1
        else:
            n = maxlen
        lens.append(n)
        pl, gt = predictions[i, :n, :], encodedCaptions[i, 1:1 + n]
        keep = gt != pad
        if keep.sum() == 0:
            continue
        outs.append(pl[keep])
        tgts.append(gt[keep])
    return torch.cat(outs), torch.cat(tgts), lens


def test_metric_targets_match_reference_filtering():
    from imagecaptioningconvnext_amd.metrics import metric_targets
    g = torch.Generator().manual_seed(0)
    B, T, V, L, end, pad = 5, 9, 20, 12, 19, 0
    preds = torch.randn(B, T, V, generator=g)
    seqs = torch.randint(1, V - 1, (B, T), generator=g)
    seqs[0, 3] = end
    seqs[2, 0] = end
    seqs[4, 8] = end
    caps = torch.randint(1, V - 2, (B, L), generator=g)
    caps[1, 6:] = pad
    caps[3, 2:] = pad
    ref_s, ref_t, ref_n = _ref_preprocess(preds, seqs, caps, end, pad, T)
    tg, n = metric_targets(seqs, caps, end, pad, T)
    assert n.tolist() == ref_n
    keep = tg.reshape(-1) >= 0
    assert torch.equal(preds.reshape(B * T, V)[keep], ref_s) and torch.equal(tg.reshape(-1)[keep], ref_t)

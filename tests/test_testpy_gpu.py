"""test.py (the reference's evaluation entry point, test.py:144-215) on the HIP path: greedy
decoding of two batches, loss / top-5 accumulated per batch with the reference's AverageMeter
weighting (token counts), corpus BLEU-1..4 over the reference's filtering, checked against the
reference's own greedy outputs (tests/golden/greedy_small)."""
import importlib.util
import os

import pytest
import torch
import torch.nn.functional as F

from golden_util import word_map
from test_greedy_gpu import _decoder, _fixture
from test_metrics_cpu import _ref_preprocess

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("key", ["lstm_end", "trf_end"])
def test_testpy_matches_reference_accumulation(hip_device, key):
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    spec = importlib.util.spec_from_file_location("imgcap_testpy", os.path.join(root, "test.py"))
    testpy = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(testpy)
    from imagecaptioningconvnext_amd.metrics import corpus_bleu
    t, meta = _fixture()
    m = meta[key]
    cfg = m["cfg"]
    V, T = cfg["V"], m["maxDecodeLen"]
    lstm = key.startswith("lstm")
    dec = _decoder(lstm, cfg, m["end_bias_added"], hip_device)
    enc, preds, seqs = t[key + ".enc"], t[key + ".predictions"], t[key + ".sequences"]
    alphas = t.get(key + ".alphas")
    B = enc.shape[0]
    g = torch.Generator().manual_seed(5)
    caps = torch.randint(1, V - 3, (B, 14), generator=g)
    caps[:, 0] = V - 2
    caps[1, 6:] = 0
    allcaps = torch.randint(1, V - 3, (B, 3, 14), generator=g)
    allcaps[:, :, 0] = V - 2
    batches = [slice(0, 2), slice(2, B)]
    loader = [(enc[s], caps[s], torch.full((s.stop - s.start, 1), 14), allcaps[s]) for s in batches]
    wm = word_map(V)
    got = testpy.test(loader, None, dec, wordMap=wm, lstmDecoder=lstm, device=hip_device, maxDecodeLen=T,
                      log=lambda *a, **k: None)
    # the reference's loop on its own greedy outputs
    lsum = tsum = nsum = 0.0
    refs, hyps = [], []
    for s in batches:
        sc, tg, lens = _ref_preprocess(preds[s], seqs[s], caps[s], V - 1, 0, T)
        loss = F.cross_entropy(sc, tg)
        if lstm:
            loss = loss + ((1.0 - alphas[s].sum(dim=1)) ** 2).mean()
        n = tg.numel()
        top5 = (sc.topk(5, dim=1).indices == tg.view(-1, 1)).any(dim=1).float().sum().item() * 100.0 / n
        lsum, tsum, nsum = lsum + loss.item() * n, tsum + top5 * n, nsum + n
        for img in allcaps[s].tolist():
            refs.append([[w for w in c if w not in {V - 2, 0}] for c in img])
        hyps.extend(seq[:L] for seq, L in zip(seqs[s].tolist(), lens))
    want = [lsum / nsum, tsum / nsum] + [corpus_bleu(refs, hyps, weights=w) for w in
                                         ((1.0, 0.0, 0.0, 0.0), (0.5, 0.5, 0.0, 0.0), (0.33, 0.33, 0.33, 0.0),
                                          (0.25, 0.25, 0.25, 0.25))]
    assert abs(got[0] - want[0]) < 1e-5 * abs(want[0]) + 1e-6
    assert abs(got[1] - want[1]) < 1e-4
    for a, b in zip(got[2:], want[2:]):
        assert abs(a - b) < 1e-12

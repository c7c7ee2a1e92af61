"""Greedy decoding (decoder.py:119-163, transformerDecoder.py:110-160) on
the HIP path vs the reference's own forwardWithoutTeacherForcing (tests/golden/greedy_small,
tools/gen_golden.py greedy): sequences exact, predictions / alphas within fp32 tolerance,
including rows that emit <end> at different steps (the "_end" variants: <end>'s fc bias raised
as recorded in the fixture)."""
import json
import os

import pytest
import torch
from safetensors.torch import load_file

from golden_util import GOLDEN_DIR, make_params, word_map

pytestmark = pytest.mark.gpu


def _rel(a, b):
    a, b = a.detach().float().cpu(), b.detach().float().cpu()
    return ((a - b).norm() / (b.norm() + 1e-12)).item()


def _fixture():
    t = load_file(os.path.join(GOLDEN_DIR, "greedy_small.safetensors"))
    with open(os.path.join(GOLDEN_DIR, "greedy_small.json")) as f:
        return t, json.load(f)


def _decoder(lstm, cfg, end_bias, dev, dtype=torch.float32):
    if lstm:
        from imagecaptioningconvnext_amd.models.decoder import DecoderWithAttention
        dec = DecoderWithAttention(attention_dim=cfg["A"], embed_dim=cfg["Em"], decoder_dim=cfg["D"],
                                   vocab_size=cfg["V"], device=dev, encoder_dim=cfg["E"], dropout=0.0,
                                   compute_dtype=dtype)
    else:
        from imagecaptioningconvnext_amd.models.transformerDecoder import TransformerDecoder
        dec = TransformerDecoder(embed_dim=cfg["d"], decoder_dim=cfg["ff"], vocab_size=cfg["V"], maxLen=cfg["L"],
                                 device=dev, wordMap=None, pretrained_embeddings_path=None, fine_tune_embeddings=True,
                                 dropout=0.0, encoder_dim=cfg["E"], num_heads=cfg["H"], num_layers=cfg["layers"],
                                 compute_dtype=dtype)
    p = make_params({n: tuple(q.shape) for n, q in dec.named_parameters()}, cfg["seed"])
    fcb = "fc.bias" if lstm else "fc_out.bias"
    steps = round(end_bias / 0.05)
    for _ in range(steps):  # the generator added 0.05 per try, in fp32
        p[fcb][cfg["V"] - 1] += 0.05
    sd = dict(dec.state_dict())
    sd.update(p)
    dec.load_state_dict(sd)
    return dec.to(dev).eval()


@pytest.mark.parametrize("key", ["lstm", "lstm_end", "trf", "trf_end"])
def test_greedy_matches_reference(hip_device, key):
    t, meta = _fixture()
    m = meta[key]
    cfg = m["cfg"]
    lstm = key.startswith("lstm")
    dec = _decoder(lstm, cfg, m["end_bias_added"], hip_device)
    wm = word_map(cfg["V"])
    out = dec(teacherForcing=False, encoder_out=t[key + ".enc"].to(hip_device), wordMap=wm,
              maxDecodeLen=m["maxDecodeLen"])
    assert torch.equal(out[-1].cpu(), t[key + ".sequences"])
    assert _rel(out[0], t[key + ".predictions"]) < 1e-4
    if lstm:
        assert _rel(out[1], t[key + ".alphas"]) < 1e-4
    # finished rows: everything after the <end> step stays zero, as the reference's torch.zeros
    seq = t[key + ".sequences"]
    for b in range(seq.shape[0]):
        ends = (seq[b] == cfg["V"] - 1).nonzero().flatten().tolist()
        if ends:
            assert out[0][b, ends[0] + 1:].abs().max().item() == 0.0


def test_greedy_bf16_runs_and_agrees_mostly(hip_device):
    """bf16 compute: same API and shapes; the argmax path may differ only where logits nearly tie."""
    t, meta = _fixture()
    m = meta["trf"]
    dec = _decoder(False, m["cfg"], 0.0, hip_device, torch.bfloat16)
    preds, seqs = dec(teacherForcing=False, encoder_out=t["trf.enc"].to(hip_device), wordMap=word_map(m["cfg"]["V"]),
                      maxDecodeLen=m["maxDecodeLen"])
    assert preds.shape == t["trf.predictions"].shape and preds.dtype == torch.float32
    assert (seqs.cpu() == t["trf.sequences"]).float().mean().item() > 0.7


@pytest.mark.parametrize("key", ["lstm_end", "trf_end"])
def test_greedy_validation_loss_matches_reference_filtering(hip_device, key):
    """metrics.greedy_loss (device) == train.py:398-407: preprocessDecoderOutputForMetrics +
    CrossEntropyLoss (+ the LSTM's alpha regulariser) + top-5 over the kept rows."""
    import torch.nn.functional as F
    from imagecaptioningconvnext_amd.metrics import greedy_loss
    from test_metrics_cpu import _ref_preprocess
    t, meta = _fixture()
    m = meta[key]
    cfg = m["cfg"]
    V, T = cfg["V"], m["maxDecodeLen"]
    preds, seqs = t[key + ".predictions"], t[key + ".sequences"]
    g = torch.Generator().manual_seed(3)
    caps = torch.randint(1, V - 3, (preds.shape[0], 14), generator=g)
    caps[1, 5:] = 0
    alphas = t.get(key + ".alphas")
    metrics, n = greedy_loss(preds.to(hip_device), seqs.to(hip_device), caps.to(hip_device), word_map(V), T,
                             alphas=None if alphas is None else alphas.to(hip_device))
    s, tg, lens = _ref_preprocess(preds, seqs, caps, V - 1, 0, T)
    loss = F.cross_entropy(s, tg)
    if alphas is not None:
        loss = loss + ((1.0 - alphas.sum(dim=1)) ** 2).mean()
    top5 = (s.topk(5, dim=1).indices == tg.view(-1, 1)).any(dim=1).float().sum()
    mm = metrics.cpu()
    assert n.cpu().tolist() == lens
    assert abs(mm[0].item() - loss.item()) < 1e-5 * abs(loss.item()) + 1e-6
    assert int(mm[1].item()) == tg.numel() and int(mm[2].item()) == int(top5.item())

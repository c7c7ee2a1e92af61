"""Attention-visualisation decoder (models/transformerDecoderAttVis.py,
caption.py:260-383) on the HIP path vs the reference's own TransformerDecoderForAttentionViz and
caption_image_beam_search_transformer_attention (tests/golden/attvis_small, tools/gen_golden.py
attvis; 2 heads of 64, 2 layers): teacher-forced predictions and alphas [H, B, P], greedy
predictions / sequences / alphas with rows ending at different steps, beam word ids and attention
maps for beam sizes 3 and 5.  fp32 engine: rel <= 1e-4 (predictions), abs <= 1e-5 (alphas)."""
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
    t = load_file(os.path.join(GOLDEN_DIR, "attvis_small.safetensors"))
    with open(os.path.join(GOLDEN_DIR, "attvis_small.json")) as f:
        return t, json.load(f)


def _decoder(cfg, dev, end_bias_steps=0, end_bias=0.0):
    from imagecaptioningconvnext_amd.models.transformerDecoderAttVis import TransformerDecoderForAttentionViz
    dec = TransformerDecoderForAttentionViz(embed_dim=cfg["d"], decoder_dim=cfg["ff"], vocab_size=cfg["V"],
                                            maxLen=cfg["L"], device=dev, dropout=0.0, encoder_dim=cfg["E"],
                                            num_heads=cfg["H"], num_layers=cfg["layers"], compute_dtype=torch.float32)
    p = make_params({n: tuple(q.shape) for n, q in dec.named_parameters()}, cfg["seed"])
    for _ in range(end_bias_steps):  # the generator's greedy search added 0.05 per try, in fp32
        p["fc_out.bias"][cfg["V"] - 1] += 0.05
    p["fc_out.bias"][cfg["V"] - 1] += end_bias
    sd = dict(dec.state_dict())
    sd.update(p)
    dec.load_state_dict(sd)
    return dec.to(dev).eval()


def test_attvis_state_dict_keys_match_reference_layout(hip_device):
    t, meta = _fixture()
    dec = _decoder(meta["tf"]["cfg"], hip_device)
    keys = list(dec.state_dict())
    assert "decoder_layers.1.multihead_attn.in_proj_weight" in keys and "pos_encoding.pe" in keys
    assert not any(k.startswith("transformer_decoder.") for k in keys)


def test_attvis_teacher_forced_predictions_and_alphas(hip_device):
    t, meta = _fixture()
    cfg = meta["tf"]["cfg"]
    dec = _decoder(cfg, hip_device)
    caps = t["tf.caps"].to(hip_device)
    preds, caps_out, dls, alphas = dec(teacherForcing=True, encoder_out=t["tf.enc"].to(hip_device),
                                       encoded_captions=caps, caption_lengths=t["tf.caplens"].to(hip_device),
                                       tgt_key_padding_mask=caps == 0)
    assert dls == meta["tf"]["decode_lengths"]
    assert _rel(preds, t["tf.predictions"]) < 1e-4
    assert alphas.shape == t["tf.alphas"].shape  # [H, B, P]
    assert (alphas.cpu() - t["tf.alphas"]).abs().max().item() < 1e-5
    # the predictions stay differentiable (same autograd path as TransformerDecoder)
    preds.sum().backward()
    assert dec.fc_out.weight.grad is not None


def test_attvis_greedy_matches_reference(hip_device):
    t, meta = _fixture()
    cfg = meta["tf"]["cfg"]
    dec = _decoder(cfg, hip_device, end_bias_steps=round(meta["greedy"]["end_bias_added"] / 0.05))
    wm = word_map(cfg["V"])
    preds, seqs, alphas = dec(teacherForcing=False, encoder_out=t["tf.enc"].to(hip_device), wordMap=wm,
                              maxDecodeLen=meta["greedy"]["maxDecodeLen"])
    ref_seq = t["greedy.sequences"]
    assert torch.equal(seqs.cpu(), ref_seq)
    ends = {(row == cfg["V"] - 1).nonzero()[:1].flatten().tolist()[0] if (row == cfg["V"] - 1).any() else -1
            for row in ref_seq}
    assert len(ends) >= 2  # rows stop at different steps: the finished-row bookkeeping is exercised
    assert _rel(preds, t["greedy.predictions"]) < 1e-4
    assert (alphas.cpu() - t["greedy.alphas"]).abs().max().item() < 1e-5


@pytest.mark.parametrize("k", [3, 5])
def test_attvis_beam_search_matches_reference(hip_device, k):
    from imagecaptioningconvnext_amd import beam
    from test_beam_gpu import _FixedEncoder
    t, meta = _fixture()
    cfg = meta["beam"]["cfg"]
    dec = _decoder(cfg, hip_device, end_bias=meta["beam"]["end_bias_added"])
    enc = _FixedEncoder(t["beam.feats"].to(hip_device))
    image = torch.zeros(3, 256, 256, dtype=torch.uint8)
    seq, alphas = beam.caption_image_beam_search_transformer_attention(enc, dec, image, word_map(cfg["V"]), "unused",
                                                                        beamSize=k)
    assert seq == t[f"beam.k{k}.seq"].tolist()
    got = torch.tensor(alphas)
    assert got.shape == t[f"beam.k{k}.alphas"].shape  # [max_decode_len, P], zero past the caption
    assert (got - t[f"beam.k{k}.alphas"]).abs().max().item() < 1e-5
    assert got[len(seq) - 1:].abs().sum().item() == 0.0

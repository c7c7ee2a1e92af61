"""Beam search (caption.py:39-255) on the HIP path vs the reference's own
caption_image_beam_search / caption_image_beam_search_transformer run on the same features
(tests/golden/beam_small, tools/gen_golden.py beam): returned word ids exact, LSTM attention
maps within fp32 tolerance, beam sizes 3 and 5."""
import json
import os

import pytest
import torch
from safetensors.torch import load_file

from golden_util import GOLDEN_DIR, word_map
from test_greedy_gpu import _decoder

pytestmark = pytest.mark.gpu


class _FixedEncoder(torch.nn.Module):
    def __init__(self, feats):
        super().__init__()
        self.feats = feats

    def forward(self, image):
        assert image.dim() == 4 and image.shape[:2] == (1, 3)
        return self.feats


@pytest.mark.parametrize("name", ["lstm", "trf"])
@pytest.mark.parametrize("k", [3, 5])
def test_beam_search_matches_reference(hip_device, name, k):
    from imagecaptioningconvnext_amd import beam
    t = load_file(os.path.join(GOLDEN_DIR, "beam_small.safetensors"))
    with open(os.path.join(GOLDEN_DIR, "beam_small.json")) as f:
        meta = json.load(f)[name]
    cfg = meta["cfg"]
    lstm = name == "lstm"
    dec = _decoder(lstm, cfg, 0.0, hip_device)
    with torch.no_grad():
        (dec.fc if lstm else dec.fc_out).bias[cfg["V"] - 1] += meta["end_bias_added"]
    enc = _FixedEncoder(t[f"{name}.feats"].to(hip_device))
    image = torch.zeros(3, 256, 256, dtype=torch.uint8)
    wm = word_map(cfg["V"])
    if lstm:
        seq, alphas = beam.caption_image_beam_search(enc, dec, image, wm, beamSize=k)
        ref_a = t[f"{name}.k{k}.alphas"]
        got_a = torch.tensor(alphas)
        assert got_a.shape == ref_a.shape
        assert (got_a - ref_a).abs().max().item() < 1e-4
    else:
        seq, none = beam.caption_image_beam_search_transformer(enc, dec, image, wm, beamSize=k)
        assert none is None
    assert seq == t[f"{name}.k{k}.seq"].tolist()
    assert seq[0] == cfg["V"] - 2 and seq[-1] == cfg["V"] - 1

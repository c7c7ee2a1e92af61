"""Checkpoint schema compatibility (utils.py:195-224, train.py:118-147)
against checkpoints written by the reference's own save_checkpoint (tests/golden/ckpt_*,
made by tools/gen_golden.py ckpt).  CPU only: flat fp32 buffers, no kernel launches."""
import json
import os

import pytest
import torch

from golden_util import GOLDEN_DIR


def _fixture(name):
    from imagecaptioningconvnext_amd.checkpoint import load_checkpoint
    ck = load_checkpoint(os.path.join(GOLDEN_DIR, name + ".pth.tar"))
    with open(os.path.join(GOLDEN_DIR, name + ".json")) as f:
        return ck, json.load(f)


def _decoder(lstm, cfg):
    if lstm:
        from imagecaptioningconvnext_amd.models.decoder import DecoderWithAttention
        return DecoderWithAttention(attention_dim=cfg["A"], embed_dim=cfg["Em"], decoder_dim=cfg["D"],
                                    vocab_size=cfg["V"], device="cpu", encoder_dim=cfg["E"], dropout=0.0)
    from imagecaptioningconvnext_amd.models.transformerDecoder import TransformerDecoder
    return TransformerDecoder(embed_dim=cfg["d"], decoder_dim=cfg["ff"], vocab_size=cfg["V"], maxLen=cfg["L"],
                              device="cpu", wordMap=None, pretrained_embeddings_path=None, fine_tune_embeddings=True,
                              dropout=0.0, encoder_dim=cfg["E"], num_heads=cfg["H"], num_layers=cfg["layers"])


def _flat(dec):
    from imagecaptioningconvnext_amd.flat import FlatParams
    return FlatParams([[(n, p)] for n, p in dec.named_parameters()], "cpu", torch.float32)


@pytest.mark.parametrize("lstm", [True, False])
def test_reference_checkpoint_roundtrip(lstm, tmp_path):
    from imagecaptioningconvnext_amd import checkpoint as C
    name = "ckpt_lstm_small" if lstm else "ckpt_transformer_small"
    ck, meta = _fixture(name)
    assert set(ck) == {'epoch', 'epochsSinceImprovement', 'bleu-4', 'encoder', 'decoder', 'encoderOptimizer',
                       'decoderOptimizer', 'results'}
    dec = _decoder(lstm, meta["cfg"])
    dec.load_state_dict(ck["decoder"])  # strict: same keys and shapes as the reference module
    params = C.trainable_parameters(dec)
    names = {id(p): n for n, p in dec.named_parameters()}
    assert [names[id(p)] for p in params] == meta["param_order"]  # Adam's parameter indices line up
    fp = _flat(dec)
    lr = C.load_optimizer_state_dict(fp, params, ck["decoderOptimizer"])
    assert lr == ck["decoderOptimizer"]["param_groups"][0]["lr"] and fp.step_count == 1
    out = C.optimizer_state_dict(fp, params, lr)
    ref = ck["decoderOptimizer"]
    assert out["param_groups"] == [dict(g, betas=tuple(g["betas"])) for g in ref["param_groups"]]
    assert set(out["state"]) == set(ref["state"])
    for i, st in ref["state"].items():
        assert torch.equal(out["state"][i]["step"], st["step"])
        assert torch.equal(out["state"][i]["exp_avg"], st["exp_avg"])
        assert torch.equal(out["state"][i]["exp_avg_sq"], st["exp_avg_sq"])
    # the state dict written here loads into the reference's optimizer (torch.optim.Adam over
    # the same parameter list) and the file has the reference's name and schema
    torch.optim.Adam(params=[torch.nn.Parameter(p.detach().clone()) for p in params], lr=1e-4).load_state_dict(out)
    path = C.save_checkpoint("coco_5_cap_per_img_5_min_word_freq", 0, 0, None, dec.state_dict(), None, out, 0.0,
                             True, [], lstm, 5, 1e-4, None if lstm else "none", directory=str(tmp_path))
    assert os.path.basename(path) == meta["filename"]
    assert os.path.exists(os.path.join(str(tmp_path), "BEST_" + meta["filename"]))
    back = C.load_checkpoint(path)
    assert set(back) == set(ck)
    for k, v in ck["decoder"].items():
        assert torch.equal(back["decoder"][k], v), k


def test_optimizer_state_rejects_mismatch():
    from imagecaptioningconvnext_amd import checkpoint as C
    ck, meta = _fixture("ckpt_lstm_small")
    dec = _decoder(True, meta["cfg"])
    fp = _flat(dec)
    params = C.trainable_parameters(dec)
    with pytest.raises(ValueError):
        C.load_optimizer_state_dict(fp, params[:-1], ck["decoderOptimizer"])
    bad = {"state": dict(ck["decoderOptimizer"]["state"]), "param_groups": ck["decoderOptimizer"]["param_groups"]}
    bad["state"][0] = dict(bad["state"][0], step=torch.tensor(2.0))
    with pytest.raises(ValueError):
        C.load_optimizer_state_dict(fp, params, bad)

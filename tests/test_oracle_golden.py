"""Pin the CPU oracle against golden vectors produced by the real reference (tools/gen_golden.py)."""
import json
import os

import pytest
import torch
from safetensors.torch import load_file

from golden_util import GOLDEN_DIR, make_captions, make_features, make_params
from oracle import convnext, decoders, train_step


def _load(name):
    t = load_file(os.path.join(GOLDEN_DIR, name + ".safetensors"))
    with open(os.path.join(GOLDEN_DIR, name + ".json")) as f:
        meta = json.load(f)
    return t, meta


def _params(t):
    return {k[len("param."):]: v.clone().requires_grad_(True) for k, v in t.items() if k.startswith("param.")}


def _close(a, b, rtol=1e-5, atol=1e-6):
    torch.testing.assert_close(a, b, rtol=rtol, atol=atol)


def _check_post(new, t, grads, lr=1e-4):
    """Post-Adam params vs the reference's.  Adam's first step moves each weight by ~lr*sign(g);
    where g is round-off noise (the attention key bias and full_att.bias have true gradient 0:
    softmax is shift-invariant) the sign is arbitrary, so those entries need only agree within
    2*lr; all others to 1e-6."""
    for k, v in new.items():
        ref = t["post." + k]
        deg = grads[k].abs() < 1e-6
        torch.testing.assert_close(v[~deg], ref[~deg], rtol=1e-5, atol=1e-6)
        if deg.any():
            assert (v[deg] - ref[deg]).abs().max().item() <= 2 * lr * 1.0001


def test_convnext_known_answers():
    # torchvision's published totals (incl. classifier) and GFLOPS at 224x224
    for v, n, g in (("tiny", 28589128, 4.46), ("base", 88591464, 15.36), ("large", 197767336, 34.36)):
        assert convnext.param_count(v) + convnext.classifier_params(v) == n
        assert abs(convnext.macs_per_image(v) / 1e9 - g) < 0.01


def test_convnext_shapes_and_pool():
    sd = convnext.init_params("tiny")
    x = torch.randn(1, 3, 224, 224)
    out = convnext.encoder_forward(sd, "tiny", x)
    assert out.shape == (1, 7, 7, 768)
    out256 = convnext.encoder_forward(sd, "tiny", torch.randn(1, 3, 256, 256))
    assert out256.shape == (1, 7, 7, 768)


def test_lstm_small_forward_loss_grads_step():
    t, meta = _load("lstm_tf_small")
    p = _params(t)
    preds, caps_sorted, dls, alphas, sort_ind = decoders.lstm_tf_forward(p, t["enc"], t["caps"], t["caplens"])
    assert dls == meta["decode_lengths"]
    _close(preds, t["predictions"])
    _close(alphas, t["alphas"])
    assert torch.equal(sort_ind, t["sort_ind"]) and torch.equal(caps_sorted, t["caps_sorted"])
    loss, scores, targets = train_step.lstm_loss(preds, caps_sorted, dls, alphas)
    _close(scores, t["packed_scores"])
    assert torch.equal(targets, t["packed_targets"])
    _close(loss.detach().view(1), t["loss"])
    loss.backward()
    grads = {k: v.grad for k, v in p.items()}
    for k, g in grads.items():
        _close(g, t["grad." + k], rtol=1e-4, atol=1e-6)
    # one clip + Adam step == the reference's own train.trainWithTeacherForcing
    new = train_step.adam_step({k: v.detach() for k, v in p.items()}, train_step.clip_gradient(grads, 5.0), {}, 1e-4, 1)
    _check_post(new, t, grads)
    _close(loss.detach().view(1).double(), t["ref_step_loss"].double(), rtol=1e-5, atol=1e-6)
    top5 = train_step.top5_correct(scores, targets) * 100.0 / targets.numel()
    assert abs(top5 - float(t["ref_step_top5"])) < 1e-5


def test_transformer_small_forward_loss_grads_step():
    t, meta = _load("transformer_tf_small")
    p = _params(t)
    cfg = meta["cfg"]
    mask = t["caps"] == 0
    preds, caps, dls = decoders.transformer_tf_forward(p, t["enc"], t["caps"], t["caplens"], mask,
                                                       cfg["H"], cfg["layers"], pe=t["pe"])
    assert dls == meta["decode_lengths"]
    _close(preds, t["predictions"], rtol=1e-4, atol=1e-5)
    loss, scores, targets = train_step.transformer_loss(preds, caps, dls)
    assert torch.equal(targets, t["packed_targets"])
    _close(loss.detach().view(1), t["loss"], rtol=1e-5, atol=1e-6)
    loss.backward()
    grads = {k: v.grad for k, v in p.items()}
    for k, g in grads.items():
        _close(g, t["grad." + k], rtol=1e-3, atol=1e-5)
    new = train_step.adam_step({k: v.detach() for k, v in p.items()}, train_step.clip_gradient(grads, 5.0), {}, 1e-4, 1)
    _check_post(new, t, grads)


def test_ddp2_average_then_clip_adam():
    """trainMultiGPU: DDP mean of per-rank grads, then clip + Adam (trainMultiGPU.py:384-394)."""
    t, meta = _load("ddp2_lstm")
    s, _ = _load("lstm_tf_small")
    base = {k[len("param."):]: v for k, v in s.items() if k.startswith("param.")}
    grads = []
    losses, toks, c5 = [], [], 0.0
    for r in range(2):
        p = {k: v.clone().requires_grad_(True) for k, v in base.items()}
        preds, cs, dls, al, _ = decoders.lstm_tf_forward(p, t[f"rank{r}.enc"], t[f"rank{r}.caps"], t[f"rank{r}.caplens"])
        loss, scores, targets = train_step.lstm_loss(preds, cs, dls, al)
        loss.backward()
        grads.append({k: v.grad for k, v in p.items()})
        losses.append(float(loss))
        toks.append(sum(dls))
        c5 += train_step.top5_correct(scores, targets)
    avg = {k: (grads[0][k] + grads[1][k]) / 2 for k in base}
    new = train_step.adam_step(base, train_step.clip_gradient(avg, 5.0), {}, 1e-4, 1)
    _check_post(new, t, avg)
    # reduceLossAndTokens (trainMultiGPU.py:96-108): token-weighted global loss
    gl = (losses[0] * toks[0] + losses[1] * toks[1]) / (toks[0] + toks[1])
    assert abs(gl - float(t["ref_loss"])) < 1e-5
    assert abs(c5 / sum(toks) * 100 - float(t["ref_top5"])) < 1e-4


@pytest.mark.parametrize("name", ["lstm_full_spot", "transformer_full_spot"])
def test_full_size_spot(name):
    t, meta = _load(name)
    cfg = meta["cfg"]
    from oracle import shapes
    if name.startswith("lstm"):
        p = make_params(shapes.lstm_decoder_shapes(cfg["E"], cfg["A"], cfg["D"], cfg["Em"], cfg["V"]), cfg["seed"])
    else:
        p = make_params(shapes.transformer_decoder_shapes(cfg["E"], cfg["d"], cfg["ff"], cfg["V"], cfg["layers"]),
                        cfg["seed"])
    enc = make_features((cfg["B"], cfg["S"], cfg["S"], cfg["E"]), cfg["seed"] + 1)
    caps, caplens = make_captions(cfg["B"], cfg["L"], cfg["caplens"], cfg["V"], cfg["seed"] + 2)
    with torch.no_grad():
        if name.startswith("lstm"):
            preds, cs, dls, al, _ = decoders.lstm_tf_forward(p, enc, caps, caplens)
            loss, scores, _ = train_step.lstm_loss(preds, cs, dls, al)
        else:
            preds, cs, dls = decoders.transformer_tf_forward(p, enc, caps, caplens, caps == 0, cfg["H"], cfg["layers"])
            loss, scores, _ = train_step.transformer_loss(preds, cs, dls)
    assert dls == meta["decode_lengths"]
    _close(loss.view(1), t["loss"], rtol=1e-5, atol=1e-5)
    _close(scores[t["rows"], t["cols"]], t["values"], rtol=1e-4, atol=1e-5)

"""LSTM-attention decoder on the HIP path vs the golden vectors of the reference and the CPU
oracle (decoder.py:69-113, train.py:263-291)."""
import json
import os

import pytest
import torch
from safetensors.torch import load_file

from golden_util import GOLDEN_DIR, make_captions, make_features, make_params
from oracle import decoders, shapes, train_step

pytestmark = pytest.mark.gpu


def _load(name):
    t = load_file(os.path.join(GOLDEN_DIR, name + ".safetensors"))
    with open(os.path.join(GOLDEN_DIR, name + ".json")) as f:
        return t, json.load(f)


def _decoder(cfg, params, dtype, dev, dropout=0.0):
    from imagecaptioningconvnext_amd.models.decoder import DecoderWithAttention
    dec = DecoderWithAttention(attention_dim=cfg["A"], embed_dim=cfg["Em"], decoder_dim=cfg["D"], vocab_size=cfg["V"],
                               device=dev, encoder_dim=cfg["E"], dropout=dropout, compute_dtype=dtype)
    dec.load_state_dict(params)
    return dec.to(dev)


def _rel(a, b):
    a, b = a.detach().float().cpu(), b.detach().float().cpu()
    return ((a - b).norm() / (b.norm() + 1e-12)).item()


def test_lstm_small_reference_api_and_grads(hip_device):
    """Module API (predictions/alphas/sort) + autograd grads vs the reference golden (fp32)."""
    t, meta = _load("lstm_tf_small")
    cfg = meta["cfg"]
    params = {k[6:]: v for k, v in t.items() if k.startswith("param.")}
    dec = _decoder(cfg, params, torch.float32, hip_device)
    enc = t["enc"].to(hip_device)
    preds, caps_s, dls, alphas, sort_ind = dec(teacherForcing=True, encoder_out=enc,
                                               encoded_captions=t["caps"].to(hip_device),
                                               caption_lengths=t["caplens"].to(hip_device))
    assert dls == meta["decode_lengths"]
    assert torch.equal(sort_ind.cpu(), t["sort_ind"]) and torch.equal(caps_s.cpu(), t["caps_sorted"])
    assert _rel(preds, t["predictions"]) < 1e-5
    assert _rel(alphas, t["alphas"]) < 1e-5
    loss, _, _ = train_step.lstm_loss(preds, caps_s, dls, alphas)
    assert abs(loss.item() - t["loss"].item()) < 1e-5 * abs(t["loss"].item())
    for p in dec.parameters():
        p.grad = None
    loss.backward()
    for n, p in dec.named_parameters():
        if n == "attention.full_att.bias":  # true gradient 0 (softmax shift invariance)
            assert p.grad.abs().max().item() < 1e-6
            continue
        assert _rel(p.grad, t["grad." + n]) < 1e-4, n


@pytest.mark.parametrize("dtype,tol", [(torch.float32, 1e-4), (torch.bfloat16, 3e-2)])
def test_lstm_small_fused_step(hip_device, dtype, tol):
    """Fused engine: loss, grads, and one clip+Adam step vs the reference's own train step."""
    t, meta = _load("lstm_tf_small")
    cfg = meta["cfg"]
    params = {k[6:]: v for k, v in t.items() if k.startswith("param.")}
    dec = _decoder(cfg, params, dtype, hip_device)
    eng = dec.engine()
    s = eng.forward(t["enc"].to(hip_device), t["caps"].to(hip_device), t["caplens"].to(hip_device), fixed_T=True)
    m = s["metrics"].cpu()
    assert abs(m[0].item() - t["loss"].item()) < tol * abs(t["loss"].item())
    assert int(m[1].item()) == sum(meta["decode_lengths"])
    if dtype == torch.float32:
        assert abs(m[2].item() / m[1].item() * 100 - t["ref_step_top5"].item()) < 1e-4
    # the fused top-5 count is exact for the logits the kernel saw: target's rank among strictly
    # greater logits < 5 (utils.py:248-250 topk), recomputed here from the engine's own logits
    lg = s["logits"][:, :cfg["V"]].float()
    tg = s["targets"]
    ok = tg >= 0
    tl = lg[ok].gather(1, tg[ok].view(-1, 1))
    assert int(m[2].item()) == int(((lg[ok] > tl).sum(1) < 5).sum().item())
    eng.backward(s)
    for n in eng.fp.params:
        if n == "attention.full_att.bias":
            continue
        assert _rel(eng.fp.g(n), t["grad." + n]) < tol * (1 if dtype == torch.float32 else 2), n
    eng.fp.adam_step(1e-4, 5.0)
    if dtype == torch.float32:
        for n, p in dec.named_parameters():
            ref = t["post." + n]
            g = t["grad." + n]
            ok = g.abs() >= 1e-6  # Adam's first step is sign(g)*lr; noise-level grads excluded
            torch.testing.assert_close(p.detach().cpu()[ok], ref[ok], rtol=1e-5, atol=2e-6)


@pytest.mark.parametrize("dtype,tol", [(torch.float32, 1e-4), (torch.bfloat16, 2e-2)])
def test_lstm_full_size_spot(hip_device, dtype, tol):
    """Full-size dims (E=768, V=9490, A=D=512, L=52): loss + sampled logits vs the reference."""
    t, meta = _load("lstm_full_spot")
    cfg = meta["cfg"]
    p = make_params(shapes.lstm_decoder_shapes(cfg["E"], cfg["A"], cfg["D"], cfg["Em"], cfg["V"]), cfg["seed"])
    dec = _decoder(cfg, p, dtype, hip_device)
    enc = make_features((cfg["B"], cfg["S"], cfg["S"], cfg["E"]), cfg["seed"] + 1).to(hip_device)
    caps, caplens = make_captions(cfg["B"], cfg["L"], cfg["caplens"], cfg["V"], cfg["seed"] + 2)
    with torch.no_grad():
        preds, cs, dls, al, _ = dec(True, enc, caps.to(hip_device), caplens.to(hip_device))
    assert dls == meta["decode_lengths"]
    loss, scores, _ = train_step.lstm_loss(preds.cpu(), cs.cpu(), dls, al.cpu())
    assert abs(loss.item() - t["loss"].item()) < tol * abs(t["loss"].item())
    got = scores[t["rows"], t["cols"]]
    print(f"lstm full size {dtype}: loss rel {abs(loss.item() / t['loss'].item() - 1):.2e}, "
          f"logits rel {_rel(got, t['values']):.2e}, alphas rel {_rel(al, t['alphas']):.2e}")
    assert _rel(got, t["values"]) < (1e-4 if dtype == torch.float32 else 1e-2)
    assert _rel(al, t["alphas"]) < (1e-4 if dtype == torch.float32 else 1e-2)


def test_lstm_medium_vs_oracle_with_dropout_determinism(hip_device):
    """Random medium case (P=49, variable lengths) vs the oracle (fp32), and dropout path sanity."""
    torch.manual_seed(0)
    E, A, D, Em, V, B, L = 64, 32, 32, 32, 300, 5, 20
    p = make_params(shapes.lstm_decoder_shapes(E, A, D, Em, V), 77)
    cfg = dict(E=E, A=A, D=D, Em=Em, V=V)
    enc = make_features((B, 7, 7, E), 78)
    caps, caplens = make_captions(B, L, [20, 5, 13, 13, 9], V, 79)
    pr = {k: v.clone().requires_grad_(True) for k, v in p.items()}
    preds, cs, dls, al, _ = decoders.lstm_tf_forward(pr, enc, caps, caplens)
    loss, _, _ = train_step.lstm_loss(preds, cs, dls, al)
    loss.backward()
    dec = _decoder(cfg, p, torch.float32, hip_device)
    eng = dec.engine()
    s = eng.forward(enc.to(hip_device), caps.to(hip_device), caplens.to(hip_device), fixed_T=True)
    assert abs(s["metrics"][0].item() - loss.item()) < 1e-4 * loss.item()
    eng.backward(s)
    for n in eng.fp.params:
        if n == "attention.full_att.bias":
            continue
        assert _rel(eng.fp.g(n), pr[n].grad) < 1e-4, n
    # dropout active: deterministic for a fixed seed, and changes the loss
    dec.train()
    dec.dropout_p = 0.5
    eng.step_id = 0
    s1 = eng.forward(enc.to(hip_device), caps.to(hip_device), caplens.to(hip_device), fixed_T=True)
    eng.step_id = 0
    s2 = eng.forward(enc.to(hip_device), caps.to(hip_device), caplens.to(hip_device), fixed_T=True)
    assert torch.equal(s1["metrics"], s2["metrics"])
    assert abs(s1["metrics"][0].item() - loss.item()) > 1e-4


def _live_mask(lens, T, dev):
    """[B, T] True where step t < the decode length of sorted row b (caption length - 1)"""
    dls = torch.tensor(sorted((n - 1 for n in lens), reverse=True), device=dev)
    return torch.arange(T, device=dev)[None, :] < dls[:, None]


@pytest.mark.parametrize("dtype,B", [(torch.float32, 5), (torch.bfloat16, 32), (torch.float32, 24)])
def test_lstm_persistent_recurrence_matches_per_step(hip_device, dtype, B):
    """The one-launch forward recurrence (csrc/lstm_persist.hip) against the per-step launches
    on the same descriptor: every saved buffer for t < max decode length, zeros past it."""
    import ctypes
    from imagecaptioningconvnext_amd import _abi
    from imagecaptioningconvnext_amd import kernels as K
    E, A, D, Em, V, L = (768, 512, 512, 512, 300, 24) if B == 32 else (64, 32, 48, 32, 100, 14)
    p = make_params(shapes.lstm_decoder_shapes(E, A, D, Em, V), 5)
    dec = _decoder(dict(E=E, A=A, D=D, Em=Em, V=V), p, dtype, hip_device)
    eng = dec.engine()
    enc = make_features((B, 7, 7, E), 6).to(hip_device).to(dtype)
    lens = [L - 3 - (i * 7) % (L - 6) for i in range(B)]  # maximum L - 3 < L: skipped tail steps
    caps, caplens = make_captions(B, L, lens, V, 7)
    s = eng.forward(enc, caps.to(hip_device), caplens.to(hip_device), fixed_T=True, loss=False)
    torch.cuda.synchronize()
    d = s["desc"]
    assert d.sync and eng.sync_error() == 0
    names = ("alphas", "awe", "zs", "gates", "cs", "hs", "hprev")
    got = {k: s[k].clone() for k in names}
    g1 = s["g1"][..., :A + E].clone()
    for k in names:
        (s[k][:, 1:] if k == "hprev" else s[k]).fill_(float("nan"))  # hprev slot 0 = h0 (input)
    d.sync, d.sync_words = None, 0
    _abi.call("imgcap_lstm_tf_fwd", ctypes.byref(d), K.stream())
    torch.cuda.synchronize()
    T, tm = s["T"], max(lens) - 1
    tol = 1e-5 if dtype == torch.float32 else 2e-2
    # rows past their own decode length are don't-care (decoder.py:95 runs batch_size_t rows):
    # with row groups (B > 16) a group stops at its own longest row
    live = _live_mask(lens, T, hip_device)
    for k in names:
        a, b = got[k].float(), s[k].float()
        lo = 1 if k == "hprev" else 0  # hprev slot t holds h_{t-1}
        assert _rel(a[live], b[live]) < tol, k
        assert torch.all(a[:, tm + lo:] == 0), k
    assert torch.equal(got["alphas"], s["alphas"]) or _rel(got["alphas"], s["alphas"]) < tol
    assert _rel(g1[live], s["g1"][..., :A + E][live]) < tol


@pytest.mark.parametrize("dtype,B", [(torch.float32, 5), (torch.bfloat16, 32), (torch.float32, 24),
                                     (torch.bfloat16, 13)])
def test_lstm_persistent_backward_matches_per_step(hip_device, dtype, B):
    """The one-launch backward recurrence (lstm_bwd_persist_kernel) against the per-step launches
    on the same descriptor: dcat ([d att2 | d gate_pre | dgates] per step), de, dawe, dL/dh0,
    dL/dc0 and the attention-parameter partials computed from them; zeros past max(dl)."""
    import ctypes
    from imagecaptioningconvnext_amd import _abi
    from imagecaptioningconvnext_amd import kernels as K
    E, A, D, Em, V, L = (768, 512, 512, 512, 300, 24) if B == 32 else (64, 32, 48, 32, 100, 14)
    p = make_params(shapes.lstm_decoder_shapes(E, A, D, Em, V), 8)
    dec = _decoder(dict(E=E, A=A, D=D, Em=Em, V=V), p, dtype, hip_device)
    eng = dec.engine()
    enc = make_features((B, 7, 7, E), 9).to(hip_device).to(dtype)
    lens = [L - 3 - (i * 5) % (L - 6) for i in range(B)]  # maximum L - 3 < L: skipped tail steps
    caps, caplens = make_captions(B, L, lens, V, 10)
    s = eng.forward(enc, caps.to(hip_device), caplens.to(hip_device), fixed_T=True)
    eng.backward(s, want_denc=True)
    torch.cuda.synchronize()
    d = s["desc"]
    assert d.sync and eng.sync_error() == 0
    bufs = s["bwd_bufs"]
    names = ("dcat", "de", "dh", "dc", "datt1", "dwf", "dbea")
    got = {k: bufs[k].clone() for k in names}
    T = s["T"]
    got["dawe"] = bufs["dawe"][:, :T].clone()
    for k in names:
        bufs[k].fill_(float("nan"))
    bufs["dawe"][:, :T].fill_(float("nan"))
    d.sync, d.sync_words = None, 0
    _abi.call("imgcap_lstm_tf_bwd", ctypes.byref(d), K.stream())
    torch.cuda.synchronize()
    tm = max(lens) - 1
    tol = 1e-5 if dtype == torch.float32 else 2e-2
    live = _live_mask(lens, T, hip_device)
    for k in names + ("dawe",):
        a, b = got[k].float(), (bufs[k][:, :T] if k == "dawe" else bufs[k]).float()
        assert torch.isfinite(a).all(), k
        if k in ("dcat", "de", "dawe"):
            assert _rel(a[live], b[live]) < tol, k
            assert torch.all(a[:, tm:] == 0), k
        else:
            assert _rel(a, b) < tol, k

"""Transformer decoder on the HIP path vs the reference's golden vectors and the CPU oracle
(transformerDecoder.py:88-108, train.py:271-291), plus the attention kernel vs torch."""
import json
import math
import os

import pytest
import torch
import torch.nn.functional as F
from safetensors.torch import load_file

from golden_util import GOLDEN_DIR, make_captions, make_features, make_params
from oracle import decoders, shapes, train_step

pytestmark = pytest.mark.gpu


def _load(name):
    t = load_file(os.path.join(GOLDEN_DIR, name + ".safetensors"))
    with open(os.path.join(GOLDEN_DIR, name + ".json")) as f:
        return t, json.load(f)


def _rel(a, b):
    a, b = a.detach().float().cpu(), b.detach().float().cpu()
    return ((a - b).norm() / (b.norm() + 1e-12)).item()


def _decoder(cfg, params, dtype, dev, dropout=0.0):
    from imagecaptioningconvnext_amd.models.transformerDecoder import TransformerDecoder
    dec = TransformerDecoder(embed_dim=cfg["d"], decoder_dim=cfg["ff"], vocab_size=cfg["V"], maxLen=cfg["L"],
                             device=dev, wordMap=None, pretrained_embeddings_path=None, fine_tune_embeddings=True,
                             dropout=dropout, encoder_dim=cfg["E"], num_heads=cfg["H"], num_layers=cfg["layers"],
                             compute_dtype=dtype)
    sd = dict(dec.state_dict())
    sd.update(params)
    dec.load_state_dict(sd)
    return dec.to(dev)


def _ref_attention(q, k, v, causal, key_pad, emulate=False):
    """softmax(q k^T / 8 + masks) v; ``emulate``: the bf16 kernel's rounding points (P rounded before
    P V and dV = P^T dO, dS rounded before dQ = dS K and dK = dS^T Q; oracle/decoders.py)."""
    nm = decoders._Bf16 if emulate else decoders._Fp32
    B, H, Lq, dh = q.shape
    s = nm.grad(q @ k.transpose(-1, -2)) / math.sqrt(dh)
    Lk = k.shape[2]
    if causal:
        s = s.masked_fill(torch.triu(torch.ones(Lq, Lk, dtype=torch.bool), 1), float("-inf"))
    if key_pad is not None:
        s = s.masked_fill(key_pad.view(B, 1, 1, Lk), float("-inf"))
    return nm.value(torch.softmax(s, -1)) @ v


# bf16: against the kernel's own rounding points evaluated in fp64 (what remains is the outputs'
# bf16 rounding and the fp32 accumulation order: measured fwd 1.5-1.6e-3, dq / dk / dv 1.6-1.7e-3
# at every shape, round 6), and against plain fp32 attention with the round-5 gates


@pytest.mark.parametrize("dtype,tol", [(torch.float32, 1e-5), (torch.bfloat16, 2.5e-3)])
@pytest.mark.parametrize("Lq,Lk,causal", [(52, 52, True), (52, 49, False), (12, 12, True), (64, 64, True)])
def test_mha_kernel_fwd_bwd(hip_device, dtype, tol, Lq, Lk, causal):
    from imagecaptioningconvnext_amd import _abi
    from imagecaptioningconvnext_amd import kernels as K
    import ctypes
    torch.manual_seed(Lq + Lk)
    B, H, d = 3, 2, 128
    q = torch.randn(B, Lq, d)
    k = torch.randn(B, Lk, d)
    v = torch.randn(B, Lk, d)
    ids = torch.randint(1, 50, (B, Lk))
    if causal:
        ids[1, Lk - 3:] = 0  # padded tail keys
    pad = ids == 0
    emu = dtype == torch.bfloat16
    rdt = torch.float64 if emu else torch.float32
    qr, kr, vr = (t.to(dtype).to(rdt).view(B, -1, H, 64).transpose(1, 2).requires_grad_(True) for t in (q, k, v))
    ref = _ref_attention(qr, kr, vr, causal, pad if causal else None, emulate=emu)
    dout = torch.randn(ref.shape).to(dtype).to(rdt)
    ref.backward(dout)
    if emu:  # the plain fp32 attention on the same bf16 operands: the round-5 gates
        q3, k3, v3 = (t.detach().float().requires_grad_(True) for t in (qr, kr, vr))
        ref32 = _ref_attention(q3, k3, v3, causal, pad if causal else None)
        ref32.backward(dout.float())
    dev = hip_device
    qd, kd, vd = (t.to(dev, dtype).contiguous() for t in (q, k, v))
    o = torch.empty(B, Lq, d, device=dev, dtype=dtype)
    lse = torch.empty(B, H, Lq, device=dev)
    m = _abi.MhaDesc()
    m.dtype, m.B, m.H, m.Lq, m.Lk, m.dh, m.causal = K.dt(qd), B, H, Lq, Lk, 64, int(causal)
    m.pad_id = 0
    m.ldq = m.ldk = m.ldv = m.ldo = d
    m.q, m.k, m.v, m.o, m.lse = qd.data_ptr(), kd.data_ptr(), vd.data_ptr(), o.data_ptr(), lse.data_ptr()
    idsd = ids.to(dev)
    m.key_ids = idsd.data_ptr() if causal else None
    m.scale = 1 / 8.0
    _abi.call("imgcap_mha_fwd", ctypes.byref(m), K.stream())
    e_fwd = _rel(o.view(B, Lq, H, 64).transpose(1, 2), ref)
    print(f"\nmha {dtype} Lq={Lq} Lk={Lk} causal={causal}: fwd {e_fwd:.2e}")
    assert e_fwd < tol
    if emu:
        assert _rel(o.view(B, Lq, H, 64).transpose(1, 2), ref32) < 2e-2
    do = dout.transpose(1, 2).reshape(B, Lq, d).to(dev, dtype).contiguous()
    dq, dk, dv = torch.empty_like(qd), torch.empty_like(kd), torch.empty_like(vd)
    m.dout, m.lddo = do.data_ptr(), d
    m.dq, m.dk, m.dv = dq.data_ptr(), dk.data_ptr(), dv.data_ptr()
    m.lddq = m.lddk = m.lddv = d
    _abi.call("imgcap_mha_bwd", ctypes.byref(m), K.stream())
    for name, got, r in (("dq", dq, qr.grad), ("dk", dk, kr.grad), ("dv", dv, vr.grad)):
        e = _rel(got.view(B, -1, H, 64).transpose(1, 2), r)
        print(f"  {name} {e:.2e}")
        assert e < (tol if emu else tol * 2)
    if emu:
        for got, r in ((dq, q3.grad), (dk, k3.grad), (dv, v3.grad)):
            assert _rel(got.view(B, -1, H, 64).transpose(1, 2), r) < 4e-2


def test_transformer_h64_reference_api_and_grads(hip_device):
    t, meta = _load("transformer_tf_h64")
    cfg = meta["cfg"]
    p = make_params(shapes.transformer_decoder_shapes(cfg["E"], cfg["d"], cfg["ff"], cfg["V"], cfg["layers"]),
                    cfg["seed"])
    dec = _decoder(cfg, p, torch.float32, hip_device)
    caps = t["caps"].to(hip_device)
    preds, caps_out, dls = dec(teacherForcing=True, encoder_out=t["enc"].to(hip_device), encoded_captions=caps,
                               caption_lengths=t["caplens"].to(hip_device), tgt_key_padding_mask=caps == 0)
    assert dls == meta["decode_lengths"]
    assert _rel(preds, t["predictions"]) < 1e-4
    loss, _, _ = train_step.transformer_loss(preds, caps_out, dls)
    assert abs(loss.item() - t["loss"].item()) < 1e-5 * abs(t["loss"].item())
    for q in dec.parameters():
        q.grad = None
    loss.backward()
    for n, q in dec.named_parameters():
        g = t["grad." + n]
        if g.norm() < 1e-6:  # e.g. the key bias of attention: true gradient 0
            assert q.grad.norm().item() < 1e-5
            continue
        assert _rel(q.grad, g) < 2e-4, n


@pytest.mark.parametrize("dtype,tol", [(torch.float32, 2e-4), (torch.bfloat16, 3e-2)])
def test_transformer_h64_fused_step(hip_device, dtype, tol):
    t, meta = _load("transformer_tf_h64")
    cfg = meta["cfg"]
    p = make_params(shapes.transformer_decoder_shapes(cfg["E"], cfg["d"], cfg["ff"], cfg["V"], cfg["layers"]),
                    cfg["seed"])
    dec = _decoder(cfg, p, dtype, hip_device)
    eng = dec.engine()
    s = eng.forward(t["enc"].to(hip_device), t["caps"].to(hip_device), t["caplens"].to(hip_device), pad_id=0)
    m = s["metrics"].cpu()
    assert abs(m[0].item() - t["loss"].item()) < tol * abs(t["loss"].item())
    assert int(m[1].item()) == sum(meta["decode_lengths"])
    eng.backward(s)
    big = [n for n in eng.fp.params if t["grad." + n].norm() > 1e-6]
    for n in big:
        assert _rel(eng.fp.g(n), t["grad." + n]) < tol * (1 if dtype == torch.float32 else 3), n
    eng.fp.adam_step(1e-4, 5.0)
    if dtype == torch.float32:
        for n, q in dec.named_parameters():
            ok = t["grad." + n].abs() >= 1e-6
            torch.testing.assert_close(q.detach().cpu()[ok], t["post." + n][ok], rtol=1e-5, atol=2e-6)


@pytest.mark.parametrize("dtype,tol", [(torch.float32, 1e-4), (torch.bfloat16, 2e-2)])
def test_transformer_full_size_spot(hip_device, dtype, tol):
    t, meta = _load("transformer_full_spot")
    cfg = meta["cfg"]
    p = make_params(shapes.transformer_decoder_shapes(cfg["E"], cfg["d"], cfg["ff"], cfg["V"], cfg["layers"]),
                    cfg["seed"])
    dec = _decoder(cfg, p, dtype, hip_device)
    enc = make_features((cfg["B"], cfg["S"], cfg["S"], cfg["E"]), cfg["seed"] + 1).to(hip_device)
    caps, caplens = make_captions(cfg["B"], cfg["L"], cfg["caplens"], cfg["V"], cfg["seed"] + 2)
    with torch.no_grad():
        preds, cs, dls = dec(True, enc, caps.to(hip_device), caplens.to(hip_device), caps.to(hip_device) == 0)
    loss, scores, _ = train_step.transformer_loss(preds.cpu(), cs.cpu(), dls)
    assert abs(loss.item() - t["loss"].item()) < tol * abs(t["loss"].item())
    print(f"transformer full size {dtype}: loss rel {abs(loss.item() / t['loss'].item() - 1):.2e}, "
          f"logits rel {_rel(scores[t['rows'], t['cols']], t['values']):.2e}")
    assert _rel(scores[t["rows"], t["cols"]], t["values"]) < (1e-4 if dtype == torch.float32 else 1e-2)


def test_transformer_medium_vs_oracle_and_dropout(hip_device):
    E, d, ff, V, layers, B, L = 96, 128, 128, 200, 2, 4, 20
    p = make_params(shapes.transformer_decoder_shapes(E, d, ff, V, layers), 91)
    enc = make_features((B, 7, 7, E), 92)
    caps, caplens = make_captions(B, L, [20, 6, 13, 17], V, 93)
    pr = {k: v.clone().requires_grad_(True) for k, v in p.items()}
    preds, cs, dls = decoders.transformer_tf_forward(pr, enc, caps, caplens, caps == 0, 2, layers)
    loss, _, _ = train_step.transformer_loss(preds, cs, dls)
    loss.backward()
    cfg = dict(E=E, d=d, ff=ff, V=V, layers=layers, H=2, L=L)
    dec = _decoder(cfg, p, torch.float32, hip_device)
    eng = dec.engine()
    s = eng.forward(enc.to(hip_device), caps.to(hip_device), caplens.to(hip_device), pad_id=0)
    assert abs(s["metrics"][0].item() - loss.item()) < 1e-4 * loss.item()
    eng.backward(s)
    for n in eng.fp.params:
        g = pr[n].grad
        if g.norm() < 1e-6:
            continue
        assert _rel(eng.fp.g(n), g) < 2e-4, n
    dec.train()
    dec.dropout_p = 0.5
    eng.step_id = 0
    a = eng.forward(enc.to(hip_device), caps.to(hip_device), caplens.to(hip_device))["metrics"].clone()
    eng.step_id = 0
    b = eng.forward(enc.to(hip_device), caps.to(hip_device), caplens.to(hip_device))["metrics"].clone()
    assert torch.equal(a, b) and abs(a[0].item() - loss.item()) > 1e-3


@pytest.mark.parametrize("dtype,tol", [(torch.float32, 2e-4), (torch.bfloat16, 3e-2)])
def test_transformer_vocab_past_fused_ce_limit_vs_oracle(hip_device, dtype, tol):
    """V = 30000 is past imgcap_ce_fused's register row (24576 bf16 / 12288 fp32): the training
    CE falls back to ce_fwd -> loss_finalize -> ce_bwd (kernels.ce_train); loss and gradients
    against the oracle as for the fused path (train.py:266-276)."""
    from imagecaptioningconvnext_amd import kernels as K
    E, d, ff, V, layers, B, L = 64, 128, 128, 30000, 1, 3, 14
    p = make_params(shapes.transformer_decoder_shapes(E, d, ff, V, layers), 71)
    enc = make_features((B, 7, 7, E), 72)
    caps, caplens = make_captions(B, L, [14, 9, 5], V, 73)
    pr = {k: v.clone().requires_grad_(True) for k, v in p.items()}
    preds, cs, dls = decoders.transformer_tf_forward(pr, enc, caps, caplens, caps == 0, 2, layers)
    loss, _, _ = train_step.transformer_loss(preds, cs, dls)
    loss.backward()
    dec = _decoder(dict(E=E, d=d, ff=ff, V=V, layers=layers, H=2, L=L), p, dtype, hip_device)
    eng = dec.engine()
    s = eng.forward(enc.to(hip_device), caps.to(hip_device), caplens.to(hip_device), pad_id=0)
    assert not K.ce_fused_fits(s["logits"], s["dlogits"], V)
    assert abs(s["metrics"][0].item() - loss.item()) < tol * loss.item()
    assert int(s["metrics"][1].item()) == sum(dls)
    eng.backward(s)
    for n in eng.fp.params:
        g = pr[n].grad
        if g.norm() < 1e-6:
            continue
        assert _rel(eng.fp.g(n), g) < tol * (1 if dtype == torch.float32 else 3), n

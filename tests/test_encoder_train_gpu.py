"""Encoder fine-tuning (Encoder.fine_tune, encoder.py:29-34; train.py:113-114,278-290) on the
HIP path: the backward kernels against torch CPU autograd, and the trainable-suffix encoder /
full train step against the CPU oracle's autograd (oracle/convnext.py restates torchvision's
ConvNeXt; encoder parity vs torchvision itself is unpinned)."""
import pytest
import torch
import torch.nn.functional as F

from golden_util import make_captions, make_params
from oracle import convnext, decoders, shapes, train_step

pytestmark = pytest.mark.gpu


def _rel(a, b):
    a, b = a.detach().float().cpu(), b.detach().float().cpu()
    return ((a - b).norm() / (b.norm() + 1e-12)).item()


def _g(seed):
    return torch.Generator().manual_seed(seed)


# ---- kernels ------------------------------------------------------------------------------
@pytest.mark.parametrize("H,C", [(7, 96), (14, 64), (56, 96), (7, 1536), (7, 160)])  # W = 7: the unrolled wgrad
def test_dwconv7_backward(hip_device, H, C):
    from imagecaptioningconvnext_amd import kernels as K
    B = 2
    x = torch.randn(B, C, H, H, generator=_g(1), requires_grad=True)
    w = torch.randn(C, 1, 7, 7, generator=_g(2), requires_grad=True)
    b = torch.randn(C, generator=_g(3), requires_grad=True)
    dz = torch.randn(B, C, H, H, generator=_g(4))
    res = torch.randn(B, H, H, C, generator=_g(5))
    F.conv2d(x, w, b, padding=3, groups=C).backward(dz)
    dev = hip_device
    xn = x.detach().permute(0, 2, 3, 1).contiguous().to(dev)
    dzn = dz.permute(0, 2, 3, 1).contiguous().to(dev)
    w49 = w.detach().reshape(C, 49).t().contiguous().to(dev)
    dx = torch.empty_like(xn)
    K.dwconv7_bwd_data(dzn, w49, dx, res=res.to(dev))
    ref_dx = x.grad.permute(0, 2, 3, 1) + res
    assert _rel(dx, ref_dx) < 1e-5
    dw = torch.empty(C, 49, device=dev)
    db = torch.empty(C, device=dev)
    K.dwconv7_wgrad(dzn, xn, dw, db)
    assert _rel(dw, w.grad.reshape(C, 49)) < 1e-5
    assert _rel(db, b.grad) < 1e-5


def test_gemm_gelu_saves_preactivation_and_dgelu(hip_device):
    from imagecaptioningconvnext_amd import kernels as K
    M, N, Kd = 200, 136, 72
    a = torch.randn(M, Kd, generator=_g(1))
    w = torch.randn(N, Kd, generator=_g(2)) / Kd ** 0.5
    bias = torch.randn(N, generator=_g(3))
    dev = hip_device
    pre = torch.empty(M, N, device=dev)
    out = K.gemm(a.to(dev), w.to(dev), trans_b=True, bias=bias.to(dev), act=K.ACT_GELU, aux=pre)
    h = a @ w.t() + bias
    assert _rel(pre, h) < 1e-5
    assert _rel(out, F.gelu(h)) < 1e-5
    # d/dh GELU(h) through the DGELU epilogue: g (M x N) = (u @ v) * GELU'(h)
    u = torch.randn(M, 40, generator=_g(4))
    v = torch.randn(40, N, generator=_g(5))
    hh = h.clone().requires_grad_(True)
    F.gelu(hh).backward(u @ v)
    got = K.gemm(u.to(dev), v.to(dev), act=K.ACT_DGELU, aux=pre)
    assert _rel(got, hh.grad) < 1e-5


@pytest.mark.parametrize("cmajor", [False, True])
def test_ln_patchify2_backward(hip_device, cmajor):
    from imagecaptioningconvnext_amd import kernels as K
    B, H, C = 2, 14, 96
    x = torch.randn(B, H, H, C, generator=_g(1))
    lw = (1 + 0.1 * torch.randn(C, generator=_g(2))).requires_grad_(True)
    lb = (0.1 * torch.randn(C, generator=_g(3))).requires_grad_(True)
    xr = x.clone().requires_grad_(True)
    y = F.layer_norm(xr, (C,), lw, lb, 1e-6)                        # [B,H,W,C]
    y6 = y.view(B, H // 2, 2, H // 2, 2, C)                         # b, oh, kh, ow, kw, c
    if cmajor:
        patches = y6.permute(0, 1, 3, 5, 2, 4).reshape(-1, 4 * C)   # (c, kh, kw)
    else:
        patches = y6.permute(0, 1, 3, 2, 4, 5).reshape(-1, 4 * C)   # (kh, kw, c)
    dp = torch.randn(patches.shape, generator=_g(4))
    patches.backward(dp)
    dev = hip_device
    got_p = torch.empty(patches.shape, device=dev)
    K.ln_patchify2(x.to(dev), lw.detach().to(dev), lb.detach().to(dev), got_p, cmajor=cmajor)
    assert _rel(got_p, patches) < 1e-5
    dx = torch.empty(B, H, H, C, device=dev)
    dlw = torch.empty(C, device=dev)
    dlb = torch.empty(C, device=dev)
    K.ln_patchify2_bwd(x.to(dev), dp.to(dev), lw.detach().to(dev), dx, dlw, dlb, cmajor=cmajor)
    assert _rel(dx, xr.grad) < 1e-5
    assert _rel(dlw, lw.grad) < 1e-5 and _rel(dlb, lb.grad) < 1e-5


def test_adaptive_pool_backward(hip_device):
    from imagecaptioningconvnext_amd import kernels as K
    x = torch.randn(2, 64, 8, 8, generator=_g(1), requires_grad=True)
    dy = torch.randn(2, 64, 7, 7, generator=_g(2))
    F.adaptive_avg_pool2d(x, (7, 7)).backward(dy)
    dx = torch.empty(2, 8, 8, 64, device=hip_device)
    K.adaptive_pool_bwd(dy.permute(0, 2, 3, 1).contiguous().to(hip_device), 8, 8, dx)
    assert _rel(dx, x.grad.permute(0, 2, 3, 1)) < 1e-6


def test_layer_scale_grad(hip_device):
    from imagecaptioningconvnext_amd import kernels as K
    C, C4 = 96, 384
    G = torch.randn(C, C4, generator=_g(1))
    w2 = torch.randn(C, C4, generator=_g(2))
    b2, gam, cs = (torch.randn(C, generator=_g(i)) for i in (3, 4, 5))
    dev = hip_device
    dw2 = torch.empty(C, C4, device=dev)
    wg = torch.empty(C, C4, device=dev)
    dgam = torch.empty(C, device=dev)
    db2 = torch.empty(C, device=dev)
    K.layer_scale_grad(G.to(dev), w2.to(dev), b2.to(dev), gam.to(dev), cs.to(dev), dw2, wg, dgam, db2)
    assert _rel(dw2, gam[:, None] * G) < 1e-6
    assert _rel(wg, gam[:, None] * w2) < 1e-6
    assert _rel(dgam, (w2 * G).sum(1) + b2 * cs) < 1e-5
    assert _rel(db2, gam * cs) < 1e-6


# ---- encoder with a trainable suffix ------------------------------------------------------
def _oracle_grads(sd, img, R, start, sd_keep=None, variant="tiny"):
    children = {f"convnext.{i}." for i in range(start, 8)}
    p = {k: v.clone().requires_grad_(any(k.startswith(c) for c in children)) for k, v in sd.items()}
    out = convnext.encoder_forward(p, variant, img, sd_keep=sd_keep)
    (out * R).sum().backward()
    return out.detach(), {k: v.grad for k, v in p.items() if v.requires_grad}


@pytest.mark.parametrize("start", [7, 5, 2])
@pytest.mark.parametrize("dtype,tol", [(torch.float32, 2e-4), (torch.bfloat16, 4e-2)])
def test_encoder_finetune_grads_vs_oracle(hip_device, start, dtype, tol):
    from imagecaptioningconvnext_amd.models.encoder import Encoder
    sd = make_params(convnext.param_shapes("tiny"), 11)
    enc = Encoder(variant="tiny", compute_dtype=dtype)
    enc.load_state_dict(sd)
    enc = enc.to(hip_device).eval()
    enc.fine_tune(True, startingLayer=start)
    img = torch.randn(2, 3, 224, 224, generator=_g(12))
    R = torch.randn(2, 7, 7, 768, generator=_g(13))
    ref_out, ref_g = _oracle_grads(sd, img, R, start)
    out = enc(img.to(hip_device))
    assert out.requires_grad
    assert _rel(out, ref_out) < tol
    (out.float() * R.to(hip_device)).sum().backward()
    got = dict(enc.named_parameters())
    assert set(ref_g) == {n for n, p in got.items() if p.requires_grad}
    for n, g in ref_g.items():
        assert _rel(got[n].grad, g) < tol, n


@pytest.mark.parametrize("variant,start", [("base", 7), ("base", 5), ("large", 7)])
@pytest.mark.parametrize("dtype,tol", [(torch.float32, 2e-4), (torch.bfloat16, 4e-2)])
def test_encoder_finetune_grads_base_large(hip_device, variant, start, dtype, tol):
    """Base (C4 / the reference's encoder.py:18) and Large (C5) with trainable suffixes: output
    and every trainable gradient vs the oracle's autograd."""
    from imagecaptioningconvnext_amd.models.encoder import Encoder
    from oracle.convnext import VARIANTS
    sd = make_params(convnext.param_shapes(variant), 17)
    enc = Encoder(variant=variant, compute_dtype=dtype)
    enc.load_state_dict(sd)
    enc = enc.to(hip_device).eval()
    enc.fine_tune(True, startingLayer=start)
    img = torch.randn(2, 3, 224, 224, generator=_g(18))
    R = torch.randn(2, 7, 7, VARIANTS[variant][0][3], generator=_g(19))
    ref_out, ref_g = _oracle_grads(sd, img, R, start, variant=variant)
    out = enc(img.to(hip_device))
    assert _rel(out, ref_out) < tol
    (out.float() * R.to(hip_device)).sum().backward()
    got = dict(enc.named_parameters())
    assert set(ref_g) == {n for n, p in got.items() if p.requires_grad}
    errs = {n: _rel(got[n].grad, g) for n, g in ref_g.items()}
    worst = max(errs, key=errs.get)
    print(f"{variant} start {start} {dtype}: worst grad {worst} {errs[worst]:.2e}")
    assert errs[worst] < tol


def test_encoder_finetune_train_mode_stochastic_depth(hip_device):
    """train(): the per-sample drop-path scales enter the backward exactly as the forward."""
    from imagecaptioningconvnext_amd.models.encoder import Encoder
    sd = make_params(convnext.param_shapes("tiny"), 21)
    enc = Encoder(variant="tiny", compute_dtype=torch.float32)
    enc.load_state_dict(sd)
    enc = enc.to(hip_device).train()
    enc.fine_tune(True, startingLayer=5)
    img = torch.randn(4, 3, 224, 224, generator=_g(22))
    R = torch.randn(4, 7, 7, 768, generator=_g(23))
    enc.sd_seed = 9
    scales = enc._sd_scales(4, hip_device).cpu()
    enc.sd_seed = 9
    out = enc(img.to(hip_device))
    (out * R.to(hip_device)).sum().backward()
    ref_out, ref_g = _oracle_grads(sd, img, R, 5, sd_keep=list(scales))
    assert _rel(out, ref_out) < 2e-4
    got = dict(enc.named_parameters())
    for n, g in ref_g.items():
        assert _rel(got[n].grad, g) < 2e-4, n


# ---- the fused train step with a fine-tuned encoder ---------------------------------------
@pytest.mark.parametrize("decoder", ["lstm", "transformer"])
def test_trainer_finetune_step_vs_oracle(hip_device, decoder):
    """One TeacherForcedTrainer step with fine_tune(True, 7): loss, the decoder's and the
    encoder's post-Adam parameters vs the oracle (autograd through encoder + decoder, clip,
    two Adams with their own learning rates: train.py:110,114,278-291)."""
    from imagecaptioningconvnext_amd.models.decoder import DecoderWithAttention
    from imagecaptioningconvnext_amd.models.encoder import Encoder
    from imagecaptioningconvnext_amd.models.transformerDecoder import TransformerDecoder
    from imagecaptioningconvnext_amd.train_step import TeacherForcedTrainer
    dev = hip_device
    E, V, L, B = 768, 120, 16, 3
    esd = make_params(convnext.param_shapes("tiny"), 31)
    enc = Encoder(variant="tiny", compute_dtype=torch.float32)
    enc.load_state_dict(esd)
    for m in enc.modules():  # eval-equivalent drop path so the oracle needs no masks
        if hasattr(m, "sd_prob"):
            m.sd_prob = 0.0
    enc = enc.to(dev)
    enc.fine_tune(True, startingLayer=7)
    if decoder == "lstm":
        dsh = shapes.lstm_decoder_shapes(E, 32, 32, 32, V)
        dp = make_params(dsh, 32)
        dec = DecoderWithAttention(attention_dim=32, embed_dim=32, decoder_dim=32, vocab_size=V, device=dev,
                                   encoder_dim=E, dropout=0.0, compute_dtype=torch.float32)
    else:
        dsh = shapes.transformer_decoder_shapes(E, 128, 64, V, 2)
        dp = make_params(dsh, 32)
        dec = TransformerDecoder(embed_dim=128, decoder_dim=64, vocab_size=V, maxLen=L, device=dev, wordMap=None,
                                 pretrained_embeddings_path=None, fine_tune_embeddings=True, dropout=0.0,
                                 encoder_dim=E, num_heads=2, num_layers=2, compute_dtype=torch.float32)
        dp["pos_encoding.pe"] = dec.pos_encoding.pe.clone()
    dec.load_state_dict(dp)
    dec = dec.to(dev)
    caps, caplens = make_captions(B, L, [L, 11, 7], V, 33)
    img = torch.randn(B, 3, 224, 224, generator=_g(34))
    tr = TeacherForcedTrainer(enc, dec, lstm=decoder == "lstm", decoder_lr=1e-3, encoder_lr=2e-3)
    tr.step(img.to(dev), caps.to(dev), caplens.to(dev))
    got_loss = tr.drain_metrics()[0][0]
    # oracle
    ep = {k: v.clone().requires_grad_(k.startswith("convnext.7.")) for k, v in esd.items()}
    dq = {k: v.clone().requires_grad_(k != "pos_encoding.pe") for k, v in dp.items()}
    feats = convnext.encoder_forward(ep, "tiny", img)
    if decoder == "lstm":
        preds, cs, dls, al, _ = decoders.lstm_tf_forward(dq, feats, caps, caplens)
        loss, _, _ = train_step.lstm_loss(preds, cs, dls, al)
    else:
        pad = caps == 0
        preds, cs, dls = decoders.transformer_tf_forward(dq, feats, caps, caplens, pad, 2, 2)
        loss, _, _ = train_step.transformer_loss(preds, cs, dls)
    loss.backward()
    assert abs(got_loss - loss.item()) < 2e-4 * abs(loss.item())
    for ps, lr, named in ((ep, 2e-3, dict(enc.named_parameters())), (dq, 1e-3, dict(dec.named_parameters()))):
        grads = {k: v.grad for k, v in ps.items() if v.requires_grad and v.grad is not None}
        new = train_step.adam_step({k: ps[k].detach() for k in grads}, train_step.clip_gradient(grads, 5.0), {},
                                   lr, 1)
        for k, v in new.items():
            # entries whose true gradient is ~0 (e.g. the key bias of softmax attention) take a
            # noise-driven first Adam step (g / (|g| + eps)); compare the others
            live = grads[k].abs() > 1e-6
            if not live.any():
                continue
            moved = (v - ps[k].detach())[live].abs().max().item()
            err = (named[k].detach().cpu() - v)[live].abs().max().item()
            # Adam's first step moves each entry by ~lr * sign(g): compare the update, not the value
            assert err <= 0.05 * max(moved, lr) + 1e-6, (k, err, moved)


# ---- C5: ConvNeXt-Large, MX-FP8 frozen prefix, stage 4 fine-tuned ------------------------
def test_c5_large_fp8_finetune_vs_emulating_oracle(hip_device):
    """BASELINE configs[4] (C5) at B = 2: Large encoder with frozen_fp8 (children 1-6 of the
    trunk with MX-FP8 Linears where C >= 384), fine_tune(True, 7) (stage 4 trains in bf16),
    a Transformer decoder on top.  Features, loss and the stage-4 gradients vs the oracle that
    emulates the same numerics (MX quantise-dequantise in the frozen stages, bf16 rounding
    elsewhere), then one fused TeacherForcedTrainer step: its loss vs the same oracle."""
    from imagecaptioningconvnext_amd.models.encoder import Encoder
    from imagecaptioningconvnext_amd.models.transformerDecoder import TransformerDecoder
    from imagecaptioningconvnext_amd.train_step import TeacherForcedTrainer
    dev = hip_device
    E, V, L, B, d = 1536, 150, 14, 2, 128  # head dim 64 (the HIP attention kernel's)
    esd = make_params(convnext.param_shapes("large"), 61)
    enc = Encoder(variant="large", frozen_fp8=True)
    enc.load_state_dict(esd)
    for m in enc.modules():  # eval-equivalent drop path so the oracle needs no masks
        if hasattr(m, "sd_prob"):
            m.sd_prob = 0.0
    enc = enc.to(dev)
    enc.fine_tune(True, startingLayer=7)
    dp = make_params(shapes.transformer_decoder_shapes(E, d, d, V, 2), 62)
    dec = TransformerDecoder(embed_dim=d, decoder_dim=d, vocab_size=V, maxLen=L, device=dev, wordMap=None,
                             pretrained_embeddings_path=None, fine_tune_embeddings=True, dropout=0.0,
                             encoder_dim=E, num_heads=2, num_layers=2, compute_dtype=torch.float32)
    dp["pos_encoding.pe"] = dec.pos_encoding.pe.clone()
    dec.load_state_dict(dp)
    dec = dec.to(dev)
    caps, caplens = make_captions(B, L, [L, 9], V, 63)
    img = torch.randn(B, 3, 224, 224, generator=_g(64))
    # oracle: MX prefix (children 1, 3, 5 hold the qualifying stages), bf16 stage 4, fp32 decoder
    ep = {k: v.clone().requires_grad_(k.startswith("convnext.7.")) for k, v in esd.items()}
    feats = convnext.encoder_forward(ep, "large", img, numerics="mx", mx_children=(1, 3, 5))
    dq = {k: v.clone() for k, v in dp.items()}
    pad = caps == 0
    preds, cs, dls = decoders.transformer_tf_forward(dq, feats, caps, caplens, pad, 2, 2)
    loss, _, _ = train_step.transformer_loss(preds, cs, dls)
    loss.backward()
    # HIP: differentiable encoder (EncoderEngine) + the decoder module
    out = enc(img.to(dev))
    f_err = _rel(out, feats)
    p_out, _, _ = dec(True, out.float(), caps.to(dev), caplens.to(dev), pad.to(dev))
    g_loss, _, _ = train_step.transformer_loss(p_out, caps.to(dev), dls)
    g_loss.backward()
    named = dict(enc.named_parameters())
    g_errs = {k: _rel(named[k].grad, v.grad) for k, v in ep.items() if v.requires_grad}
    worst = max(g_errs, key=g_errs.get)
    print(f"C5: features rel {f_err:.2e}, loss rel {abs(g_loss.item() / loss.item() - 1):.2e}, "
          f"worst stage-4 grad {worst} {g_errs[worst]:.2e}")
    # measured (MI355X, round 2): features 1.3e-2, loss 6e-7, worst stage-4 gradient 3.5e-3
    assert f_err < 2.5e-2
    assert abs(g_loss.item() - loss.item()) < 1e-4 * abs(loss.item())
    assert g_errs[worst] < 1e-2
    # the fused step (MX prefix, bf16 stage-4 forward/backward, encoder Adam at encoderLr)
    for p_ in list(enc.parameters()) + list(dec.parameters()):
        p_.grad = None
    tr = TeacherForcedTrainer(enc, dec, lstm=False, decoder_lr=1e-4, encoder_lr=1e-4)
    assert tr.enc_eng is not None
    tr.step(img.to(dev), caps.to(dev), caplens.to(dev))
    (t_loss, t_tok, _), = tr.drain_metrics()
    print(f"C5 fused step: loss rel {abs(t_loss / loss.item() - 1):.2e}")
    assert t_tok == sum(dls)
    assert abs(t_loss - loss.item()) < 1e-4 * abs(loss.item())

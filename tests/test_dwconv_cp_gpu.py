"""Depthwise 7x7 for the narrow late stages (the channel-pair kernel of convnext.hip: W = 7 and 14,
C <= 1024 with the fused LayerNorm, any C % 128 == 0 without; bf16; one or two output rows per
block, IMGCAP_DW_CP_R) against torch fp32 conv2d(groups=C) on the bf16-rounded input and against
the channel-tiled kernel (IMGCAP_DW_CP=0), plain and in the backward data-gradient form (flipped
taps + residual, odd H with two rows per block); C = 768 runs 2-wave channel-group blocks, and imgcap_dwconv7_ln
(row kernel) against torch LayerNorm of the same conv."""
import os

import pytest
import torch
import torch.nn.functional as F

from imagecaptioningconvnext_amd import kernels as K

pytestmark = pytest.mark.gpu


def _rel(a, b):
    return float((a.float() - b.float()).norm() / b.float().norm().clamp_min(1e-30))


def _ref(x, w49, bias, flip=False):
    B, H, W, C = x.shape
    wk = w49.t().reshape(C, 1, 7, 7)
    if flip:
        wk = wk.flip(2, 3)
    y = F.conv2d(x.permute(0, 3, 1, 2).float(), wk.float(), None if bias is None else bias.float(), padding=3, groups=C)
    return y.permute(0, 2, 3, 1)


@pytest.mark.parametrize("rows", ["1", "2"])
@pytest.mark.parametrize("B,H,C", [(3, 14, 384), (2, 14, 512), (2, 7, 768), (3, 7, 1024), (1, 14, 1024), (2, 14, 768),
                                   (2, 7, 1536)])
def test_dwconv_cp_matches_torch(hip_device, monkeypatch, rows, B, H, C):
    monkeypatch.setenv("IMGCAP_DW_CP_R", rows)
    g = torch.Generator(device="cpu").manual_seed(B * H + C)
    x = torch.randn(B, H, H, C, generator=g).bfloat16()
    w49 = torch.randn(49, C, generator=g) * 0.1
    bias, lw, lb = (torch.randn(C, generator=g) for _ in range(3))
    d = lambda t: t.to(hip_device)  # noqa: E731
    ref = _ref(x, w49, bias)
    y = torch.empty(B, H, H, C, device=hip_device, dtype=torch.bfloat16)
    K.dwconv7(d(x), d(w49), d(bias), y)
    assert _rel(y.cpu(), ref) < 1e-2
    # LayerNorm fused: vs torch LN of the fp32 conv output
    z = torch.empty_like(y)
    K.dwconv7_ln(d(x), d(w49), d(bias), d(lw), d(lb), z)
    zr = F.layer_norm(ref, (C,), lw, lb, 1e-6)
    assert _rel(z.cpu(), zr) < 1e-2
    # the channel-tiled kernels on the same inputs (bf16 depthwise output, then LN)
    os.environ["IMGCAP_DW_CP"] = "0"
    try:
        y0 = torch.empty_like(y)
        K.dwconv7(d(x), d(w49), d(bias), y0)
    finally:
        del os.environ["IMGCAP_DW_CP"]
    assert _rel(y.cpu(), y0.cpu()) < 1e-2


@pytest.mark.parametrize("rows", ["1", "2"])
@pytest.mark.parametrize("H,C", [(14, 384), (7, 768), (7, 1536)])
def test_dwconv_cp_backward_data_form(hip_device, monkeypatch, rows, H, C):
    """Flipped taps + residual (imgcap_dwconv7_bwd_data's use of the forward kernel)."""
    monkeypatch.setenv("IMGCAP_DW_CP_R", rows)
    B = 2
    g = torch.Generator(device="cpu").manual_seed(7)
    dz = torch.randn(B, H, H, C, generator=g).bfloat16()
    res = torch.randn(B, H, H, C, generator=g).bfloat16()
    w49 = torch.randn(49, C, generator=g) * 0.1
    d = lambda t: t.to(hip_device)  # noqa: E731
    out = torch.empty(B, H, H, C, device=hip_device, dtype=torch.bfloat16)
    K.dwconv7_bwd_data(d(dz), d(w49), out, res=d(res))
    ref = _ref(dz, w49, None, flip=True) + res.float()
    assert _rel(out.cpu(), ref) < 1e-2



"""Wide fused CNBlock MLP (csrc/cnblock_mlp_wide.hip: C = 384 / 512, an opt-in beside
the LayerNorm + two-GEMM path) vs torch fp32 on the bf16-rounded operands -- the same reference and gate as
the narrow kernel's tests (test_kernels_gpu.py::test_cnblock_mlp_fused: x + gamma*sd*(GELU(LN(y)
W1^T + b1) W2^T + b2), hidden rounded to bf16, relative error of the update < 2e-2).  Row counts
cover both launch forms: split hidden (< 128 64-row tiles: two blocks per tile, the second adds the
first one's partial) and whole hidden per block, with ragged last tiles."""
import math

import pytest
import torch
import torch.nn.functional as F

from imagecaptioningconvnext_amd import kernels as K

pytestmark = pytest.mark.gpu


def _rel(a, b):
    return float((a.float() - b.float()).norm() / b.float().norm().clamp_min(1e-30))


def _case(C, M, seed, with_ln=True, with_sd=True, rps=196):
    g = torch.Generator(device="cpu").manual_seed(seed)
    y = (torch.randn(M, C, generator=g) * 2 + 0.5).bfloat16()
    x = torch.randn(M, C, generator=g).bfloat16()
    w1 = (torch.randn(4 * C, C, generator=g) / math.sqrt(C)).bfloat16()
    w2 = (torch.randn(C, 4 * C, generator=g) / math.sqrt(4 * C)).bfloat16()
    b1, b2, gamma, lw, lb = (torch.randn(n, generator=g) for n in (4 * C, C, C, C, C))
    sd = (torch.rand((M + rps - 1) // rps, generator=g) > 0.3).float() / 0.7 if with_sd else None
    z = F.layer_norm(y.float(), (C,), lw, lb, 1e-6).bfloat16().float() if with_ln else y.float()
    hid = F.gelu(z @ w1.float().t() + b1).bfloat16().float()
    delta = (hid @ w2.float().t() + b2) * gamma
    if with_sd:
        delta = delta * sd.repeat_interleave(rps)[:M].view(M, 1)
    return dict(y=y, x=x, w1=w1, w2=w2, b1=b1, b2=b2, gamma=gamma, lw=lw if with_ln else None,
                lb=lb if with_ln else None, sd=sd, rps=rps, delta=delta)


def _run(c, dev):
    d = lambda t: None if t is None else t.to(dev)  # noqa: E731
    M, C = c["x"].shape
    img = K.cnblock_mlp_wide_pack(d(c["w1"]), d(c["w2"]))
    scratch = K.cnblock_mlp_wide_scratch(M, C, dev)
    xd = d(c["x"])
    K.cnblock_mlp_wide(d(c["y"]), img, d(c["b1"]), d(c["b2"]), d(c["gamma"]), xd, scratch, sd=d(c["sd"]),
                       rows_per_sample=c["rps"], ln_w=d(c["lw"]), ln_b=d(c["lb"]))
    return xd, scratch


@pytest.mark.parametrize("C", [384, 512])
@pytest.mark.parametrize("M", [200, 6272, 8257 + 64 * 120])
def test_wide_mlp_matches_torch(hip_device, C, M):
    c = _case(C, M, C * 7 + M)
    xd, scratch = _run(c, hip_device)
    got = xd.cpu().float() - c["x"].float()
    assert _rel(got, c["delta"]) < 2e-2
    if scratch[1] is not None:  # the split launch leaves its ticket / flag words zero
        assert int(scratch[1].abs().sum()) == 0


@pytest.mark.parametrize("C", [384, 512])
def test_wide_mlp_without_layernorm_and_drop_path(hip_device, C):
    c = _case(C, 1000, C, with_ln=False, with_sd=False)
    xd, _ = _run(c, hip_device)
    assert _rel(xd.cpu().float() - c["x"].float(), c["delta"]) < 2e-2


@pytest.mark.parametrize("M", [1568, 12544])
def test_wide_mlp_repeatable_and_matches_two_gemm_path(hip_device, M):
    """Bitwise repeatable over calls (the split form adds the two partials in a fixed order) and
    within bf16 rounding of the LayerNorm + two-GEMM path it replaces."""
    C = 384
    c = _case(C, M, M)
    dev = hip_device
    d = lambda t: None if t is None else t.to(dev)  # noqa: E731
    img = K.cnblock_mlp_wide_pack(d(c["w1"]), d(c["w2"]))
    scratch = K.cnblock_mlp_wide_scratch(M, C, dev)
    outs = []
    for _ in range(3):
        xd = d(c["x"])
        K.cnblock_mlp_wide(d(c["y"]), img, d(c["b1"]), d(c["b2"]), d(c["gamma"]), xd, scratch, sd=d(c["sd"]),
                           rows_per_sample=c["rps"], ln_w=d(c["lw"]), ln_b=d(c["lb"]))
        outs.append(xd)
    assert all(torch.equal(outs[0], o) for o in outs[1:])
    # the two-GEMM path (LayerNorm kernel, GEMM + GELU epilogue, GEMM + scale + residual epilogue)
    zn = torch.empty(M, C, device=dev, dtype=torch.bfloat16)
    hid = torch.empty(M, 4 * C, device=dev, dtype=torch.bfloat16)
    x2 = d(c["x"])
    K.add_layernorm(d(c["y"]), None, d(c["lw"]), d(c["lb"]), 1e-6, y=zn)
    K.gemm(zn, d(c["w1"]), trans_b=True, bias=d(c["b1"]), act=K.ACT_GELU, out=hid)
    K.gemm(hid, d(c["w2"]), trans_b=True, bias=d(c["b2"]), colscale=d(c["gamma"]), rowscale=d(c["sd"]),
           rows_per_scale=c["rps"], res=x2, out=x2)
    x0 = c["x"].float()
    assert _rel(outs[0].cpu().float() - x0, x2.cpu().float() - x0) < 1e-2

"""Weight-stationary short-K GEMM (csrc/gemm_ws.h, imgcap_gemm_set_ws): K = 384 / 512, A and B
k-major, bf16 C, against a PyTorch fp32 product of the same bf16 operands and against the LDS-staged
kernels on the same call (imgcap_gemm_set_ws(0)), for both block forms (8-wave / 4-wave), the
epilogue forms it serves (bias, GELU, ReLU, alpha, column scale, dropout -- the mask compared with
the LDS kernel's, the same counter-based draw), ragged M (a last chunk of < 32 rows), N not a
multiple of the 32-column wave slice, pitches wider than the rows, and the encoder / decoder
shapes of C3 (12544 x 1536 x 384, 3328 x 512 x 512, ...).  Every test restores the policy it
found."""
import pytest
import torch

pytestmark = pytest.mark.gpu

bf = torch.bfloat16


def _gelu(x):
    return 0.5 * x * (1.0 + torch.erf(x * 0.7071067811865476))


def _ops(dev, M, N, K, seed, pad=0):
    g = torch.Generator().manual_seed(seed)
    a = torch.randn(M, K + pad, generator=g).to(bf)
    b = (torch.randn(N, K + pad, generator=g) / K ** 0.5).to(bf)
    return a.to(dev)[:, :K], b.to(dev)[:, :K], a[:, :K].float() @ b[:, :K].float().t()


SHAPES = [(12544, 1536, 384), (3328, 512, 512), (3328, 1536, 512), (1000, 776, 384), (333, 200, 512),
          (64, 96, 384), (50176, 192, 384)]


@pytest.mark.parametrize("M,N,K", SHAPES)
@pytest.mark.parametrize("mode", [1, 2])
def test_ws_plain_and_bias_gelu(hip_device, M, N, K, mode):
    from imagecaptioningconvnext_amd import kernels as K_
    dev = hip_device
    a, b, prod = _ops(dev, M, N, K, M + N + K, pad=8 if M == 1000 else 0)
    bias = torch.randn(N, generator=torch.Generator().manual_seed(1))
    with K_.gemm_ws_mode(mode):
        ep = K_.Epilogue()
        ep.c_dtype, ep.alpha = K_.BF16, 1.0
        kind, _ = K_.gemm_plan(K_.BF16, 1, 1, M, N, K, a.stride(0), b.stride(0), ep=ep)
        assert kind == (K_.GEMM_WS if mode == 1 else K_.GEMM_WS4), kind
        out = K_.gemm(a, b, trans_b=True)
        outg = K_.gemm(a, b, trans_b=True, bias=bias.to(dev), act=K_.ACT_GELU)
        torch.cuda.synchronize()
    err = ((out.float().cpu() - prod).abs().max() / prod.abs().max()).item()
    assert err < 8e-3, err
    ref = _gelu(prod + bias)
    errg = ((outg.float().cpu() - ref).abs().max() / ref.abs().max()).item()
    assert errg < 8e-3, errg


@pytest.mark.parametrize("mode", [1, 2])
@pytest.mark.parametrize("form", ["relu_alpha", "colscale", "dropout"])
def test_ws_epilogues_match_lds_kernels(hip_device, mode, form):
    from imagecaptioningconvnext_amd import kernels as K_
    dev = hip_device
    M, N, K = 1500, 776, 512
    a, b, prod = _ops(dev, M, N, K, 7)
    g = torch.Generator().manual_seed(3)
    bias = torch.randn(N, generator=g).to(dev)
    cs = (torch.rand(N, generator=g) + 0.5).to(dev)
    if form == "relu_alpha":
        kw = dict(bias=bias, act=K_.ACT_RELU, alpha=0.75)
    elif form == "colscale":
        kw = dict(bias=bias, act=K_.ACT_GELU, colscale=cs)
    else:
        kw = dict(bias=bias, drop_p=0.3, seed=1234, drop_stream=5)
    outs = []
    for m in (mode, 0):
        with K_.gemm_ws_mode(m), K_.gemm_pt_mode(0):
            outs.append(K_.gemm(a, b, trans_b=True, **kw).float().cpu())
    torch.cuda.synchronize()
    got, base = outs
    diff = (got - base).abs()
    assert bool((diff <= 1e-2 * base.abs() + 1e-2).all()), float(diff.max())
    if form == "dropout":
        assert torch.equal(got == 0, base == 0)
    if form == "relu_alpha":
        ref = torch.relu(0.75 * prod + bias.cpu())
        assert ((got - ref).abs().max() / ref.abs().max()).item() < 8e-3


def test_ws_bitwise_repeatable_and_default_plan(hip_device):
    from imagecaptioningconvnext_amd import kernels as K_
    dev = hip_device
    assert K_.gemm_get_ws() == -1
    a, b, _ = _ops(dev, 12544, 1536, 384, 5)
    with K_.gemm_ws_mode(1):
        o1 = K_.gemm(a, b, trans_b=True, act=K_.ACT_GELU)
        o2 = K_.gemm(a, b, trans_b=True, act=K_.ACT_GELU)
        torch.cuda.synchronize()
    assert torch.equal(o1, o2)

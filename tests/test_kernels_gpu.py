"""HIP kernels vs plain PyTorch fp32 references of the same op (GPU only)."""
import math

import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu

from imagecaptioningconvnext_amd import kernels as K  # noqa: E402


def _padded(x, dev, dtype):
    """Copy x [r, c] into storage whose leading dim is a multiple of 8 (16-byte rows)."""
    r, c = x.shape
    buf = torch.zeros(r, (c + 7) // 8 * 8, dtype=dtype, device=dev)
    buf[:, :c] = x.to(dtype)
    return buf[:, :c]


def _rel(a, b):
    return ((a.float() - b.float()).norm() / (b.float().norm() + 1e-12)).item()


@pytest.mark.parametrize("dtype,tol", [(torch.float32, 2e-6), (torch.bfloat16, 1e-2)])
@pytest.mark.parametrize("ta,tb", [(False, True), (False, False), (True, False), (True, True)])
@pytest.mark.parametrize("M,N,Kd", [(37, 50, 72), (32, 3328, 512), (64, 200, 136), (300, 260, 1000), (1030, 520, 96),
                                     (5, 50, 20), (17, 33, 40), (64, 100, 1000), (1, 16, 8), (130, 9490, 40),
                                     (1500, 1800, 192), (4100, 520, 256), (1500, 1800, 200), (2100, 1100, 584),
                                     (1600, 2000, 1001), (300, 520, 9490)])
def test_gemm_layouts(hip_device, dtype, tol, ta, tb, M, N, Kd):
    g = torch.Generator(device="cpu").manual_seed(M * 7 + N)
    a = torch.randn(M, Kd, generator=g)
    b = torch.randn(Kd, N, generator=g)
    ref = a @ b
    ad = _padded(a.t() if ta else a, hip_device, dtype)
    bd = _padded(b.t() if tb else b, hip_device, dtype)
    out = K.gemm(ad, bd, trans_a=ta, trans_b=tb, out_dtype=torch.float32)
    if dtype == torch.bfloat16:
        ref = a.bfloat16().float() @ b.bfloat16().float()
    assert _rel(out.cpu(), ref) < tol
    if dtype == torch.bfloat16:  # the same product on the 256x256 tile (forced), the small-grid
        for pol in (1, 2, 3, 0, 6, 8):  # 64x64 LDS-DMA tile and the register-staged one (the 128x64 tile,
            # policy 7, is in the diagnostic build only: tests/test_gemm_pt_gpu.py checks the refusal)
            K.gemm_set_policy(pol)
            try:
                out = K.gemm(ad, bd, trans_a=ta, trans_b=tb, out_dtype=torch.float32)
            finally:
                K.gemm_set_policy(-1)
            assert _rel(out.cpu(), ref) < tol, pol


@pytest.mark.parametrize("dtype,tol", [(torch.float32, 2e-6), (torch.bfloat16, 1e-2)])
@pytest.mark.parametrize("split", [-1, 3, 7])
@pytest.mark.parametrize("M,N,Kd,ta,tb", [(512, 1536, 3328, True, False), (300, 260, 1000, True, False),
                                          (130, 200, 4100, False, True), (96, 520, 777, True, True)])
def test_gemm_split_k_accumulate(hip_device, dtype, tol, split, M, N, Kd, ta, tb):
    """Weight-gradient form: out = alpha*A.B + beta*out with K sliced over the grid."""
    g = torch.Generator(device="cpu").manual_seed(M + N + Kd)
    a = torch.randn(M, Kd, generator=g)
    b = torch.randn(Kd, N, generator=g)
    c0 = torch.randn(M, N, generator=g)
    ref = c0 + (a.to(dtype).float() @ b.to(dtype).float()) * 0.5
    ad = _padded(a.t() if ta else a, hip_device, dtype)
    bd = _padded(b.t() if tb else b, hip_device, dtype)
    out = _padded(c0, hip_device, torch.float32)
    K.gemm(ad, bd, trans_a=ta, trans_b=tb, out=out, alpha=0.5, beta=1.0, split_k=split)
    assert _rel(out.cpu(), ref) < tol
    o2 = K.gemm(ad, bd, trans_a=ta, trans_b=tb, out=out.clone(), split_k=split)
    assert _rel(o2.cpu(), (ref - c0) * 2) < tol
    with pytest.raises(RuntimeError):
        K.gemm(ad, bd, trans_a=ta, trans_b=tb, out=out, bias=torch.zeros(N, device=hip_device), split_k=split)


@pytest.mark.parametrize("dtype,tol", [(torch.bfloat16, 1e-2)])
def test_gemm_auto_split_with_epilogue(hip_device, dtype, tol):
    """Small grid + long K takes the split-K path unasked; the reduce applies the whole epilogue
    (bias, ReLU, dropout, bf16 out) -- the decoder's fc dX shape (K = vocab)."""
    g = torch.Generator(device="cpu").manual_seed(9)
    M, N, Kd = 400, 256, 9490
    a = torch.randn(M, Kd, generator=g)
    w = torch.randn(Kd, N, generator=g) / math.sqrt(Kd)
    bias = torch.randn(N, generator=g)
    ad, wd = _padded(a, hip_device, dtype), _padded(w, hip_device, dtype)
    o = K.gemm(ad, wd, bias=bias.to(hip_device), act=K.ACT_RELU, out_dtype=torch.float32)
    ref = torch.relu(a.to(dtype).float() @ w.to(dtype).float() + bias)
    assert _rel(o.cpu(), ref) < tol
    d1 = K.gemm(ad, wd, drop_p=0.5, seed=3, drop_stream=2, out_dtype=torch.bfloat16)
    d2 = K.gemm(ad, wd, drop_p=0.5, seed=3, drop_stream=2, out_dtype=torch.bfloat16)
    assert torch.equal(d1, d2)
    base = a.to(dtype).float() @ w.to(dtype).float()
    kept = d1.cpu().float() != 0
    assert 0.4 < kept.float().mean().item() < 0.6
    assert _rel(d1.cpu().float()[kept], 2 * base[kept]) < tol


@pytest.mark.parametrize("dtype,tol", [(torch.float32, 1e-5), (torch.bfloat16, 1.5e-2)])
@pytest.mark.parametrize("policy", [-1, 1, 2, 8])
def test_gemm_epilogues(hip_device, dtype, tol, policy):
    K.gemm_set_policy(policy)
    try:
        _gemm_epilogues(hip_device, dtype, tol)
    finally:
        K.gemm_set_policy(-1)


def _gemm_epilogues(hip_device, dtype, tol):
    torch.manual_seed(0)
    M, N, Kd = 196, 96, 384
    x = torch.randn(M, Kd)
    w = torch.randn(N, Kd) / math.sqrt(Kd)
    bias = torch.randn(N)
    res = torch.randn(M, N)
    gamma = torch.randn(N)
    rs = torch.rand(4) + 0.5
    dev = lambda t, d=dtype: t.to(hip_device, d)  # noqa: E731
    # bias + GELU
    out = K.gemm(dev(x), dev(w), trans_b=True, bias=dev(bias, torch.float32), act=K.ACT_GELU)
    assert _rel(out.cpu(), F.gelu(x @ w.t() + bias)) < tol
    # layer-scale * rowscale + residual (ConvNeXt block tail), output written in place of res
    r = dev(res)
    K.gemm(dev(x), dev(w), trans_b=True, bias=dev(bias, torch.float32), colscale=dev(gamma, torch.float32),
           rowscale=dev(rs, torch.float32), rows_per_scale=49, res=r, out=r)
    ref = res + (x @ w.t() + bias) * gamma * rs.repeat_interleave(49).view(M, 1)
    assert _rel(r.cpu(), ref) < tol
    # beta accumulate (fp32 out)
    acc = torch.randn(M, N).to(hip_device)
    acc0 = acc.cpu().clone()
    K.gemm(dev(x), dev(w), trans_b=True, out=acc, beta=1.0, alpha=0.5)
    assert _rel(acc.cpu(), acc0 + 0.5 * x @ w.t()) < tol
    # relu + dropout: deterministic, p-fraction dropped, kept scaled by 1/(1-p)
    o1 = K.gemm(dev(x), dev(w), trans_b=True, act=K.ACT_RELU, drop_p=0.5, seed=7, drop_stream=3, out_dtype=torch.float32)
    o2 = K.gemm(dev(x), dev(w), trans_b=True, act=K.ACT_RELU, drop_p=0.5, seed=7, drop_stream=3, out_dtype=torch.float32)
    assert torch.equal(o1, o2)
    base = torch.relu(x @ w.t())
    kept = (o1.cpu() != 0) & (base > 0)
    frac = kept.sum().item() / (base > 0).sum().item()
    assert 0.4 < frac < 0.6
    assert _rel(o1.cpu()[kept], 2 * base[kept]) < tol


@pytest.mark.parametrize("rows,cols", [(1000, 77), (3328, 512), (1632, 9490), (40, 64), (0, 16)])
def test_colsum(hip_device, rows, cols):
    x = torch.randn(rows, cols)
    out = torch.ones(cols, device=hip_device)
    K.colsum(x.to(hip_device), out, beta=0.5)
    assert _rel(out.cpu(), x.sum(0) + 0.5) < 1e-6


def test_colsum_multi(hip_device):
    """The batched bias-gradient column sums (imgcap_colsum_multi: a block of 32 row lanes x 8
    column vectors per 64-column group): bf16 and fp32 items, ragged widths
    (non-vector tails), row counts of 0, below, at and past a row-lane trip, beta accumulation, a row
    pitch wider than the item, an item not 16-byte aligned (scalar path); the same sums twice are
    bitwise equal."""
    g = torch.Generator().manual_seed(5)
    cases = [(1632, 9490, torch.bfloat16, 0.0, 0), (3264, 512, torch.bfloat16, 0.5, 0),
             (1023, 77, torch.float32, 0.0, 0), (1025, 2048, torch.float32, 1.0, 0), (32, 1024, torch.bfloat16, 0.0, 0),
             (5000, 100, torch.bfloat16, 0.0, 0), (0, 64, torch.bfloat16, 0.5, 0), (255, 65, torch.float32, 0.0, 0),
             (256, 512, torch.bfloat16, 0.0, 0), (257, 512, torch.bfloat16, 0.0, 1), (3328, 1536, torch.float32, 0.0, 3)]
    outs = []
    for rep in range(4):  # single-pass twice, two-pass twice
        K.ColsumBatch.TWO_PASS = rep >= 2
        cb, refs = K.ColsumBatch(), []
        for rows, cols, dtype, beta, off in cases:
            x = torch.randn(rows, cols + 8, generator=torch.Generator().manual_seed(rows * 7 + cols)).to(dtype)
            out0 = torch.randn(cols, generator=torch.Generator().manual_seed(cols))
            out = out0.to(hip_device)
            cb.add(x.to(hip_device)[:, off:off + cols], out, beta=beta)
            refs.append((out, x[:, off:off + cols].float().sum(0) + beta * out0))
        cb.run()
        for out, ref in refs:
            assert _rel(out.cpu(), ref) < 1e-5
        outs.append([o.cpu() for o, _ in refs])
    K.ColsumBatch.TWO_PASS = True
    assert all(torch.equal(a, b) for a, b in zip(outs[0], outs[1]))
    assert all(torch.equal(a, b) for a, b in zip(outs[2], outs[3]))


@pytest.mark.parametrize("dtype,tol", [(torch.float32, 1e-5), (torch.bfloat16, 1e-2)])
def test_add_layernorm_fwd_bwd(hip_device, dtype, tol):
    torch.manual_seed(1)
    rows, cols = 300, 512
    x, r = torch.randn(rows, cols), torch.randn(rows, cols)
    g, b = torch.randn(cols), torch.randn(cols)
    dy = torch.randn(rows, cols)
    xd, rd = x.to(hip_device, dtype), r.to(hip_device, dtype)
    s = torch.empty_like(xd)
    y, mean, rstd = K.add_layernorm(xd, rd, g.to(hip_device), b.to(hip_device), 1e-5, s_out=s)
    xs = (x.to(dtype).float() + r.to(dtype).float()).requires_grad_(True)
    gg, bb = g.clone().requires_grad_(True), b.clone().requires_grad_(True)
    yref = F.layer_norm(xs, (cols,), gg, bb, 1e-5)
    assert _rel(y.cpu(), yref) < tol
    yref.backward(dy)
    dg = torch.zeros(cols, device=hip_device)
    db = torch.zeros(cols, device=hip_device)
    dr = torch.empty_like(xd)
    dx = K.add_layernorm_bwd(dy.to(hip_device, dtype), s, mean, rstd, g.to(hip_device), dg, db, dr=dr)
    assert _rel(dx.cpu(), xs.grad) < tol and _rel(dr.cpu(), xs.grad) < tol
    assert _rel(dg.cpu(), gg.grad) < tol and _rel(db.cpu(), bb.grad) < tol
    # deferred parameter sums: the kernel's per-block partials, reduced with the backward's other column sums
    cb = K.ColsumBatch()
    dg2 = torch.full((cols,), 0.5, device=hip_device)
    db2 = torch.full((cols,), -0.5, device=hip_device)
    dx2 = K.add_layernorm_bwd(dy.to(hip_device, dtype), s, mean, rstd, g.to(hip_device), dg2, db2, dr=dr, cb=cb)
    cb.run()
    assert torch.equal(dx2, dx)
    assert _rel(dg2.cpu() - 0.5, gg.grad) < tol and _rel(db2.cpu() + 0.5, bb.grad) < tol


@pytest.mark.parametrize("dtype,tol", [(torch.float32, 1e-5), (torch.bfloat16, 1e-2)])
def test_cross_entropy_top5(hip_device, dtype, tol):
    torch.manual_seed(2)
    n, V = 200, 9490
    logits = torch.randn(n, V) * 3
    tgt = torch.randint(0, V, (n,))
    tgt[::7] = -1
    ld = 9496
    lg = torch.zeros(n, ld, dtype=dtype)
    lg[:, :V] = logits.to(dtype)
    lgd = lg.to(hip_device)
    lse = torch.empty(n, device=hip_device)
    loss = torch.empty(n, device=hip_device)
    hit = torch.empty(n, device=hip_device)
    td = tgt.to(hip_device)
    K.ce_fwd(lgd, td, V, lse, loss, hit)
    lf = lg[:, :V].float()
    valid = tgt >= 0
    ref_rows = F.cross_entropy(lf[valid], tgt[valid], reduction="none")
    assert _rel(loss.cpu()[valid], ref_rows) < 1e-5
    top5 = lf.topk(5, 1).indices
    ref_hit = (top5 == tgt.clamp(min=0).view(-1, 1)).any(1) & valid
    assert torch.equal(hit.cpu().bool(), ref_hit)
    out = torch.empty(4, device=hip_device)
    K.loss_finalize(loss, hit, td, None, out)
    assert abs(out[0].item() - ref_rows.mean().item()) < 1e-4 and out[1].item() == valid.sum().item()
    dl = torch.zeros(n, ld, dtype=dtype, device=hip_device)
    K.ce_bwd(lgd, td, V, lse, out[3:4], dl)
    x = lf.clone().requires_grad_(True)
    F.cross_entropy(x[valid], tgt[valid]).backward()
    assert _rel(dl[:, :V].cpu(), x.grad) < tol


@pytest.mark.parametrize("dtype,tol,V,ld", [(torch.float32, 1e-5, 9490, 9496), (torch.bfloat16, 1e-2, 9490, 9496),
                                            (torch.bfloat16, 1e-2, 9491, 9496), (torch.float32, 1e-5, 37, 40),
                                            (torch.bfloat16, 1e-2, 16384, 16384), (torch.float32, 1e-5, 12288, 12288)])
def test_cross_entropy_fused(hip_device, dtype, tol, V, ld):
    """imgcap_ce_fused (train step) == torch's cross_entropy / topk / autograd, and == the
    separate fwd + bwd kernels (same lse up to summation order, same hits, same gradient)."""
    torch.manual_seed(5)
    n = 203
    logits = torch.randn(n, V) * 3
    tgt = torch.randint(0, V, (n,))
    tgt[::7] = -1
    tgt[3] = V - 1  # target in the last (ragged) vector
    lg = torch.full((n, ld), 7.0, dtype=dtype)  # padding columns must be ignored
    lg[:, :V] = logits.to(dtype)
    lgd, td = lg.to(hip_device), tgt.to(hip_device)
    f32 = dict(device=hip_device, dtype=torch.float32)
    scale, lse, loss, hit = (torch.empty(1, **f32), torch.empty(n, **f32), torch.empty(n, **f32),
                             torch.empty(n, **f32))
    dl = torch.full((n, ld), 5.0, dtype=dtype, device=hip_device)
    K.ce_fused(lgd, td, V, scale, lse, loss, hit, dl)
    lf = lg[:, :V].float()
    valid = tgt >= 0
    assert scale.item() == torch.tensor(1.0, dtype=torch.float32).div(float(valid.sum().item())).item()
    ref_rows = F.cross_entropy(lf[valid], tgt[valid], reduction="none")
    assert _rel(loss.cpu()[valid], ref_rows) < 1e-5
    ref_hit = (lf.topk(5, 1).indices == tgt.clamp(min=0).view(-1, 1)).any(1) & valid
    assert torch.equal(hit.cpu().bool(), ref_hit)
    x = lf.clone().requires_grad_(True)
    F.cross_entropy(x[valid], tgt[valid]).backward()
    assert _rel(dl[:, :V].cpu().float(), x.grad) < tol
    pad_end = (V + (8 if dtype == torch.bfloat16 else 4) - 1) // (8 if dtype == torch.bfloat16 else 4) * (
        8 if dtype == torch.bfloat16 else 4)
    assert torch.all(dl[:, V:pad_end] == 0)
    # the two-kernel path on the same rows
    lse2, loss2, hit2 = torch.empty(n, **f32), torch.empty(n, **f32), torch.empty(n, **f32)
    K.ce_fwd(lgd, td, V, lse2, loss2, hit2)
    assert torch.allclose(lse, lse2, rtol=1e-6, atol=1e-5) and torch.equal(hit, hit2)
    dl2 = torch.zeros(n, ld, dtype=dtype, device=hip_device)
    K.ce_bwd(lgd, td, V, lse2, scale, dl2)
    assert _rel(dl[:, :V].float(), dl2[:, :V].float()) < (1e-5 if dtype == torch.float32 else 5e-3)


def test_clamp_adam_matches_oracle(hip_device):
    from oracle import train_step
    torch.manual_seed(3)
    n = 10007
    p, g = torch.randn(n), torch.randn(n) * 4
    m, v = torch.zeros(n), torch.zeros(n)
    pd, gd, md, vd = (t.to(hip_device) for t in (p, g, m, v))
    shadow = torch.empty(n, dtype=torch.bfloat16, device=hip_device)
    st = {}
    ref = {"x": p}
    for step in (1, 2, 3):
        K.clamp_adam(pd, gd, md, vd, shadow, 1e-4, step, 5.0)
        ref = train_step.adam_step(ref, train_step.clip_gradient({"x": g}, 5.0), st, 1e-4, step)
    torch.testing.assert_close(pd.cpu(), ref["x"], rtol=1e-6, atol=1e-7)
    assert torch.equal(shadow.cpu(), pd.cpu().bfloat16())


def test_embedding_fwd_bwd(hip_device):
    V, dim, n = 50, 64, 300
    table = torch.randn(V, dim)
    ids = torch.randint(0, V, (n,))
    pe = torch.randn(12, dim)
    out = torch.empty(n, dim, device=hip_device)
    K.embedding_fwd(ids.to(hip_device), table.to(hip_device), out, pe=pe.to(hip_device), L=12)
    ref = table[ids] + pe[torch.arange(n) % 12]
    assert _rel(out.cpu(), ref) < 1e-6
    dout = torch.randn(n, dim)
    dt_ = torch.zeros(V, dim, device=hip_device)
    K.embedding_bwd(ids.to(hip_device), dout.to(hip_device), dt_)
    refd = torch.zeros(V, dim).index_add_(0, ids, dout)
    assert _rel(dt_.cpu(), refd) < 1e-5


@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float32])
@pytest.mark.parametrize("with_pe", [False, True])
def test_embedding_fwd_vector_form_bitwise(hip_device, dtype, with_pe):
    """The 8-column form (dim % 8 == 0, 16-byte aligned rows) against the element form (forced by
    a misaligned output view): bitwise equal, dropout mask included."""
    g = torch.Generator().manual_seed(3)
    V, dim, n, L = 9490, 512, 1632, 51
    table = torch.randn(V, dim, generator=g).to(hip_device)
    ids = torch.randint(0, V, (n,), generator=g).to(hip_device)
    pe = torch.randn(L, dim, generator=g).to(hip_device) if with_pe else None
    out = torch.empty(n, dim, device=hip_device, dtype=dtype)
    K.embedding_fwd(ids, table, out, pe=pe, L=L, drop_p=0.3, seed=11, drop_stream=4)
    base = torch.empty(n * dim + 1, device=hip_device, dtype=dtype)
    out2 = base[1:].view(n, dim)  # 2 / 4 bytes off 16-byte alignment: the element form
    K.embedding_fwd(ids, table, out2, pe=pe, L=L, drop_p=0.3, seed=11, drop_stream=4)
    assert torch.equal(out, out2)
    if not with_pe:
        kept = (out != 0).float().mean().item()
        assert 0.6 < kept < 0.8


@pytest.mark.parametrize("dtype,tol", [(torch.float32, 1e-5), (torch.bfloat16, 1.5e-2)])
@pytest.mark.parametrize("H,C", [(56, 96), (28, 192), (14, 384), (7, 768), (8, 256), (16, 128)])
def test_dwconv7_ln(hip_device, dtype, tol, H, C):
    torch.manual_seed(H + C)
    B = 2
    x = torch.randn(B, H, H, C)
    w = torch.randn(C, 1, 7, 7) * 0.2
    bias, lw, lb = torch.randn(C), torch.randn(C), torch.randn(C)
    xin = x.to(dtype).float()
    ref = F.conv2d(xin.permute(0, 3, 1, 2), w, bias, padding=3, groups=C).permute(0, 2, 3, 1)
    ref = F.layer_norm(ref, (C,), lw, lb, 1e-6)
    w49 = w.view(C, 49).t().contiguous().to(hip_device)
    out = torch.empty(B, H, H, C, dtype=dtype, device=hip_device)
    K.dwconv7_ln(x.to(hip_device, dtype), w49, bias.to(hip_device), lw.to(hip_device), lb.to(hip_device), out)
    assert _rel(out.cpu(), ref) < tol


@pytest.mark.parametrize("dtype,tol", [(torch.float32, 1e-6), (torch.bfloat16, 1e-2)])
@pytest.mark.parametrize("B,H,C", [(3, 56, 96), (2, 28, 192), (3, 14, 384), (5, 7, 768), (2, 8, 256), (3, 16, 128), (3, 4, 64), (2, 12, 96), (3, 2, 32),
                                   (1, 64, 32), (4, 32, 1536)])
def test_dwconv7(hip_device, dtype, tol, B, H, C):
    """Depthwise 7x7 + bias (no LN), tiles spanning image boundaries in the flattened rows."""
    torch.manual_seed(B * H + C)
    x = torch.randn(B, H, H, C)
    w = torch.randn(C, 1, 7, 7) * 0.2
    bias = torch.randn(C)
    xin = x.to(dtype).float()
    ref = F.conv2d(xin.permute(0, 3, 1, 2), w, bias, padding=3, groups=C).permute(0, 2, 3, 1)
    w49 = w.view(C, 49).t().contiguous().to(hip_device)
    out = torch.empty(B, H, H, C, dtype=dtype, device=hip_device)
    K.dwconv7(x.to(hip_device, dtype), w49, bias.to(hip_device), out)
    assert _rel(out.cpu(), ref) < tol


@pytest.mark.parametrize("dtype,tol", [(torch.float32, 1e-6), (torch.bfloat16, 1e-2)])
@pytest.mark.parametrize("B,H,C", [(5, 56, 96), (3, 28, 64), (7, 14, 32), (11, 7, 64), (3, 16, 32), (2, 15, 32)])
def test_dwconv7_row_tiles(hip_device, dtype, tol, B, H, C):
    """The depthwise kernels (compile-time widths, and the runtime-width one at W = 15): tiles
    crossing image boundaries and the partial last block; forward, and the flipped (transposed)
    pass of the backward + residual."""
    from imagecaptioningconvnext_amd import kernels as K
    torch.manual_seed(B * H + C)
    x = torch.randn(B, H, H, C)
    w = torch.randn(C, 1, 7, 7) * 0.2
    bias = torch.randn(C)
    res = torch.randn(B, H, H, C)
    xin = x.to(dtype).float()
    ref = F.conv2d(xin.permute(0, 3, 1, 2), w, bias, padding=3, groups=C).permute(0, 2, 3, 1)
    w49 = w.view(C, 49).t().contiguous().to(hip_device)
    out = torch.empty(B, H, H, C, dtype=dtype, device=hip_device)
    K.dwconv7(x.to(hip_device, dtype), w49, bias.to(hip_device), out)
    assert _rel(out.cpu(), ref) < tol
    # backward data: the transposed conv (flipped taps) of x, plus the residual
    reft = F.conv_transpose2d(xin.permute(0, 3, 1, 2), w, padding=3, groups=C).permute(0, 2, 3, 1)
    reft = reft + res.to(dtype).float()
    dx = torch.empty(B, H, H, C, dtype=dtype, device=hip_device)
    K.dwconv7_bwd_data(x.to(hip_device, dtype), w49, dx, res=res.to(hip_device, dtype))
    assert _rel(dx.cpu(), reft) < tol


@pytest.mark.parametrize("C,M", [(96, 700), (192, 300)])
def test_cnblock_mlp_with_layernorm(hip_device, C, M):
    """LN (eps 1e-6) in the MLP prologue == LN kernel then MLP (z rounded to bf16 either way)."""
    g = torch.Generator(device="cpu").manual_seed(C)
    y = (torch.randn(M, C, generator=g) * 3 + 1).bfloat16()
    x = torch.randn(M, C, generator=g).bfloat16()
    w1 = (torch.randn(4 * C, C, generator=g) / math.sqrt(C)).bfloat16()
    w2 = (torch.randn(C, 4 * C, generator=g) / math.sqrt(4 * C)).bfloat16()
    b1, b2, gamma, lw, lb = (torch.randn(n, generator=g) for n in (4 * C, C, C, C, C))
    z = F.layer_norm(y.float(), (C,), lw, lb, 1e-6).bfloat16().float()
    hid = F.gelu(z @ w1.float().t() + b1).bfloat16().float()
    delta = (hid @ w2.float().t() + b2) * gamma
    d = lambda t: t.to(hip_device)  # noqa: E731
    xd = d(x)
    K.cnblock_mlp(d(y), d(w1), d(b1), d(w2), d(b2), d(gamma), xd, ln_w=d(lw), ln_b=d(lb))
    assert _rel(xd.cpu().float() - x.float(), delta) < 2e-2


@pytest.mark.parametrize("dtype,tol", [(torch.float32, 1e-5), (torch.bfloat16, 1e-2)])
@pytest.mark.parametrize("C0,HW,B", [(96, 224, 2), (128, 224, 2), (192, 256, 2), (192, 224, 24)])  # last: > 1024 groups
def test_stem(hip_device, dtype, tol, C0, HW, B):
    torch.manual_seed(C0)
    img = torch.randn(B, 3, HW, HW)
    w = torch.randn(C0, 3, 4, 4) * 0.1
    b, lw, lb = torch.randn(C0), torch.randn(C0), torch.randn(C0)
    ref = F.conv2d(img, w, b, stride=4).permute(0, 2, 3, 1)
    ref = F.layer_norm(ref, (C0,), lw, lb, 1e-6)
    out = torch.empty(B, HW // 4, HW // 4, C0, dtype=dtype, device=hip_device)
    K.convnext_stem(img.to(hip_device), w.view(C0, 48).contiguous().to(hip_device), b.to(hip_device),
                    lw.to(hip_device), lb.to(hip_device), out)
    assert _rel(out.cpu(), ref) < tol


@pytest.mark.parametrize("dtype,tol", [(torch.float32, 1e-5), (torch.bfloat16, 1e-2)])
def test_ln_patchify_and_downsample(hip_device, dtype, tol):
    torch.manual_seed(5)
    B, H, C = 2, 14, 384
    x = torch.randn(B, H, H, C)
    lw, lb = torch.randn(C), torch.randn(C)
    wc = torch.randn(2 * C, C, 2, 2) * 0.05
    bc = torch.randn(2 * C)
    xin = x.to(dtype).float()
    ref = F.layer_norm(xin, (C,), lw, lb, 1e-6).permute(0, 3, 1, 2)
    ref = F.conv2d(ref, wc, bc, stride=2).permute(0, 2, 3, 1)
    patches = torch.empty(B * (H // 2) ** 2, 4 * C, dtype=dtype, device=hip_device)
    K.ln_patchify2(x.to(hip_device, dtype), lw.to(hip_device), lb.to(hip_device), patches)
    wpk = wc.permute(0, 2, 3, 1).reshape(2 * C, 4 * C).to(hip_device, dtype)
    out = K.gemm(patches, wpk, trans_b=True, bias=bc.to(hip_device), out_dtype=torch.float32)
    assert _rel(out.cpu().view(B, H // 2, H // 2, 2 * C), ref) < tol


def test_adaptive_pool(hip_device):
    x = torch.randn(2, 8, 8, 64)
    ref = F.adaptive_avg_pool2d(x.permute(0, 3, 1, 2), 7).permute(0, 2, 3, 1)
    out = torch.empty(2, 7, 7, 64, device=hip_device)
    K.adaptive_pool(x.to(hip_device), 7, 7, out)
    assert _rel(out.cpu(), ref) < 1e-6


def test_transpose(hip_device):
    for dtype in (torch.float32, torch.bfloat16):
        x = torch.randn(130, 200).to(hip_device, dtype)
        view = x[:, 8:72]
        out = K.transpose(view)
        assert torch.equal(out.cpu(), view.cpu().t())


@pytest.mark.parametrize("C,M", [(96, 1000), (128, 300), (192, 520)])
@pytest.mark.parametrize("with_sd", [False, True])
def test_cnblock_mlp_fused(hip_device, C, M, with_sd):
    """Fused CNBlock MLP vs torch: x + gamma*sd*(GELU(z W1^T + b1) W2^T + b2), hidden in bf16."""
    g = torch.Generator(device="cpu").manual_seed(C + M)
    z = torch.randn(M, C, generator=g).bfloat16()
    x = torch.randn(M, C, generator=g).bfloat16()
    w1 = (torch.randn(4 * C, C, generator=g) / math.sqrt(C)).bfloat16()
    w2 = (torch.randn(C, 4 * C, generator=g) / math.sqrt(4 * C)).bfloat16()
    b1, b2, gamma = (torch.randn(n, generator=g) for n in (4 * C, C, C))
    rps = 49
    sd = (torch.rand((M + rps - 1) // rps, generator=g) > 0.3).float() / 0.7 if with_sd else None
    hid = F.gelu(z.float() @ w1.float().t() + b1).bfloat16().float()
    delta = (hid @ w2.float().t() + b2) * gamma
    if with_sd:
        delta = delta * sd.repeat_interleave(rps)[:M].view(M, 1)
    xd = x.to(hip_device)
    dev = lambda t: None if t is None else t.to(hip_device)  # noqa: E731
    K.cnblock_mlp(dev(z), dev(w1), dev(b1), dev(w2), dev(b2), dev(gamma), xd, sd=dev(sd), rows_per_sample=rps)
    got = xd.cpu().float() - x.float()
    assert _rel(got, delta) < 2e-2


@pytest.mark.parametrize("C,M", [(96, 70001), (192, 40000)])
def test_cnblock_mlp_large_grids(hip_device, C, M):
    """Stage-sized row counts: the resident C = 96 kernel deals more 32-row units than the grid
    has waves (each wave walks several), the streamed C = 192 kernel runs hundreds of blocks; LN in
    the prologue and drop path on, vs torch fp32 on the bf16-rounded operands (gate as above)."""
    g = torch.Generator(device="cpu").manual_seed(M)
    y = (torch.randn(M, C, generator=g) * 2 + 0.5).bfloat16()
    x = torch.randn(M, C, generator=g).bfloat16()
    w1 = (torch.randn(4 * C, C, generator=g) / math.sqrt(C)).bfloat16()
    w2 = (torch.randn(C, 4 * C, generator=g) / math.sqrt(4 * C)).bfloat16()
    b1, b2, gamma, lw, lb = (torch.randn(n, generator=g) for n in (4 * C, C, C, C, C))
    rps = 3136
    sd = (torch.rand((M + rps - 1) // rps, generator=g) > 0.3).float() / 0.7
    z = F.layer_norm(y.float(), (C,), lw, lb, 1e-6).bfloat16().float()
    hid = F.gelu(z @ w1.float().t() + b1).bfloat16().float()
    delta = (hid @ w2.float().t() + b2) * gamma * sd.repeat_interleave(rps)[:M].view(M, 1)
    d = lambda t: t.to(hip_device)  # noqa: E731
    xd = d(x)
    K.cnblock_mlp(d(y), d(w1), d(b1), d(w2), d(b2), d(gamma), xd, sd=d(sd), rows_per_sample=rps, ln_w=d(lw),
                  ln_b=d(lb))
    got = xd.cpu().float() - x.float()
    assert _rel(got, delta) < 2e-2
    assert torch.isfinite(got).all()


def test_gemm_grouped_weight_gradients(hip_device):
    """GemmBatch / imgcap_gemm_grouped: many dW = dY^T X products (ragged M, N, K, strided
    outputs, alpha/beta) in one grouped launch vs torch fp32 on the bf16-rounded operands."""
    g = torch.Generator().manual_seed(3)
    shapes = [(512, 512, 3328), (1536, 512, 3328), (9490, 512, 1632), (70, 200, 100), (256, 768, 3136), (8, 16, 64)]
    batch = K.GemmBatch()
    cases = []
    for i, (M, N, Kd) in enumerate(shapes):
        dy = torch.randn(Kd, M, generator=g)
        x = torch.randn(Kd, N, generator=g)
        dyd, xd = _padded(dy, hip_device, torch.bfloat16), _padded(x, hip_device, torch.bfloat16)
        big = torch.randn(M, N + 24, generator=g)
        out = big.to(hip_device)[:, 8:8 + N]                      # strided fp32 output view
        alpha, beta = (1.0, 0.0) if i % 2 == 0 else (0.5, 1.0)
        batch.add(dyd, xd, out, trans_a=True, M=M, N=N, K=Kd, alpha=alpha, beta=beta)
        ref = alpha * dy.bfloat16().float().t() @ x.bfloat16().float() + beta * big[:, 8:8 + N]
        cases.append((out, ref))
    batch.run()
    for out, ref in cases:
        assert _rel(out.cpu(), ref) < 1e-5


@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float32])
@pytest.mark.parametrize("B,P,E", [(1, 49, 768), (5, 49, 768), (32, 49, 768), (256, 49, 768), (3, 64, 1000),
                                   (2, 1, 1024)])
def test_sort_gather_rows(hip_device, dtype, B, P, E):
    """decoder.py:64,79-81 fused: stable descending length sort (ties keep batch order), the
    gathered encoder rows / captions bit-exact, decode lengths, and the pixel mean (column chunks
    of 32 vectors: a ragged last chunk at E = 1000)."""
    g = torch.Generator(device="cpu").manual_seed(B)
    L = 52
    lens = torch.randint(8, 14, (B, 1), generator=g)  # many ties
    enc = torch.randn(B, P, E, generator=g).to(dtype)
    caps = torch.randint(0, 9490, (B, L), generator=g)
    enc_s, mean, caps_s, ind, dl = K.sort_gather_rows(lens.reshape(-1).to(hip_device), enc.to(hip_device),
                                                      caps.to(hip_device))
    ref_len, ref_ind = lens.reshape(-1).sort(dim=0, descending=True, stable=True)
    assert torch.equal(ind.cpu(), ref_ind)
    assert torch.equal(dl.cpu(), (ref_len - 1).to(torch.int32))
    assert torch.equal(enc_s.cpu(), enc.index_select(0, ref_ind))
    assert torch.equal(caps_s.cpu(), caps.index_select(0, ref_ind))
    ref_mean = torch.empty(B, E, device=hip_device, dtype=dtype)
    K.mean_mid(enc_s, ref_mean)  # the unfused kernel: identical summation order
    assert torch.equal(mean, ref_mean)
    assert _rel(mean.cpu(), enc.index_select(0, ref_ind).float().mean(1)) < (1e-2 if dtype == torch.bfloat16 else 1e-6)


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("n,V,dim", [(1632, 9490, 512), (3328, 120, 512), (7, 5, 40), (200, 9490, 1000)])
def test_embedding_bwd_deterministic(hip_device, dtype, n, V, dim):
    """Rows of each id summed in position order (no float atomics): equal to a sequential fp64
    sum to fp32 rounding, bitwise identical across runs, dropout mask as the forward's."""
    from imagecaptioningconvnext_amd import kernels as K
    g = torch.Generator().manual_seed(n)
    ids = torch.randint(0, V, (n,), generator=g)
    ids[: n // 3] = ids[0]  # a very frequent word
    dout = torch.randn(n, dim, generator=g).to(dtype)
    ref = torch.zeros(V, dim, dtype=torch.float64).index_add_(0, ids, dout.double())
    outs = []
    for _ in range(3):
        dt_ = torch.zeros(V, dim, device=hip_device)
        K.embedding_bwd(ids.to(hip_device), dout.to(hip_device), dt_)
        outs.append(dt_.cpu())
    assert torch.equal(outs[0], outs[1]) and torch.equal(outs[0], outs[2])
    assert ((outs[0].double() - ref).norm() / ref.norm()).item() < 1e-6
    # with dropout: bitwise repeatable too
    a = torch.zeros(V, dim, device=hip_device)
    b = torch.zeros(V, dim, device=hip_device)
    K.embedding_bwd(ids.to(hip_device), dout.to(hip_device), a, drop_p=0.5, seed=9, drop_stream=3)
    K.embedding_bwd(ids.to(hip_device), dout.to(hip_device), b, drop_p=0.5, seed=9, drop_stream=3)
    assert torch.equal(a, b) and not torch.equal(a.cpu(), outs[0])


def test_caller_workspace_grows_on_demand(hip_device):
    """Split-K scratch comes from the caller's attached buffer (imgcap_workspace_attach); a call
    that needs more returns IMGCAP_EWORKSPACE without enqueuing anything, the binding attaches a
    bigger buffer and retries."""
    import ctypes
    from imagecaptioningconvnext_amd import _abi
    from imagecaptioningconvnext_amd import kernels as K
    dev = torch.cuda.current_device()
    a = torch.randn(512, 9600, device=hip_device).bfloat16()
    b = torch.randn(9600, 512, device=hip_device).bfloat16()
    K.gemm(a[:8], b)  # first call attaches the initial buffers
    _abi._attach(dev, 0, 1 << 20)  # shrink slot 0 to 1 MB
    small = _abi._ws[(dev, 0)]
    c = K.gemm(a, b, split_k=8, out_dtype=torch.float32)  # 8 x 512 x 512 fp32 partials = 8 MB
    assert _abi._ws[(dev, 0)].numel() > small.numel()
    need = ctypes.c_uint64(0)
    _abi.lib().imgcap_workspace_needed(0, ctypes.byref(need))
    assert need.value >= 8 * 512 * 512 * 4
    ref = a.float() @ b.float()
    assert ((c - ref).norm() / ref.norm()).item() < 1e-5


@pytest.mark.parametrize("C", [96, 192, 768, 1024, 20])
@pytest.mark.parametrize("cmajor", [False, True])
@pytest.mark.parametrize("dtype,tol", [(torch.float32, 1e-5), (torch.bfloat16, 1e-2)])
def test_ln_patchify2_widths(hip_device, C, cmajor, dtype, tol):
    """LayerNorm2d + 2x2 patch rows at the ConvNeXt widths (the vectorised patch kernel: thread
    = 8 channels of a patch's four pixels) and at C % 8 != 0 (the wave-per-pixel kernel), both
    patch-row layouts, against torch LN + the same permutation."""
    B, H = 3, 10
    g = torch.Generator().manual_seed(C)
    x = torch.randn(B, H, H, C, generator=g) * 2 + 0.5
    lw, lb = 1 + 0.2 * torch.randn(C, generator=g), 0.2 * torch.randn(C, generator=g)
    y = F.layer_norm(x.to(dtype).float(), (C,), lw, lb, 1e-6).view(B, H // 2, 2, H // 2, 2, C)
    ref = (y.permute(0, 1, 3, 5, 2, 4) if cmajor else y.permute(0, 1, 3, 2, 4, 5)).reshape(-1, 4 * C)
    got = torch.empty(ref.shape, dtype=dtype, device=hip_device)
    K.ln_patchify2(x.to(hip_device, dtype), lw.to(hip_device), lb.to(hip_device), got, cmajor=cmajor)
    assert _rel(got.cpu(), ref) < tol


@pytest.mark.gpu
@pytest.mark.parametrize("B,L", [(1, 1), (3, 7), (64, 52), (5, 300)])
def test_tf_targets_match_reference_formulas(hip_device, B, L):
    """imgcap_tf_targets vs the Transformer trainer's torch formulas (transformerDecoder.py:88-108,
    train.py:262-276): decode mask l < len - 1, target caps[:, l+1] or -1, metrics zeroed.  Lengths
    cover 1 (nothing decoded), 2, L and values in between; ids are arbitrary int64."""
    g = torch.Generator().manual_seed(11 + B * L)
    caps = torch.randint(0, 1 << 40, (B, L), generator=g, dtype=torch.int64)
    lens = torch.randint(1, L + 1, (B, 1), generator=g, dtype=torch.int64)
    lens[0, 0] = 1
    if B > 1:
        lens[1, 0] = L
    if B > 2:
        lens[2, 0] = min(2, L)
    dl = lens.reshape(-1) - 1
    tmask = torch.arange(L).view(1, L) < dl.view(B, 1)
    nxt = torch.cat([caps[:, 1:], caps[:, :1]], dim=1)
    targets = torch.where(tmask, nxt, torch.full_like(nxt, -1)).reshape(-1)
    tm, tg, mt = K.tf_targets(caps.to(hip_device), lens.to(hip_device))
    torch.cuda.synchronize()
    assert torch.equal(tm.cpu(), tmask)
    assert torch.equal(tg.cpu(), targets)
    assert torch.equal(mt.cpu(), torch.zeros(5))


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("n,V,dim,run", [(3328, 120, 512, 2500), (700, 50, 40, 300), (129, 7, 1000, 100),
                                         (256, 3, 64, 0)])
def test_embedding_bwd_long_runs_chunked_order(hip_device, dtype, n, V, dim, run):
    """A padding id occupying thousands of positions (captions padded to L) is summed by many
    waves: the sorted index array is cut at multiples of 16 (EMB_CH), each piece of a run is added
    in position order and the pieces of a run in chunk order.  The table must be bitwise that fp32
    order (restated here), and within fp32 rounding of the fp64 sum."""
    from imagecaptioningconvnext_amd import kernels as K
    g = torch.Generator().manual_seed(n + run)
    ids = torch.randint(0, V, (n,), generator=g)
    if run:
        ids[torch.randperm(n, generator=g)[:run]] = 0  # the padding id, spread over the positions
    dout = torch.randn(n, dim, generator=g).to(dtype)
    x = dout.float()
    order = sorted(range(n), key=lambda i: (int(ids[i]), i))
    sid = [int(ids[o]) for o in order]
    ref = torch.zeros(V, dim, dtype=torch.float32)
    i = 0
    while i < n:
        e = i
        while e < n and sid[e] == sid[i]:
            e += 1
        pieces, a = [], i
        while a < e:
            b = min(e, (a // 16 + 1) * 16)
            acc = torch.zeros(dim)
            for t in range(a, b):
                acc = acc + x[order[t]]
            pieces.append(acc)
            a = b
        tot = pieces[0]
        for pc in pieces[1:]:
            tot = tot + pc
        ref[sid[i]] = ref[sid[i]] + tot
        i = e
    got = torch.zeros(V, dim, device=hip_device)
    K.embedding_bwd(ids.to(hip_device), dout.to(hip_device), got)
    got = got.cpu()
    assert torch.equal(got, ref)
    r64 = torch.zeros(V, dim, dtype=torch.float64).index_add_(0, ids, x.double())
    assert ((got.double() - r64).norm() / r64.norm()).item() < 1e-6


"""Kernel microbenchmarks at the bench step's shapes (GPU box): python tools/microbench.py [group]

Times each launch with HIP events over back-to-back repetitions on random data and prints
achieved TFLOP/s or GB/s.  Used to iterate on kernel variants; numbers quoted in DESIGN.md.
"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from imagecaptioningconvnext_amd import kernels as K  # noqa: E402

dev = torch.device("cuda:0")
bf = torch.bfloat16


def time_launch(fn, reps=50, warm=5, graph=True):
    """Seconds per launch of ``fn``, HIP events around ``reps`` back-to-back launches (captured
    into one HIP graph and replayed with graph=True, so host launch cost does not hide short
    kernels)."""
    for _ in range(warm):
        fn()
    torch.cuda.synchronize()
    g = None
    if graph:
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            for _ in range(reps):
                fn()
        g.replay()
        torch.cuda.synchronize()
    st = torch.cuda.current_stream()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record(st)
    if g is not None:
        g.replay()
    else:
        for _ in range(reps):
            fn()
    b.record(st)
    b.synchronize()
    return a.elapsed_time(b) / reps * 1e-3


def gemm_case(name, M, N, Kd, ta=False, tb=True, act=0, out_dtype=bf, reps=30, split_k=0):
    r8 = lambda x: (x + 7) // 8 * 8  # noqa: E731  (16-byte row pitch, as the engines allocate)
    a = torch.randn(Kd, r8(M), device=dev).to(bf)[:, :M] if ta else torch.randn(M, r8(Kd), device=dev).to(bf)[:, :Kd]
    b = torch.randn(N, r8(Kd), device=dev).to(bf)[:, :Kd] if tb else torch.randn(Kd, r8(N), device=dev).to(bf)[:, :N]
    out = torch.empty(M, N, device=dev, dtype=out_dtype)
    beta = 0.0
    t = time_launch(lambda: K.gemm(a, b, trans_a=ta, trans_b=tb, out=out, act=act, beta=beta, split_k=split_k),
                    reps=reps)
    tf = 2.0 * M * N * Kd / t / 1e12
    name = name + (f" split={split_k}" if split_k else "")
    print(f"{name:46s} M={M:6d} N={N:5d} K={Kd:5d} {'T' if ta else 'N'}{'T' if tb else 'N'}  "
          f"{t * 1e6:8.1f} us  {tf:7.1f} TFLOP/s")


def gemms():
    B = 32
    gemm_case("enc s1 pw1 (C->4C, GELU)", B * 3136, 384, 96, act=K.ACT_GELU)
    gemm_case("enc s1 pw2 (4C->C)", B * 3136, 96, 384)
    gemm_case("enc s3 pw1", B * 196, 1536, 384, act=K.ACT_GELU)
    gemm_case("enc s3 pw2", B * 196, 384, 1536)
    gemm_case("fc logits", 1632, 9490, 512)
    gemm_case("fc dW (TN)", 9490, 512, 1632, ta=True, tb=False, out_dtype=torch.float32)
    gemm_case("fc dX (NN)", 1632, 512, 9490, tb=False)
    gemm_case("trf in_proj (B=64)", 3328, 1536, 512)
    gemm_case("trf in_proj dW (TN)", 1536, 512, 3328, ta=True, tb=False, out_dtype=torch.float32)
    for sk in (0, -1, 4, 8):
        gemm_case("trf in_proj dW (TN)", 1536, 512, 3328, ta=True, tb=False, out_dtype=torch.float32, split_k=sk)
        gemm_case("trf ff dW (TN)", 512, 512, 3328, ta=True, tb=False, out_dtype=torch.float32, split_k=sk)
        gemm_case("fc dW (TN) C3", 9490, 512, 3328, ta=True, tb=False, out_dtype=torch.float32, split_k=sk)
    gemm_case("trf in_proj dX (NN)", 3328, 512, 1536, tb=False)
    gemm_case("trf ffn (B=64)", 3328, 512, 512)
    gemm_case("big square", 4096, 4096, 4096)
    gemm_case("lstm G1 (skinny)", 32, 3328, 512, out_dtype=torch.float32)
    gemm_case("lstm G2 (skinny)", 32, 2048, 768, out_dtype=torch.float32)
    gemm_case("lstm dz (skinny)", 32, 768, 2048, out_dtype=torch.float32)
    gemm_case("lstm dh (skinny)", 32, 512, 3328, out_dtype=torch.float32)


def gemm_probe():
    for pol in (0, 1):
        K.gemm_set_policy(pol)
        print(f"-- policy glds256={pol}")
        _gemm_probe()
    for pol in (-1, 4, 5):
        K.gemm_set_policy(pol)
        print(f"-- policy {pol}: step shapes")
        gemms()
    K.gemm_set_policy(-1)


def _gemm_probe():
    """Where the time of a 128x128-tile GEMM goes at the encoder shapes: epilogue variants and K."""
    M, N = 6272, 1536
    for Kd in (384, 768, 1536, 3072):
        gemm_case("probe act=none bf16", M, N, Kd)
    gemm_case("probe act=gelu bf16", M, N, 384, act=K.ACT_GELU)
    gemm_case("probe act=none f32", M, N, 384, out_dtype=torch.float32)
    for Mx in (1568, 3136, 12544, 25088):
        gemm_case("probe M sweep", Mx, N, 384)
    gemm_case("probe square 4096", 4096, 4096, 4096)
    gemm_case("probe square 8192", 8192, 8192, 8192, reps=5)


def mlp():
    """Fused CNBlock MLP vs the two-GEMM form at the Tiny stage shapes (B=32)."""
    B = 32
    for (H, C) in ((56, 96), (28, 192), (14, 384)):
        M = B * H * H
        z = torch.randn(M, C, device=dev).to(bf)
        x = torch.randn(M, C, device=dev).to(bf)
        w1 = (torch.randn(4 * C, C, device=dev) / C ** 0.5).to(bf)
        w2 = (torch.randn(C, 4 * C, device=dev) / (4 * C) ** 0.5).to(bf)
        b1, b2, gm = torch.randn(4 * C, device=dev), torch.randn(C, device=dev), torch.randn(C, device=dev) * 1e-3
        hid = torch.empty(M, 4 * C, device=dev, dtype=bf)
        flops = 2.0 * 2 * M * C * 4 * C
        if C <= 192:
            t = time_launch(lambda: K.cnblock_mlp(z, w1, b1, w2, b2, gm, x), reps=20)
            print(f"cnblock_mlp fused  M={M:6d} C={C:4d}: {t * 1e6:8.1f} us {flops / t / 1e12:7.1f} TFLOP/s")

        def unfused():
            K.gemm(z, w1, trans_b=True, bias=b1, act=K.ACT_GELU, out=hid)
            K.gemm(hid, w2, trans_b=True, bias=b2, colscale=gm, res=x, out=x)
        t = time_launch(unfused, reps=20)
        print(f"cnblock_mlp 2-GEMM M={M:6d} C={C:4d}: {t * 1e6:8.1f} us {flops / t / 1e12:7.1f} TFLOP/s")


def lstm():
    """LSTM recurrence at the C2 shape (B=32, T=51, E=768, A=D=M=512): whole imgcap_lstm_tf_fwd /
    _bwd launches (3 kernels per step each) replayed from a graph; per-step time = total / T."""
    import ctypes
    from imagecaptioningconvnext_amd import _abi
    from imagecaptioningconvnext_amd.models.decoder import DecoderWithAttention
    B, L, V = int(os.environ.get("IMGCAP_MB_B", "32")), 52, 9490
    dec = DecoderWithAttention(attention_dim=512, embed_dim=512, decoder_dim=512, vocab_size=V, device=dev,
                               encoder_dim=768, dropout=0.5, compute_dtype=bf).to(dev)
    eng = dec.engine()
    enc = torch.randn(B, 7, 7, 768, device=dev).to(bf)
    caps = torch.randint(1, V - 3, (B, L), device=dev)
    lens = torch.full((B, 1), L, device=dev, dtype=torch.long)
    s = eng.forward(enc, caps, lens, fixed_T=True)
    eng.backward(s)
    d = s["desc"]
    T = s["T"]
    ws = s["bwd_bufs"]["chain_ws"]
    t = time_launch(lambda: eng._launch("imgcap_lstm_tf_fwd", d), reps=5, warm=2)
    print(f"lstm fwd recurrence B={B} ({eng.CHAINS} chains): {t * 1e6:8.1f} us total, {t * 1e6 / T:6.2f} us/step")
    te = time_launch(lambda: eng._launch("imgcap_lstm_tf_fwd", d), reps=5, warm=2, graph=False)
    print(f"lstm fwd recurrence ({eng.CHAINS} chains, eager streams): {te * 1e6:8.1f} us total")
    t = time_launch(lambda: eng._launch("imgcap_lstm_tf_bwd", d, ws), reps=5, warm=2)
    print(f"lstm bwd recurrence: {t * 1e6:8.1f} us total, {t * 1e6 / T:6.2f} us/step")
    if os.environ.get("IMGCAP_LSTM_STAMPS") == "1" and d.sync:
        # phase stamps of the persistent forward (lstm_persist.hip, stamp()): 100 MHz ticks
        eng._launch("imgcap_lstm_tf_fwd", d)
        torch.cuda.synchronize()
        words = _abi.lib().imgcap_lstm_sync_words(ctypes.byref(d))
        off = (words + 63) // 64 * 64 + 64
        st = eng._sync[off:off + 2 * 64 * 16 * 2].view(torch.int64).view(2, 64, 16).cpu().double() * 10.0  # ns
        u, r = st[0, 1:T - 1], st[1, 1:T - 1]
        nxt = st[0, 2:T, 0]
        names = ["wait h", "G h loads", "G mma+store", "G publish", "wait z (U)", "U z loads", "U mma",
                 "cell+h store", "h publish", "->next step"]
        segs = [u[:, 1] - u[:, 0], u[:, 9] - u[:, 1], u[:, 2] - u[:, 9], u[:, 3] - u[:, 2], u[:, 4] - u[:, 3],
                u[:, 8] - u[:, 4], u[:, 5] - u[:, 8], u[:, 6] - u[:, 5], u[:, 7] - u[:, 6], nxt - u[:, 7]]
        print("U/G block 0, mean ns per step: " + ", ".join(f"{n} {x.mean():.0f}" for n, x in zip(names, segs)))
        rn = ["wait g", "g loads", "scores", "softmax", "context+z", "z publish", "->next"]
        rs = [r[:, 1] - r[:, 0], r[:, 5] - r[:, 1], r[:, 6] - r[:, 5], r[:, 7] - r[:, 6], r[:, 3] - r[:, 7],
              r[:, 4] - r[:, 3], st[1, 2:T, 0] - r[:, 4]]
        print("R block 0,     mean ns per step: " + ", ".join(f"{n} {x.mean():.0f}" for n, x in zip(rn, rs)))
        clk = (st[0, T - 2, 15] - st[0, 1, 15]) / 10.0 / (st[0, T - 2, 0] - st[0, 1, 0]) * 1e3  # MHz
        print(f"shader clock during the recurrence: {clk:.0f} MHz")
        print("cross: G published -> R got g %.0f ns; R published -> U got z %.0f ns; U published -> U got h %.0f" % (
            (r[:, 1] - u[:, 3]).mean(), (u[:, 4] - r[:, 4]).mean(), (st[0, 2:T, 1] - u[:, 7]).mean()))
        # the persistent backward (lstm_bwd_persist_kernel, bstamp()): steps run T-1 .. 0
        eng._launch("imgcap_lstm_tf_bwd", d, ws)
        torch.cuda.synchronize()
        sb = eng._sync[off:off + 3 * 64 * 16 * 2].view(torch.int64).view(3, 64, 16).cpu().double() * 10.0
        U, X, R = sb[0, 1:T - 1], sb[1, 1:T - 1], sb[2, 1:T - 1]
        nxtU = sb[0, 0:T - 2, 0]  # the next step processed is t - 1
        un = ["cell+publish", "wait dgates", "dgates mma", "wait datt", "datt mma+reduce", "->next"]
        us = [U[:, 1] - U[:, 0], U[:, 2] - U[:, 1], U[:, 3] - U[:, 2], U[:, 4] - U[:, 3], U[:, 5] - U[:, 4],
              nxtU - U[:, 5]]
        print("bwd U block 0, mean ns per step: " + ", ".join(f"{n} {x.mean():.0f}" for n, x in zip(un, us)))
        xn = ["wait dgates", "loads+mma", "reduce+granules"]
        xs = [X[:, 2] - X[:, 0], X[:, 3] - X[:, 2], X[:, 5] - X[:, 3]]
        print("bwd X block 0, mean ns per step: " + ", ".join(f"{n} {x.mean():.0f}" for n, x in zip(xn, xs)))
        rn = ["wait dz", "dawe", "dalpha", "softmax+datt2", "store+publish", "->next"]
        rs = [R[:, 1] - R[:, 0], R[:, 2] - R[:, 1], R[:, 3] - R[:, 2], R[:, 4] - R[:, 3], R[:, 5] - R[:, 4],
              sb[2, 0:T - 2, 0] - R[:, 5]]
        print("bwd R block 0, mean ns per step: " + ", ".join(f"{n} {x.mean():.0f}" for n, x in zip(rn, rs)))
        sn = ["dalpha products", "dalpha reductions", "dalpha barrier", "softmax bwd", "datt2 sums", "barrier",
              "datt2 reduce+barrier"]
        ss = [R[:, 6] - R[:, 2], R[:, 7] - R[:, 6], R[:, 3] - R[:, 7], R[:, 8] - R[:, 3], R[:, 9] - R[:, 8],
              R[:, 10] - R[:, 9], R[:, 4] - R[:, 10]]
        print("bwd R block 0 sub-phases (ns): " + ", ".join(f"{n} {x.mean():.0f}" for n, x in zip(sn, ss)))
        print("bwd cross: U published dgates -> X got %.0f ns, X got -> X done %.0f, R got dz - X done %.0f, "
              "R published -> U got datt %.0f, U done -> next U published %.0f" % (
                  (X[:, 2] - U[:, 1]).mean(), (X[:, 5] - X[:, 2]).mean(), (R[:, 1] - X[:, 5]).mean(),
                  (U[:, 4] - R[:, 5]).mean(), (sb[0, 0:T - 2, 1] - U[:, 5]).mean()))


def misc():
    B = 32
    for (H, C) in ((56, 96), (28, 192), (14, 384), (7, 768)):
        x = torch.randn(B, H, H, C, device=dev).to(bf)
        y = torch.empty_like(x)
        w = torch.randn(49, C, device=dev)
        b = torch.randn(C, device=dev)
        t = time_launch(lambda: K.dwconv7_ln(x, w, b, b, b, y))
        gbs = 2 * x.numel() * 2 / t / 1e9
        print(f"dwconv7_ln B={B} H={H} C={C}: {t * 1e6:8.1f} us {gbs:8.1f} GB/s")
        t = time_launch(lambda: K.dwconv7(x, w, b, y))
        print(f"dwconv7    B={B} H={H} C={C}: {t * 1e6:8.1f} us {2 * x.numel() * 2 / t / 1e9:8.1f} GB/s")
    for rows, cols in ((3328, 512), (1632, 9490), (3328, 1536)):
        x = torch.randn(rows, cols, device=dev).to(bf)
        o = torch.empty(cols, device=dev)
        t = time_launch(lambda: K.colsum(x, o))
        print(f"colsum {rows}x{cols}: {t * 1e6:8.1f} us {x.numel() * 2 / t / 1e9:8.1f} GB/s")
    rows, cols = 3328, 512
    x = torch.randn(rows, cols, device=dev).to(bf)
    g = torch.randn(cols, device=dev)
    s = torch.empty_like(x)
    y, mu, rs = K.add_layernorm(x, x, g, g, 1e-5, s_out=s)
    dg = torch.zeros(cols, device=dev)
    t = time_launch(lambda: K.add_layernorm(x, x, g, g, 1e-5, s_out=s))
    print(f"add_ln fwd {rows}x{cols}: {t * 1e6:8.1f} us")
    t = time_launch(lambda: K.add_layernorm_bwd(x, s, mu, rs, g, dg, dg, dr=y))
    print(f"add_ln bwd {rows}x{cols}: {t * 1e6:8.1f} us")


def small():
    """The Transformer decoder's GEMMs (M = B*L = 3328 at C3, d = ff = 512) under each kernel
    policy: which tile serves latency-bound small grids best."""
    M = 64 * 52
    for (N, Kd, tb) in ((1536, 512, True), (512, 512, True), (512, 512, False), (512, 1536, True), (512, 1536, False)):
        a = torch.randn(M, Kd, device=dev).to(bf)
        w = (torch.randn(N, Kd, device=dev) if tb else torch.randn(Kd, N, device=dev)).to(bf)
        bias = torch.randn(N, device=dev)
        fl = 2.0 * M * N * Kd
        for pol, name in ((-1, "auto"), (4, "glds128"), (5, "tiled"), (6, "glds64"), (8, "tiled64")):
            K.gemm_set_policy(pol)
            t = time_launch(lambda: K.gemm(a, w, trans_b=tb, bias=bias))
            print(f"M={M} N={N} K={Kd} tb={int(tb)} {name:8s}: {t * 1e6:7.1f} us {fl / t / 1e12:6.1f} TF")
        K.gemm_set_policy(-1)
    # larger grids (encoder Linears, LSTM projections): 128x128 vs 64x64 LDS-DMA tiles
    for (M2, N, Kd) in ((12544, 1536, 384), (12544, 384, 1536), (3136, 3072, 768), (3136, 768, 3072),
                        (1632, 2048, 512), (1632, 9490, 512), (6272, 384, 768)):
        a = torch.randn(M2, Kd, device=dev).to(bf)
        w = torch.randn(N, Kd, device=dev).to(bf)
        bias = torch.randn(N, device=dev)
        fl = 2.0 * M2 * N * Kd
        for pol, name in ((-1, "auto"), (4, "glds128"), (6, "glds64")):
            K.gemm_set_policy(pol)
            t = time_launch(lambda: K.gemm(a, w, trans_b=True, bias=bias))
            print(f"M={M2} N={N} K={Kd} tb=1 {name:8s}: {t * 1e6:7.1f} us {fl / t / 1e12:6.1f} TF")
        K.gemm_set_policy(-1)
    # long-K small grids (auto split-K on the 128 tile) vs the unsplit 64 tile; tb=0 = dX form
    for (M2, N, Kd, tb) in ((1568, 768, 3072, True), (3136, 768, 3072, True), (1632, 512, 2048, False),
                            (1632, 512, 9490, False), (3328, 512, 9490, False)):
        kp = (Kd + 7) // 8 * 8  # 16-byte row pitch (the logits' padded vocab rows)
        a = torch.randn(M2, kp, device=dev).to(bf)[:, :Kd]
        w = (torch.randn(N, kp, device=dev).to(bf)[:, :Kd] if tb else torch.randn(Kd, N, device=dev).to(bf))
        fl = 2.0 * M2 * N * Kd
        for pol, name in ((-1, "auto"), (6, "glds64")):
            K.gemm_set_policy(pol)
            t = time_launch(lambda: K.gemm(a, w, trans_b=tb))
            print(f"M={M2} N={N} K={Kd} tb={int(tb)} {name:8s}: {t * 1e6:7.1f} us {fl / t / 1e12:6.1f} TF")
        K.gemm_set_policy(-1)


def mha():
    """Fused attention at the C3 shape (B=64, 8 heads of 64, L=52; self causal + key padding,
    cross over 49 pixels), forward and backward per launch."""
    import ctypes
    from imagecaptioningconvnext_amd import _abi
    B, H, d = 64, 8, 512
    for (Lq, Lk, causal) in ((52, 52, True), (52, 49, False)):
        q, k, v, o, do = (torch.randn(B, L_, d, device=dev).to(bf) for L_ in (Lq, Lk, Lk, Lq, Lq))
        dq, dk, dv = torch.empty_like(q), torch.empty_like(k), torch.empty_like(v)
        lse = torch.empty(B, H, Lq, device=dev)
        ids = torch.randint(1, 50, (B, Lk), device=dev)
        m = _abi.MhaDesc()
        m.dtype, m.B, m.H, m.Lq, m.Lk, m.dh, m.causal, m.pad_id, m.scale = K.dt(q), B, H, Lq, Lk, 64, int(causal), 0, 0.125
        m.ldq = m.ldk = m.ldv = m.ldo = m.lddo = m.lddq = m.lddk = m.lddv = d
        m.q, m.k, m.v, m.o, m.lse = q.data_ptr(), k.data_ptr(), v.data_ptr(), o.data_ptr(), lse.data_ptr()
        m.dout, m.dq, m.dk, m.dv = do.data_ptr(), dq.data_ptr(), dk.data_ptr(), dv.data_ptr()
        m.key_ids = ids.data_ptr() if causal else None
        m.drop_p = 0.5
        tf = time_launch(lambda: _abi.call("imgcap_mha_fwd", ctypes.byref(m), K.stream()))
        tb = time_launch(lambda: _abi.call("imgcap_mha_bwd", ctypes.byref(m), K.stream()))
        print(f"mha Lq={Lq} Lk={Lk} causal={int(causal)}: fwd {tf * 1e6:6.1f} us  bwd {tb * 1e6:6.1f} us")


def mx():
    """MX-FP8 vs bf16 GEMMs at the frozen ConvNeXt-Large stage-3 shapes (C5, B=64)."""
    M, C = 64 * 196, 768
    for (N, Kd) in ((4 * C, C), (C, 4 * C)):
        a = torch.randn(M, Kd, device=dev)
        w = torch.randn(N, Kd, device=dev) / Kd ** 0.5
        ab, wb = a.to(bf), w.to(bf)
        aq, wq = K.mx_quant_rows(a), K.mx_quant_rows(w)
        fl = 2.0 * M * N * Kd
        t = time_launch(lambda: K.gemm(ab, wb, trans_b=True))
        print(f"bf16 gemm M={M} N={N} K={Kd}: {t * 1e6:7.1f} us {fl / t / 1e12:7.1f} TF")
        t = time_launch(lambda: K.gemm_mx(aq, wq))
        print(f"mx   gemm M={M} N={N} K={Kd}: {t * 1e6:7.1f} us {fl / t / 1e12:7.1f} TF (bf16 out)")
        t = time_launch(lambda: K.gemm_mx(aq, wq, act=K.ACT_GELU))
        print(f"mx   gemm M={M} N={N} K={Kd}: {t * 1e6:7.1f} us {fl / t / 1e12:7.1f} TF (GELU + bf16 out)")
        t = time_launch(lambda: K.gemm_mx(aq, wq, out_dtype="mx"))
        print(f"mx   gemm M={M} N={N} K={Kd}: {t * 1e6:7.1f} us {fl / t / 1e12:7.1f} TF (MX out)")
        t = time_launch(lambda: K.gemm_mx(aq, wq, act=K.ACT_GELU, out_dtype="mx"))
        print(f"mx   gemm M={M} N={N} K={Kd}: {t * 1e6:7.1f} us {fl / t / 1e12:7.1f} TF (GELU + MX out)")
    x = torch.randn(M, C, device=dev).to(bf)
    g = torch.ones(C, device=dev)
    t = time_launch(lambda: K.mx_quant_rows(x, g, g))
    print(f"mx_quant_rows+LN {M}x{C}: {t * 1e6:7.1f} us {M * C * 3 / t / 1e9:7.1f} GB/s")


def dw():
    """depthwise 7x7 at the C5 (Large, B=64) and C3 (Tiny, B=64) stage shapes: HBM GB/s and
    the fp32-VALU floor (49 FMA per output element at 256 CUs x 128 FMA/clk x 2.4 GHz)."""
    B = 64
    for C0 in (96, 192):
        for s, H in enumerate((56, 28, 14, 7)):
            C = C0 << s
            x = torch.randn(B, H, H, C, device=dev).to(bf)
            y = torch.empty_like(x)
            w = torch.randn(49, C, device=dev)
            b = torch.randn(C, device=dev)
            t = time_launch(lambda: K.dwconv7(x, w, b, y))
            floor = x.numel() * 49 / (256 * 128 * 2.4e9)
            print(f"dwconv7 B={B} H={H:2d} C={C:4d}: {t * 1e6:7.1f} us {2 * x.numel() * 2 / t / 1e9:7.1f} GB/s"
                  f"  hbm floor {2 * x.numel() * 2 / 8e12 * 1e6:5.1f} us  valu floor {floor * 1e6:5.1f} us")


if __name__ == "__main__":
    which = sys.argv[1] if len(sys.argv) > 1 else "all"
    if which == "dw":
        dw()
    if which == "mx":
        mx()
    if which == "small":
        small()
    if which == "mha":
        mha()
    if which in ("all", "gemm"):
        gemms()
    if which == "probe":
        gemm_probe()
    if which in ("all", "misc"):
        misc()
    if which in ("all", "mlp"):
        mlp()
    if which in ("all", "lstm"):
        lstm()
    if which == "mlpdw":  # short run for PMC collection: s1 shapes only
        B, H, C = 32, 56, 96
        x = torch.randn(B, H, H, C, device=dev).to(bf)
        y = torch.empty_like(x)
        w = torch.randn(49, C, device=dev)
        b = torch.randn(C, device=dev)
        for _ in range(5):
            K.dwconv7(x, w, b, y)
        torch.cuda.synchronize()


def overlap():
    """LSTM recurrence (fwd + bwd) and the frozen Tiny encoder forward (B=32), alone and on two
    streams captured into one graph: how much of the encoder hides under the recurrence."""
    import ctypes
    from imagecaptioningconvnext_amd import _abi
    from imagecaptioningconvnext_amd.models.decoder import DecoderWithAttention
    from imagecaptioningconvnext_amd.models.encoder import Encoder
    B, L, V = int(os.environ.get("IMGCAP_MB_B", "32")), 52, 9490
    dec = DecoderWithAttention(attention_dim=512, embed_dim=512, decoder_dim=512, vocab_size=V, device=dev,
                               encoder_dim=768, dropout=0.5, compute_dtype=bf).to(dev)
    enc = Encoder(variant="tiny", compute_dtype=bf).to(dev)
    enc.fine_tune(False)
    enc.train()
    img = torch.randn(B, 3, 224, 224, device=dev)
    eng = dec.engine()
    feats = torch.randn(B, 7, 7, 768, device=dev).to(bf)
    caps = torch.randint(1, V - 3, (B, L), device=dev)
    lens = torch.full((B, 1), L, device=dev, dtype=torch.long)
    s = eng.forward(feats, caps, lens, fixed_T=True)
    eng.backward(s)
    d = s["desc"]
    ws = s["bwd_bufs"]["chain_ws"]

    def rec():
        eng._launch("imgcap_lstm_tf_fwd", d)
        eng._launch("imgcap_lstm_tf_bwd", d, ws)

    def encf():
        with torch.no_grad():
            enc(img)
    side = torch.cuda.Stream()
    hi = torch.cuda.Stream(priority=-1)

    def both(main=None):
        cur = torch.cuda.current_stream()
        side.wait_stream(cur)
        with torch.cuda.stream(side):
            encf()
        rec()
        cur.wait_stream(side)
    t_r = time_launch(rec, reps=3, warm=1)
    t_e = time_launch(encf, reps=3, warm=1)
    t_b = time_launch(both, reps=3, warm=1)
    print(f"overlap: recurrence {t_r * 1e6:.0f} us, encoder {t_e * 1e6:.0f} us, sum {(t_r + t_e) * 1e6:.0f} us, "
          f"two streams {t_b * 1e6:.0f} us")
    with torch.cuda.stream(hi):
        t_h = time_launch(both, reps=3, warm=1)
    print(f"overlap (recurrence on a high-priority stream): {t_h * 1e6:.0f} us")

    def both_rev():  # recurrence captured first, encoder second (graph node order)
        cur = torch.cuda.current_stream()
        side.wait_stream(cur)
        rec()
        with torch.cuda.stream(side):
            encf()
        cur.wait_stream(side)
    t = time_launch(both_rev, reps=3, warm=1)
    print(f"overlap (recurrence captured first): {t * 1e6:.0f} us")
    t = time_launch(both, reps=3, warm=1, graph=False)
    print(f"overlap (eager, no graph): {t * 1e6:.0f} us")

    def interleaved():  # encoder stages captured between the recurrence halves
        cur = torch.cuda.current_stream()
        side.wait_stream(cur)
        eng._launch("imgcap_lstm_tf_fwd", d)
        with torch.cuda.stream(side):
            encf()
        eng._launch("imgcap_lstm_tf_bwd", d, ws)
        cur.wait_stream(side)
    t = time_launch(interleaved, reps=3, warm=1)
    print(f"overlap (encoder captured between fwd and bwd recurrence): {t * 1e6:.0f} us")
    ge, gr = torch.cuda.CUDAGraph(), torch.cuda.CUDAGraph()
    side.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(side):
        with torch.cuda.graph(ge, stream=side):
            encf()
    with torch.cuda.graph(gr):
        rec()
    torch.cuda.synchronize()

    def two_graphs(order):
        cur = torch.cuda.current_stream()
        side.wait_stream(cur)
        for o in order:
            if o == "e":
                with torch.cuda.stream(side):
                    ge.replay()
            else:
                gr.replay()
        cur.wait_stream(side)
    for order in ("er", "re"):
        two_graphs(order)
        torch.cuda.synchronize()
        t = time_launch(lambda: two_graphs(order), reps=3, warm=1, graph=False)
        print(f"overlap (two graphs, launch order {order}): {t * 1e6:.0f} us")


def cu_stream(n_cus, first=0, total=256):
    """A HIP stream whose kernels may only use CUs [first, first + n_cus) of the mask numbering
    (hipExtStreamCreateWithCUMask), wrapped for torch."""
    import ctypes
    hip = ctypes.CDLL("libamdhip64.so")
    words = (ctypes.c_uint32 * (total // 32))()
    for i in range(first, first + n_cus):
        words[i // 32] |= 1 << (i % 32)
    st = ctypes.c_void_p()
    rc = hip.hipExtStreamCreateWithCUMask(ctypes.byref(st), ctypes.c_uint32(total // 32), words)
    assert rc == 0, rc
    return torch.cuda.ExternalStream(st.value)


def cumask():
    """Encoder on a CU-masked stream beside the LSTM recurrence: the recurrence's small grids
    keep the CUs the encoder may not use."""
    from imagecaptioningconvnext_amd.models.decoder import DecoderWithAttention
    from imagecaptioningconvnext_amd.models.encoder import Encoder
    B, L, V = int(os.environ.get("IMGCAP_MB_B", "32")), 52, 9490
    dec = DecoderWithAttention(attention_dim=512, embed_dim=512, decoder_dim=512, vocab_size=V, device=dev,
                               encoder_dim=768, dropout=0.5, compute_dtype=bf).to(dev)
    enc = Encoder(variant="tiny", compute_dtype=bf).to(dev)
    enc.fine_tune(False)
    enc.train()
    img = torch.randn(B, 3, 224, 224, device=dev)
    eng = dec.engine()
    feats = torch.randn(B, 7, 7, 768, device=dev).to(bf)
    caps = torch.randint(1, V - 3, (B, L), device=dev)
    lens = torch.full((B, 1), L, device=dev, dtype=torch.long)
    s = eng.forward(feats, caps, lens, fixed_T=True)
    eng.backward(s)
    d = s["desc"]
    ws = s["bwd_bufs"]["chain_ws"]

    def rec():
        eng._launch("imgcap_lstm_tf_fwd", d)
        eng._launch("imgcap_lstm_tf_bwd", d, ws)

    def encf():
        with torch.no_grad():
            enc(img)
    t_r = time_launch(rec, reps=3, warm=1)
    print(f"recurrence alone {t_r * 1e6:.0f} us")
    # graphs replay their nodes on the launch stream (single-branch graphs), so a CU mask on the
    # replay stream applies: the encoder graph on a masked stream, the recurrence graph beside it
    encf()
    torch.cuda.synchronize()
    plain = torch.cuda.Stream()
    ge, gr = torch.cuda.CUDAGraph(), torch.cuda.CUDAGraph()
    plain.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(plain):
        with torch.cuda.graph(ge, stream=plain):
            encf()
        with torch.cuda.graph(gr, stream=plain):
            rec()
    torch.cuda.synchronize()
    main = torch.cuda.current_stream()
    for n in (256, 224, 192, 160, 128):
        se = cu_stream(n)
        for rmask in ((None, "all") if n == 256 else (None, "all", "rest")):
            sr = main if rmask in (None, "all") else cu_stream(256 - n, first=n)

            def both():
                se.wait_stream(main)
                sr.wait_stream(main)
                with torch.cuda.stream(se):
                    ge.replay()
                with torch.cuda.stream(sr):
                    gr.replay()
                main.wait_stream(se)
                main.wait_stream(sr)
            if rmask is None:
                def enc_only():
                    se.wait_stream(main)
                    with torch.cuda.stream(se):
                        ge.replay()
                    main.wait_stream(se)
                t = time_launch(enc_only, reps=3, warm=1, graph=False)
                print(f"encoder graph on {n} CUs alone: {t * 1e6:.0f} us")
                continue
            t = time_launch(both, reps=3, warm=1, graph=False)
            print(f"encoder graph on {n} CUs + recurrence graph on {rmask}: {t * 1e6:.0f} us")


if __name__ == "__main__" and len(sys.argv) > 1 and sys.argv[1] == "overlap":
    overlap()
if __name__ == "__main__" and len(sys.argv) > 1 and sys.argv[1] == "cumask":
    cumask()

"""Tensor-level wrappers over the C ABI (device pointers + current HIP stream).

All functions enqueue on ``torch.cuda.current_stream()``; none allocates unless it is asked to
return a fresh output.  Inputs must already live on the GPU; there is no CPU path.
"""
import ctypes
import os

import torch

from . import _abi
from ._abi import ACT_DGELU, ACT_GELU, ACT_NONE, ACT_RELU, BF16, F32, GEMM_PT, GEMM_WS, GEMM_WS4, Epilogue  # noqa: F401

_DT = {torch.float32: F32, torch.bfloat16: BF16}


def dt(t):
    try:
        return _DT[t.dtype]
    except KeyError:
        raise TypeError(f"unsupported dtype {t.dtype}") from None


def ptr(t):
    return None if t is None else t.data_ptr()


def stream():
    return torch.cuda.current_stream().cuda_stream


def _check_dev(*ts):
    for t in ts:
        if t is not None and not t.is_cuda:
            raise RuntimeError("imgcap kernels need GPU tensors (no CPU fallback)")


def _ld(t, trans):
    """Leading dimension of a 2-D operand view whose innermost stride is 1."""
    if t.stride(-1) != 1:
        raise ValueError("operand must have unit inner stride")
    return t.stride(-2) if t.dim() >= 2 else t.shape[-1]


_gemm_recorder = None


def record_gemms(recorder):
    """Collect every ``gemm`` call (a replayable closure + its shape) into ``recorder`` (a list),
    or stop with None.  Used by the bench's roofline to re-time the step's GEMMs in isolation."""
    global _gemm_recorder
    _gemm_recorder = recorder


_cur_slot = [0]


class workspace_slot:
    """Context manager: library scratch slot for work that runs beside slot-0 work on another
    stream (imgcap_workspace_slot): 1 the trainer's pipelined encoder branch, 2 the decoder
    engines' side streams.  Restores the slot it found."""

    def __init__(self, slot=1):
        self.slot = slot

    def __enter__(self):
        self.prev = _cur_slot[0]
        _abi.call("imgcap_workspace_slot", self.slot)
        _cur_slot[0] = self.slot

    def __exit__(self, *a):
        _abi.call("imgcap_workspace_slot", self.prev)
        _cur_slot[0] = self.prev


# ---- stream forks inside captured steps --------------------------------------------------------
# A side stream forked from the capturing stream must be joined back before capture_end: an
# un-joined branch leaves the graph without its tail (round 5 saw a host segfault inside the
# runtime's capture_end in a variant that swapped the two branches' streams).  The
# engines and the trainer fork and join through these two calls, and the trainer asserts before
# every capture_end that nothing forked is still open.
_open_forks = {}


def fork(side, src):
    """``side`` waits for ``src``'s work so far and is recorded as an open branch.  A branch forked
    from a stream that is itself an open branch is refused: inside a HIP graph capture that nesting
    (M -> S -> X, X joined to S, S to M) crashes hipStreamEndCapture with a segfault on ROCm 7.2
    (tools/probe/capture_refork.py "nested"), so every fork starts from a stream that
    is not a branch.  Checked in eager runs too: the engines run the same code eagerly first."""
    if src.cuda_stream in _open_forks and src.cuda_stream != side.cuda_stream:
        raise RuntimeError(f"stream {hex(src.cuda_stream)} is an open branch: forking {hex(side.cuda_stream)} from "
                           "it would nest branches, which crashes HIP graph capture (DESIGN §2b)")
    side.wait_stream(src)
    _open_forks[side.cuda_stream] = side


def join(dst, side, event=None):
    """``dst`` waits for ``side`` (for ``event``, which the caller recorded as side's LAST work of
    the branch); the branch is closed."""
    if event is None:
        dst.wait_stream(side)
    else:
        dst.wait_event(event)
    _open_forks.pop(side.cuda_stream, None)


def assert_joined(where):
    if _open_forks:
        names = ", ".join(hex(k) for k in _open_forks)
        _open_forks.clear()
        raise RuntimeError(f"{where}: side stream(s) {names} forked inside the capture and never joined")


def gemm_set_policy(glds256):
    """-1 by shape (default), 0 never, 1 always use the 256x256 GEMM tile where eligible."""
    _abi.call("imgcap_gemm_set_policy", int(glds256))


def gemm_set_pt(mode):
    """Stream-tile GEMM (imgcap_gemm_set_pt): -1 by shape (the library default), 0 never, 1
    wherever eligible (cost-model tile), 2..7 wherever eligible with tile 256x128 / 128x256 /
    128x128 / 128x192 / 128x128 (4 waves, two blocks a CU) / 128x128 (128-deep k-steps)."""
    _abi.call("imgcap_gemm_set_pt", int(mode))


def gemm_get_pt():
    """The stream-tile policy currently set (imgcap_gemm_get_pt)."""
    return int(_abi.lib().imgcap_gemm_get_pt())


def gemm_set_ws(mode):
    """Weight-stationary short-K GEMM (imgcap_gemm_set_ws): -1 by shape, 0 never, 1 / 2 wherever
    eligible with 8- / 4-wave blocks."""
    _abi.call("imgcap_gemm_set_ws", int(mode))


def gemm_get_ws():
    return int(_abi.lib().imgcap_gemm_get_ws())


class gemm_ws_mode:
    """``with gemm_ws_mode(m):`` -- the weight-stationary policy m inside, the previous one after."""

    def __init__(self, mode):
        self.mode = mode

    def __enter__(self):
        self.prev = gemm_get_ws()
        gemm_set_ws(self.mode)

    def __exit__(self, *a):
        gemm_set_ws(self.prev)


class gemm_pt_mode:
    """``with gemm_pt_mode(m):`` -- the stream-tile policy m inside, the previous one restored after
    (tests and tools: a hard-coded reset would change the library default for later callers)."""

    def __init__(self, mode):
        self.mode = mode

    def __enter__(self):
        self.prev = gemm_get_pt()
        gemm_set_pt(self.mode)

    def __exit__(self, *a):
        gemm_set_pt(self.prev)


def gemm_plan(dtype, a_kmajor, b_kmajor, M, N, K, lda, ldb, batch=1, split_k=0, ep=None):
    """(kernel kind, K slices) imgcap_gemm picks for these operands (IMGCAP_GEMM_* ids); with the
    call's Epilogue ``ep`` the persistent-tile kernel's eligibility is known too."""
    sp = ctypes.c_int(1)
    if ep is not None:
        kind = _abi.lib().imgcap_gemm_plan_ep(dtype, a_kmajor, b_kmajor, M, N, K, lda, ldb, batch, ctypes.byref(ep),
                                              ctypes.byref(sp))
    else:
        kind = _abi.lib().imgcap_gemm_plan(dtype, a_kmajor, b_kmajor, M, N, K, lda, ldb, batch, split_k,
                                           ctypes.byref(sp))
    return kind, sp.value


def gemm(a, b, *, trans_a=False, trans_b=False, out=None, out_dtype=None, bias=None, act=ACT_NONE, alpha=1.0,
         beta=0.0, res=None, aux=None, aux_scale=1.0, colscale=None, rowscale=None, rows_per_scale=1, drop_p=0.0,
         seed=0, drop_stream=0, drop_ld=None, M=None, N=None, K=None, split_k=0):
    """out[M,N] = epilogue(op(a) @ op(b)); op(x) = x.T if trans else x (torch semantics).

    ``a``/``b`` are 2-D views (unit inner stride).  With trans_b=True, b is an nn.Linear
    weight [N, K] and the call is ``a @ b.T``.  split_k (-1 = auto) slices K across the grid
    for long-K fp32 products ``out = alpha * a @ b + beta * out`` (no other epilogue).
    """
    _check_dev(a, b, out, bias, res, aux)
    if a.dtype != b.dtype:
        raise TypeError("a and b must share dtype")
    if M is None:
        M = a.shape[1] if trans_a else a.shape[0]
    if K is None:
        K = a.shape[0] if trans_a else a.shape[1]
    if N is None:
        N = b.shape[0] if trans_b else b.shape[1]
    kb = b.shape[1] if trans_b else b.shape[0]
    if kb != K:
        raise ValueError(f"gemm: K mismatch {K} vs {kb}")
    if out is None:
        out = torch.empty((M, N), device=a.device, dtype=out_dtype or a.dtype)
    ep = Epilogue()
    ep.bias = ptr(bias)
    ep.colscale = ptr(colscale)
    ep.rowscale = ptr(rowscale)
    ep.rows_per_scale = rows_per_scale
    ep.res = ptr(res)
    ep.ldr = 0 if res is None else res.stride(0)
    ep.aux = ptr(aux)
    ep.ldaux = 0 if aux is None else aux.stride(0)
    ep.aux_scale = aux_scale
    ep.alpha = alpha
    ep.beta = beta
    ep.act = act
    ep.c_dtype = dt(out)
    ep.drop_p = drop_p
    ep.seed = seed
    ep.drop_stream = drop_stream
    ep.drop_ld = N if drop_ld is None else drop_ld
    ep.split_k = split_k
    args = (dt(a), 0 if trans_a else 1, 1 if trans_b else 0, M, N, K, a.data_ptr(), _ld(a, trans_a), 0, b.data_ptr(),
            _ld(b, trans_b), 0, out.data_ptr(), out.stride(0), 0, 1)
    if _gemm_recorder is not None:
        keep = (a, b, out, bias, res, aux, colscale, rowscale, ep)
        _gemm_recorder.append(dict(M=M, N=N, K=K, dtype=args[0], ak=args[1], bk=args[2], lda=args[7], ldb=args[10],
                                   split_k=split_k, keep=keep,
                                   call=lambda: _abi.call("imgcap_gemm", *args, ctypes.byref(ep), stream())))
    _abi.call("imgcap_gemm", *args, ctypes.byref(ep), stream())
    return out


def mx_quant_rows(x, ln_w=None, ln_b=None, eps=1e-6, out=None):
    """Rows of x [R, K] (bf16 / fp32), LayerNorm'd first when ln_w/ln_b are given, to MX-FP8:
    (q [R, K] uint8 e4m3fn bytes, s [R, K/32] uint8 E8M0 scales)."""
    _check_dev(x, ln_w, ln_b)
    R, Kc = x.shape
    if out is None:
        out = (torch.empty(R, Kc, device=x.device, dtype=torch.uint8),
               torch.empty(R, Kc // 32, device=x.device, dtype=torch.uint8))
    q, sc = out
    _abi.call("imgcap_mx_quant_rows", dt(x), R, Kc, x.data_ptr(), x.stride(0), ptr(ln_w), ptr(ln_b), eps,
              q.data_ptr(), sc.data_ptr(), stream())
    return q, sc


def mx_dequant(q, sc):
    """MX-FP8 (q, scales) -> fp32 (test / diagnostics helper, torch ops)."""
    v = q.view(torch.float8_e4m3fn).float()
    e = (sc.to(torch.int32) - 127).float()
    return (v.view(q.shape[0], -1, 32) * torch.exp2(e).unsqueeze(-1)).view(q.shape)


def gemm_mx(a, b, *, out=None, out_dtype=torch.bfloat16, bias=None, act=ACT_NONE, colscale=None, rowscale=None,
            rows_per_scale=1, res=None):
    """epilogue(A @ B^T) on block-scaled fp8 operands: ``a`` = (q [M, K], s [M, K/32]), ``b`` =
    (q [N, K], s [N, K/32]) as mx_quant_rows returns them (b: an nn.Linear weight).  out_dtype
    "mx" returns the product itself in MX-FP8 (q, s) -- the next GEMM's A operand."""
    (aq, as_), (bq, bs) = a, b
    _check_dev(aq, bq, bias, res, colscale, rowscale)
    M, Kc = aq.shape
    N = bq.shape[0]
    if bq.shape[1] != Kc:
        raise ValueError(f"gemm_mx: K mismatch {Kc} vs {bq.shape[1]}")
    mx = out_dtype == "mx"
    if out is None:
        out = ((torch.empty(M, N, device=aq.device, dtype=torch.uint8),
                torch.empty(M, N // 32, device=aq.device, dtype=torch.uint8)) if mx else
               torch.empty(M, N, device=aq.device, dtype=out_dtype))
    ep = Epilogue()
    ep.bias = ptr(bias)
    ep.colscale = ptr(colscale)
    ep.rowscale = ptr(rowscale)
    ep.rows_per_scale = rows_per_scale
    ep.res = ptr(res)
    ep.ldr = 0 if res is None else res.stride(0)
    ep.alpha = 1.0
    ep.act = act
    if mx:
        oq, osc = out
        ep.c_dtype = _abi.FP8MX
        ep.c_scale = osc.data_ptr()
        cptr, ldc = oq.data_ptr(), oq.stride(0)
    else:
        ep.c_dtype = dt(out)
        cptr, ldc = out.data_ptr(), out.stride(0)
    args = (M, N, Kc, aq.data_ptr(), aq.stride(0), as_.data_ptr(), bq.data_ptr(), bq.stride(0), bs.data_ptr(), cptr,
            ldc)
    if _gemm_recorder is not None:
        keep = (aq, as_, bq, bs, out, bias, res, colscale, rowscale, ep)
        _gemm_recorder.append(dict(M=M, N=N, K=Kc, mx=True, keep=keep,
                                   call=lambda: _abi.call("imgcap_gemm_mx", *args, ctypes.byref(ep), stream())))
    _abi.call("imgcap_gemm_mx", *args, ctypes.byref(ep), stream())
    return out


def gemm_raw(dtype, a_kmajor, b_kmajor, M, N, K, A, lda, B, ldb, C, ldc, c_dtype, *, batch=1, sA=0, sB=0, sC=0,
             bias=None, act=ACT_NONE, alpha=1.0, beta=0.0, rowscale=None, rows_per_scale=1, drop_p=0.0, seed=0,
             drop_stream=0, drop_ld=0, split_k=0):
    """Pointer-level GEMM for strided / batched operand views."""
    ep = Epilogue()
    ep.bias = bias
    ep.rowscale = rowscale
    ep.rows_per_scale = rows_per_scale
    ep.alpha = alpha
    ep.beta = beta
    ep.act = act
    ep.c_dtype = c_dtype
    ep.drop_p = drop_p
    ep.seed = seed
    ep.drop_stream = drop_stream
    ep.drop_ld = drop_ld
    ep.split_k = split_k
    _abi.call("imgcap_gemm", dtype, a_kmajor, b_kmajor, M, N, K, A, lda, sA, B, ldb, sB, C, ldc, sC, batch,
              ctypes.byref(ep), stream())


def colsum(x, out, beta=0.0, rows=None, cols=None, ld=None):
    rows = x.shape[0] if rows is None else rows
    cols = x.shape[1] if cols is None else cols
    _abi.call("imgcap_colsum", dt(x), rows, cols, x.data_ptr(), x.stride(0) if ld is None else ld, out.data_ptr(),
              beta, stream())
    return out


class ColsumBatch:
    """Deferred bias gradients: ``add`` records colsum(x) -> out (x kept alive), ``run`` issues
    them as ONE imgcap_colsum_multi call per 48 items (instead of 1-2 launches each)."""

    def __init__(self):
        self.items = []

    def add(self, x, out, cols=None, rows=None, ld=None, beta=0.0):
        _check_dev(x, out)
        self.items.append((x, out, x.shape[0] if rows is None else rows, x.shape[1] if cols is None else cols,
                           x.stride(0) if ld is None else ld, beta))

    # two launches over 256-row chunks with the partials in a torch-allocated buffer (the
    # default: C3's 80 bias sums, 302 MB, in 76 us vs 95 us single-pass); IMGCAP_COLSUM=1 runs the
    # single-pass kernel.  Neither takes library scratch (tests/test_stream_hazards_gpu.py).
    TWO_PASS = os.environ.get("IMGCAP_COLSUM", "2") == "2"

    def run(self):
        for i0 in range(0, len(self.items), 48):
            chunk = self.items[i0:i0 + 48]
            arr = (_abi.ColsumItem * len(chunk))()
            for a, (x, out, rows, cols, ld, beta) in zip(arr, chunk):
                a.x, a.out, a.ld, a.rows, a.cols, a.dtype, a.beta = x.data_ptr(), out.data_ptr(), ld, rows, cols, \
                    dt(x), beta
            if self.TWO_PASS:
                n = sum((rows + 255) // 256 * cols for (_, _, rows, cols, _, _) in chunk)
                part = torch.empty(max(n, 1), device=chunk[0][1].device, dtype=torch.float32)
                _abi.call("imgcap_colsum_multi_part", len(chunk), ctypes.cast(arr, ctypes.c_void_p), part.data_ptr(),
                          n, stream())
            else:
                _abi.call("imgcap_colsum_multi", len(chunk), ctypes.cast(arr, ctypes.c_void_p), stream())
        self.items = []


class GemmBatch:
    """Deferred weight gradients: ``add(a, b, out, trans_a=, trans_b=)`` records the fp32 product
    out = alpha * op(a) op(b) + beta * out (operands kept alive); ``run`` issues all of them as
    grouped launches (imgcap_gemm_grouped, one per operand layout and 48 problems) -- hundreds of
    128x128 tiles in one grid instead of a small split-K grid + reduce per product."""

    def __init__(self):
        self.items = {}

    def add(self, a, b, out, *, trans_a=False, trans_b=False, M=None, N=None, K=None, alpha=1.0, beta=0.0):
        _check_dev(a, b, out)
        if a.dtype != torch.bfloat16 or b.dtype != torch.bfloat16 or out.dtype != torch.float32:
            gemm(a, b, trans_a=trans_a, trans_b=trans_b, out=out, M=M, N=N, K=K, alpha=alpha, beta=beta, split_k=-1)
            return
        M = (a.shape[1] if trans_a else a.shape[0]) if M is None else M
        K = (a.shape[0] if trans_a else a.shape[1]) if K is None else K
        N = (b.shape[0] if trans_b else b.shape[1]) if N is None else N
        key = (0 if trans_a else 1, 1 if trans_b else 0)
        self.items.setdefault(key, []).append((a, b, out, M, N, K, _ld(a, trans_a), _ld(b, trans_b), alpha, beta))

    def run(self):
        for (ak, bk), lst in self.items.items():
            for i0 in range(0, len(lst), 48):
                chunk = lst[i0:i0 + 48]
                arr = (_abi.GemmProblem * len(chunk))()
                for p, (a, b, out, M, N, K, lda, ldb, alpha, beta) in zip(arr, chunk):
                    p.A, p.B, p.C = a.data_ptr(), b.data_ptr(), out.data_ptr()
                    p.lda, p.ldb, p.ldc = lda, ldb, out.stride(0)
                    p.M, p.N, p.K, p.alpha, p.beta = M, N, K, alpha, beta
                _abi.call("imgcap_gemm_grouped", ak, bk, len(chunk), ctypes.cast(arr, ctypes.c_void_p), stream())
        self.items = {}


def add_layernorm(x, r, gamma, beta, eps, *, drop_p=0.0, seed=0, drop_stream=0, s_out=None, y=None):
    rows, cols = x.shape
    y = torch.empty_like(x) if y is None else y
    mean = torch.empty(rows, device=x.device, dtype=torch.float32)
    rstd = torch.empty_like(mean)
    _abi.call("imgcap_add_layernorm_fwd", dt(x), rows, cols, x.data_ptr(), ptr(r), drop_p, seed, drop_stream,
              gamma.data_ptr(), beta.data_ptr(), eps, ptr(s_out), y.data_ptr(), mean.data_ptr(), rstd.data_ptr(),
              stream())
    return y, mean, rstd


def add_layernorm_bwd(dy, s, mean, rstd, gamma, dgamma, dbeta, *, drop_p=0.0, seed=0, drop_stream=0, dx=None,
                      dr=None, cb=None):
    """LN backward; dgamma/dbeta accumulate (+=).  With a ColsumBatch ``cb`` their column sums
    are deferred to cb.run(): the kernel leaves its per-block partials [nblk, 2, cols] (fp32,
    ~1/8 of the rows at C3) and cb sums them."""
    rows, cols = dy.shape
    dx = torch.empty_like(dy) if dx is None else dx
    part = None
    if cb is not None:
        nblk = _abi.lib().imgcap_add_layernorm_bwd_blocks(rows)
        part = torch.empty(nblk, 2, cols, device=dy.device, dtype=torch.float32)
        cb.add(part[:, 0], dgamma, beta=1.0)
        cb.add(part[:, 1], dbeta, beta=1.0)
        dgamma = dbeta = None
    _abi.call("imgcap_add_layernorm_bwd", dt(dy), rows, cols, dy.data_ptr(), s.data_ptr(), mean.data_ptr(),
              rstd.data_ptr(), gamma.data_ptr(), drop_p, seed, drop_stream, dx.data_ptr(), ptr(dr), ptr(dgamma),
              ptr(dbeta), ptr(part), stream())
    return dx


def ce_fwd(logits, targets, V, lse, loss, hit5):
    n = targets.numel()
    _abi.call("imgcap_ce_fwd", dt(logits), n, V, logits.data_ptr(), logits.stride(0), targets.data_ptr(),
              lse.data_ptr(), ptr(loss), ptr(hit5), stream())


def ce_bwd(logits, targets, V, lse, scale, dlogits):
    n = targets.numel()
    _abi.call("imgcap_ce_bwd", dt(logits), n, V, logits.data_ptr(), logits.stride(0), targets.data_ptr(),
              lse.data_ptr(), scale.data_ptr(), dlogits.data_ptr(), dlogits.stride(0), stream())


def ce_fused(logits, targets, V, scale, lse, loss, hit5, dlogits):
    """Training-step CE in one pass: scale[0] = 1/tokens, lse/loss/hit5, dlogits (imgcap_ce_fused)."""
    n = targets.numel()
    _abi.call("imgcap_ce_fused", dt(logits), n, V, logits.data_ptr(), logits.stride(0), targets.data_ptr(),
              scale.data_ptr(), lse.data_ptr(), ptr(loss), ptr(hit5), dlogits.data_ptr(), dlogits.stride(0), stream())


def ce_fused_fits(logits, dlogits, V):
    """Whether imgcap_ce_fused takes these rows (its per-lane register row: V <= 24576 in bf16,
    12288 in fp32; 16-byte aligned rows whose pitch covers the vectorised row)."""
    vec = 8 if logits.dtype == torch.bfloat16 else 4
    nvec = (V + vec - 1) // vec
    return ((nvec + 255) // 256 <= 12 and logits.stride(0) % vec == 0 and dlogits.stride(0) % vec == 0
            and dlogits.stride(0) >= nvec * vec and logits.data_ptr() % 16 == 0 and dlogits.data_ptr() % 16 == 0)


def ce_train(logits, targets, V, metrics, lse, loss, hit5, dlogits, finalize):
    """Training-step CE (train.py:266-276): loss rows, top-5 hits, metrics (via ``finalize``, the
    caller's loss_finalize launch) and dlogits = (softmax - onehot) / tokens.  One fused pass over
    the logits when imgcap_ce_fused takes the rows, else ce_fwd -> finalize -> ce_bwd (the scale
    1/tokens is metrics[3], written by loss_finalize)."""
    if ce_fused_fits(logits, dlogits, V):
        ce_fused(logits, targets, V, metrics[3:4], lse, loss, hit5, dlogits)
        finalize()
    else:
        ce_fwd(logits, targets, V, lse, loss, hit5)
        finalize()
        ce_bwd(logits, targets, V, lse, metrics[3:4], dlogits)


def loss_finalize(loss_rows, hit5, targets, extra, out):
    _abi.call("imgcap_loss_finalize", targets.numel(), loss_rows.data_ptr(), hit5.data_ptr(), targets.data_ptr(),
              ptr(extra), out.data_ptr(), stream())


def clamp_adam(param, grad, m, v, shadow, lr, step, clip, grad_div=1.0, betas=(0.9, 0.999), eps=1e-8, skip=None):
    """skip: optional device fp32 word; a nonzero value at run time leaves every buffer as it was."""
    _abi.call("imgcap_clamp_adam", param.numel(), param.data_ptr(), grad.data_ptr(), m.data_ptr(), v.data_ptr(),
              ptr(shadow), lr, betas[0], betas[1], eps, step, clip if clip is not None else 3.4e38, grad_div,
              ptr(skip), stream())


def greedy_select(logits, V, t, end_id, finished, next_ids, sequences, predictions, alpha=None, alphas=None):
    """One greedy step over the unfinished rows (imgcap_greedy_select)."""
    B = logits.shape[0]
    maxlen = sequences.shape[1]
    _abi.call("imgcap_greedy_select", dt(logits), B, V, logits.data_ptr(), logits.stride(0), t, maxlen, end_id,
              finished.data_ptr(), next_ids.data_ptr(), sequences.data_ptr(), predictions.data_ptr(), ptr(alpha),
              ptr(alphas), 0 if alpha is None else alpha.shape[1], stream())


def embedding_fwd(ids, table, out, *, pe=None, L=1, drop_p=0.0, seed=0, drop_stream=0):
    _abi.call("imgcap_embedding_fwd", dt(out), ids.numel(), table.shape[1], ids.data_ptr(), table.data_ptr(),
              ptr(pe), L, drop_p, seed, drop_stream, out.data_ptr(), stream())
    return out


def tf_targets(caps, lens, n_metrics=5):
    """(tmask [B, L] bool, targets [B*L] int64, zeroed metrics [n_metrics] fp32) of a caption batch
    in one launch (imgcap_tf_targets): position l's target is caps[:, l+1] where l < len - 1, else -1."""
    _check_dev(caps, lens)
    if caps.dtype != torch.int64 or lens.dtype != torch.int64:
        raise TypeError("tf_targets: caps and lens must be int64")
    B, L = caps.shape
    caps = caps.contiguous()
    lens = lens.reshape(-1).contiguous()
    if lens.numel() != B:
        raise ValueError("tf_targets: one length per caption")
    tmask = torch.empty(B, L, device=caps.device, dtype=torch.bool)
    targets = torch.empty(B * L, device=caps.device, dtype=torch.int64)
    metrics = torch.empty(n_metrics, device=caps.device, dtype=torch.float32)
    _abi.call("imgcap_tf_targets", B, L, caps.data_ptr(), lens.data_ptr(), tmask.data_ptr(), targets.data_ptr(),
              metrics.data_ptr(), n_metrics, stream())
    return tmask, targets, metrics


def embedding_bwd(ids, dout, dtable, *, drop_p=0.0, seed=0, drop_stream=0):
    _abi.call("imgcap_embedding_bwd", dt(dout), ids.numel(), dtable.shape[1], ids.data_ptr(), dout.data_ptr(),
              drop_p, seed, drop_stream, dtable.data_ptr(), stream())


def dropout(x, p, seed, drop_stream, out=None):
    out = torch.empty_like(x) if out is None else out
    _abi.call("imgcap_dropout", dt(x), x.numel(), x.data_ptr(), p, seed, drop_stream, out.data_ptr(), stream())
    return out


def cast(x, out):
    _abi.call("imgcap_cast", dt(x), dt(out), x.numel(), x.data_ptr(), out.data_ptr(), stream())
    return out


def convnext_stem(images, w, bias, ln_w, ln_b, out, norm=None):
    """Stem conv 4x4/s4 + LayerNorm2d -> NHWC.  images: normalised fp32, or raw uint8 pixels with
    ``norm`` = (mean[3], std[3]) fp32 device tensors (normalised in the kernel)."""
    B, _, H, W = images.shape
    if images.dtype == torch.uint8:
        mean, std = norm
        _abi.call("imgcap_convnext_stem_u8", dt(out), B, H, W, w.shape[0], images.data_ptr(), mean.data_ptr(),
                  std.data_ptr(), w.data_ptr(), bias.data_ptr(), ln_w.data_ptr(), ln_b.data_ptr(), out.data_ptr(),
                  stream())
        return out
    _abi.call("imgcap_convnext_stem", dt(out), B, H, W, w.shape[0], images.data_ptr(), w.data_ptr(),
              bias.data_ptr(), ln_w.data_ptr(), ln_b.data_ptr(), out.data_ptr(), stream())
    return out


def dwconv7(x, w49, bias, out):
    """Depthwise 7x7 + bias (NHWC), no LayerNorm."""
    B, H, W, C = x.shape
    _check_dev(x, out)
    _abi.call("imgcap_dwconv7", dt(x), B, H, W, C, x.data_ptr(), w49.data_ptr(), bias.data_ptr(), out.data_ptr(),
              stream())
    return out


def dw_ln_fused(W, C, dtype):
    """Whether imgcap_dwconv7_ln runs the channel-pair kernel with the LayerNorm in its epilogue
    here (convnext.hip dw_cp_fits: W = 7 or 14, C % 128 == 0, C <= 1024, bf16) --
    the encoder then skips the separate add_layernorm pass."""
    return (os.environ.get("IMGCAP_DW_CP", "1") != "0" and dtype == torch.bfloat16 and C % 128 == 0 and C <= 1024
            and W in (7, 14))


def dwconv7_ln(x, w49, bias, ln_w, ln_b, out):
    B, H, W, C = x.shape
    _abi.call("imgcap_dwconv7_ln", dt(x), B, H, W, C, x.data_ptr(), w49.data_ptr(), bias.data_ptr(),
              ln_w.data_ptr(), ln_b.data_ptr(), out.data_ptr(), stream())
    return out


def ln_patchify2(x, ln_w, ln_b, out, cmajor=False):
    B, H, W, C = x.shape
    _abi.call("imgcap_ln_patchify2", dt(x), B, H, W, C, x.data_ptr(), ln_w.data_ptr(), ln_b.data_ptr(),
              int(cmajor), out.data_ptr(), stream())
    return out


def adaptive_pool(x, OH, OW, out):
    B, H, W, C = x.shape
    _abi.call("imgcap_adaptive_pool_nhwc", dt(x), B, H, W, C, OH, OW, x.data_ptr(), out.data_ptr(), stream())
    return out


def sort_gather_rows(lens, enc, caps):
    """decoder.py:64,79-81 in one launch: (enc_sorted [B,P,E], mean [B,E], caps_sorted [B,L],
    sort_ind int64 [B], decode lengths int32 [B]), rows by caption length descending (stable)."""
    _check_dev(lens, enc, caps)
    B, P, E = enc.shape
    L = caps.shape[1]
    if lens.dtype != torch.int64 or caps.dtype != torch.int64 or not (lens.is_contiguous() and enc.is_contiguous()
                                                                     and caps.is_contiguous()):
        raise ValueError("sort_gather_rows: contiguous int64 lengths / captions and a contiguous enc")
    enc_s = torch.empty_like(enc)
    mean = torch.empty(B, E, device=enc.device, dtype=enc.dtype)
    caps_s = torch.empty_like(caps)
    sort_ind = torch.empty(B, device=enc.device, dtype=torch.int64)
    dl = torch.empty(B, device=enc.device, dtype=torch.int32)
    _abi.call("imgcap_sort_gather_rows", dt(enc), B, P, E, L, lens.data_ptr(), enc.data_ptr(), caps.data_ptr(),
              enc_s.data_ptr(), mean.data_ptr(), caps_s.data_ptr(), sort_ind.data_ptr(), dl.data_ptr(), stream())
    return enc_s, mean, caps_s, sort_ind, dl


def mean_mid(x, out):
    B, P, E = x.shape
    _abi.call("imgcap_mean_mid", dt(x), B, P, E, x.data_ptr(), out.data_ptr(), stream())
    return out


def transpose(x, out=None):
    rows, cols = x.shape
    out = torch.empty(cols, rows, device=x.device, dtype=x.dtype) if out is None else out
    _abi.call("imgcap_transpose", dt(x), rows, cols, x.data_ptr(), x.stride(0), out.data_ptr(), out.stride(0),
              stream())
    return out


_seed_counter = None  # the registered counter tensor, kept alive while the library points at it


def set_seed_counter(counter):
    """Mix the device int64 scalar ``counter`` into every mask seed (None = off); see
    imgcap_set_seed_counter.  The library keeps a raw pointer, so the tensor is held here until
    it is replaced (a trainer going away must not leave a dangling counter behind)."""
    global _seed_counter
    if counter is not None:
        _check_dev(counter)
        if counter.dtype != torch.int64 or counter.numel() != 1:
            raise ValueError("seed counter must be a one-element int64 tensor")
    _abi.call("imgcap_set_seed_counter", ptr(counter))
    _seed_counter = counter


# widths served by the fused CNBlock MLP kernel (the others run LN + two GEMMs); IMGCAP_FUSED_MLP_C
# overrides for A/B runs ("96,128")
CNBLOCK_MLP_CHANNELS = tuple(int(c) for c in os.environ.get("IMGCAP_FUSED_MLP_C", "96,128,192").split(",") if c)


def cnblock_mlp(z, w1, b1, w2, b2, gamma, x, sd=None, rows_per_sample=1, ln_w=None, ln_b=None):
    """x += gamma * sd * (GELU(LN(z) W1^T + b1) W2^T + b2), hidden on chip (bf16; x updated in
    place).  With ln_w/ln_b the LayerNorm (eps 1e-6) is applied to z in the kernel."""
    _check_dev(z, w1, w2, x)
    M, C = x.shape
    _abi.call("imgcap_cnblock_mlp", M, C, z.data_ptr(), ptr(ln_w), ptr(ln_b), w1.data_ptr(), b1.data_ptr(),
              w2.data_ptr(), b2.data_ptr(), gamma.data_ptr(), ptr(sd), rows_per_sample, x.data_ptr(), stream())
    return x


def stochastic_depth_scales(probs, B, seed, drop_stream, out):
    _check_dev(probs, out)
    _abi.call("imgcap_stochastic_depth_scales", probs.numel(), B, probs.data_ptr(), seed, drop_stream,
              out.data_ptr(), stream())
    return out


# ---- ConvNeXt backward (trainable encoder children) ----------------------------------------
def dwconv7_bwd_data(dz, w49, out, res=None):
    """out = res + dwconv7^T(dz) (flipped taps, no bias); w49 = forward weights [49][C]."""
    B, H, W, C = dz.shape
    _check_dev(dz, out)
    _abi.call("imgcap_dwconv7_bwd_data", dt(dz), B, H, W, C, dz.data_ptr(), w49.data_ptr(), ptr(res),
              out.data_ptr(), stream())
    return out


def dwconv7_wgrad(dz, x, dw, db):
    """dw [C,1,7,7] / [C,49] fp32 and db [C] fp32 written (not accumulated)."""
    B, H, W, C = dz.shape
    _abi.call("imgcap_dwconv7_wgrad", dt(dz), B, H, W, C, dz.data_ptr(), x.data_ptr(), dw.data_ptr(),
              db.data_ptr(), stream())


def layer_scale_grad(G, w2, b2, gamma, cs, dw2, wg, dgamma, db2):
    C, C4 = G.shape
    _abi.call("imgcap_layer_scale_grad", dt(wg), C, C4, G.data_ptr(), w2.data_ptr(), b2.data_ptr(),
              gamma.data_ptr(), cs.data_ptr(), dw2.data_ptr(), wg.data_ptr(), dgamma.data_ptr(), db2.data_ptr(),
              stream())


def rowscale(x, s, rows_per_scale, out=None):
    out = torch.empty_like(x) if out is None else out
    rows, cols = x.shape
    _abi.call("imgcap_rowscale", dt(x), rows, cols, x.data_ptr(), s.data_ptr(), rows_per_scale, out.data_ptr(),
              stream())
    return out


def ln_patchify2_bwd(x, dpatches, ln_w, dx, dln_w, dln_b, cmajor=False):
    B, H, W, C = x.shape
    _abi.call("imgcap_ln_patchify2_bwd", dt(x), B, H, W, C, x.data_ptr(), dpatches.data_ptr(), ln_w.data_ptr(),
              int(cmajor), dx.data_ptr(), dln_w.data_ptr(), dln_b.data_ptr(), stream())
    return dx


def adaptive_pool_bwd(dy, H, W, dx):
    B, OH, OW, C = dy.shape
    _abi.call("imgcap_adaptive_pool_bwd_nhwc", dt(dy), B, H, W, C, OH, OW, dy.data_ptr(), dx.data_ptr(), stream())
    return dx

"""Cross-stream hazards of the captured schedules ("round 4 side-stream drift and the
round 5 scratch race").

The library's split-reduction scratch is one buffer per workspace slot, and a slot is shared by
every stream of a schedule branch (the library refuses a slot's scratch to a second stream of one
captured graph: the last test).  The LSTM backward runs the embedding gradient -- a scratch
user -- on a side stream beside the main stream's grouped weight-gradient GEMMs and bias column
sums, so those two entry points must never request scratch: a round-5 two-pass column sum that
did faulted the LSTM checkpoint test with an illegal address.  The check: attach a 16-byte caller
workspace to the slot and call the entry points directly -- any scratch request returns
IMGCAP_EWORKSPACE (-3) instead of enqueuing (a split-K GEMM is the positive control)."""
import ctypes

import pytest
import torch

pytestmark = pytest.mark.gpu


def test_side_stream_entry_points_take_no_library_scratch(hip_device):
    from imagecaptioningconvnext_amd import _abi
    from imagecaptioningconvnext_amd import kernels as K
    dev = hip_device
    K.colsum(torch.zeros(1, 8, device=dev), torch.zeros(8, device=dev))  # workspaces attached
    L = _abi.lib()
    tiny = torch.empty(16, dtype=torch.uint8, device=dev)
    x = torch.randn(3328, 1536, device=dev).to(torch.bfloat16)
    xf = torch.randn(416, 1024, device=dev)
    outs = [torch.zeros(1536, device=dev), torch.zeros(512, device=dev)]
    items = (_abi.ColsumItem * 2)()
    for it, (t, o, cols, ld) in zip(items, ((x, outs[0], 1536, 1536), (xf, outs[1], 512, 1024))):
        it.x, it.out, it.ld, it.rows, it.cols, it.dtype, it.beta = t.data_ptr(), o.data_ptr(), ld, t.shape[0], cols, \
            K.dt(t), 0.0
    a = torch.randn(3328, 512, device=dev).to(torch.bfloat16)
    b = torch.randn(3328, 512, device=dev).to(torch.bfloat16)
    g = torch.zeros(512, 512, device=dev)
    probs = (_abi.GemmProblem * 1)()
    p = probs[0]
    p.A, p.B, p.C = a.data_ptr(), b.data_ptr(), g.data_ptr()
    p.lda, p.ldb, p.ldc = 512, 512, 512
    p.M, p.N, p.K, p.alpha, p.beta = 512, 512, 3328, 1.0, 0.0
    st = K.stream()
    old = _abi._ws[(dev.index or 0, 0)]
    assert L.imgcap_workspace_slot(0) == 0
    assert L.imgcap_workspace_attach(0, tiny.data_ptr(), 16) == 0
    try:
        rc_cs = L.imgcap_colsum_multi(2, ctypes.cast(items, ctypes.c_void_p), st)
        part = torch.empty(13 * 1536 + 2 * 512, device=dev)  # the two-pass form: caller-owned partials
        rc_cs2 = L.imgcap_colsum_multi_part(2, ctypes.cast(items, ctypes.c_void_p), part.data_ptr(), part.numel(), st)
        rc_gg = L.imgcap_gemm_grouped(0, 0, 1, ctypes.cast(probs, ctypes.c_void_p), st)
        # positive control: a split-K product needs scratch and is refused
        ep = _abi.Epilogue()
        ep.alpha, ep.c_dtype, ep.split_k, ep.rows_per_scale, ep.drop_ld = 1.0, _abi.F32, 4, 1, 512
        rc_split = L.imgcap_gemm(K.dt(a), 0, 0, 512, 512, 3328, a.data_ptr(), 512, 0, b.data_ptr(), 512, 0,
                                 g.data_ptr(), 512, 0, 1, ctypes.byref(ep), st)
    finally:
        assert L.imgcap_workspace_attach(0, old.data_ptr(), old.numel()) == 0
    torch.cuda.synchronize()
    assert rc_split == _abi.IMGCAP_EWORKSPACE
    assert rc_cs == 0 and rc_cs2 == 0 and rc_gg == 0
    torch.testing.assert_close(outs[0], x.float().sum(0), rtol=1e-4, atol=1e-2)
    torch.testing.assert_close(outs[1], xf[:, :512].sum(0), rtol=1e-5, atol=1e-3)
    torch.testing.assert_close(g, a.float().t() @ b.float(), rtol=2e-2, atol=2e-1)


def test_library_refuses_one_slot_scratch_from_two_streams_of_a_capture(hip_device):
    """The library-side guard (csrc/abi.cpp workspace): inside ONE captured graph, a slot's scratch
    requested from a second stream is refused before anything is enqueued (two unordered branches
    would share the buffer -- the round-5 race); the same calls on one stream, or with the second
    stream on its own slot, capture and replay normally."""
    from imagecaptioningconvnext_amd import kernels as K
    dev = hip_device
    a = torch.randn(256, 4096, device=dev).to(torch.bfloat16)
    b = torch.randn(4096, 256, device=dev).to(torch.bfloat16)
    want = a.float() @ b.float()
    out1, out2 = torch.zeros(256, 256, device=dev), torch.zeros(256, 256, device=dev)
    K.gemm(a, b, out=out1, split_k=4)  # warm-up: workspaces attached and large enough
    torch.cuda.synchronize()
    main = torch.cuda.Stream(device=dev)
    side = torch.cuda.Stream(device=dev)
    for use_slot in (False, True):
        g = torch.cuda.CUDAGraph()
        err = None
        with torch.cuda.stream(main):
            g.capture_begin()
            K.gemm(a, b, out=out1, split_k=4)
            K.fork(side, main)
            with torch.cuda.stream(side):
                try:
                    if use_slot:
                        with K.workspace_slot(1):
                            K.gemm(a, b, out=out2, split_k=4)
                    else:
                        K.gemm(a, b, out=out2, split_k=4)
                except RuntimeError as e:
                    err = str(e)
            K.join(main, side)
            K.assert_joined("test")
            g.capture_end()
        if use_slot:
            assert err is None
            out1.zero_()
            out2.zero_()
            g.replay()
            torch.cuda.synchronize()
            torch.testing.assert_close(out1, want, rtol=1e-3, atol=1e-2)
            torch.testing.assert_close(out2, want, rtol=1e-3, atol=1e-2)
        else:
            assert err is not None and "two streams of one captured graph" in err, err
        del g


def test_nested_fork_refused_before_it_reaches_the_capture(hip_device):
    """A branch forked from an open branch (M -> S -> X) crashes hipStreamEndCapture with a
    segfault on ROCm 7.2 (tools/probe/capture_refork.py "nested").  kernels.fork
    refuses it -- eagerly and inside a capture -- and the capture that asked for it still ends and
    replays normally once its open branch is joined."""
    from imagecaptioningconvnext_amd import kernels as K
    dev = hip_device
    x = torch.zeros(1024, device=dev)
    S, X = torch.cuda.Stream(device=dev), torch.cuda.Stream(device=dev)
    main = torch.cuda.current_stream(dev)
    K.fork(S, main)
    with pytest.raises(RuntimeError, match="open branch"):
        K.fork(X, S)
    K.join(main, S)
    K.assert_joined("eager")
    torch.cuda.synchronize()
    cap = torch.cuda.Stream(device=dev)
    g = torch.cuda.CUDAGraph()
    with torch.cuda.stream(cap):
        g.capture_begin()
        K.fork(S, cap)
        with torch.cuda.stream(S):
            x.add_(1.0)
            with pytest.raises(RuntimeError, match="open branch"):
                K.fork(X, S)
        K.join(cap, S)
        K.assert_joined("test")
        g.capture_end()
    g.replay()
    g.replay()
    torch.cuda.synchronize()
    assert torch.equal(x, torch.full_like(x, 2.0))

"""ctypes binding of libimgcap_hip.so (include/imgcap_abi.h).

The library is built in-tree by ``__graft_entry__.build()`` / ``make -C
imagecaptioningconvnext_amd/csrc``.  There is no fallback: if the shared object is missing
or fails to load, importing the product path raises.
"""
import ctypes
import os

_HERE = os.path.dirname(os.path.abspath(__file__))
# IMGCAP_LIB: alternative build of the same library (the diagnostic stamps build of tools/)
LIB_PATH = os.environ.get("IMGCAP_LIB") or os.path.join(_HERE, "libimgcap_hip.so")

F32, BF16 = 0, 1
# imgcap_gemm_plan kinds of the stream-tile configs 1..6 (IMGCAP_GEMM_PT .. IMGCAP_GEMM_PT128K)
GEMM_PT = 8
# ... and of the weight-stationary short-K kernel (8-wave / 4-wave blocks)
GEMM_WS, GEMM_WS4 = 14, 15
FP8MX = 2
ACT_NONE, ACT_GELU, ACT_RELU, ACT_DGELU = 0, 1, 2, 3

c_void_p, c_int, c_int64, c_float, c_uint64, c_uint32 = (ctypes.c_void_p, ctypes.c_int, ctypes.c_int64,
                                                         ctypes.c_float, ctypes.c_uint64, ctypes.c_uint32)


class Epilogue(ctypes.Structure):
    _fields_ = [
        ("bias", c_void_p), ("colscale", c_void_p), ("rowscale", c_void_p), ("res", c_void_p), ("aux", c_void_p),
        ("ldr", c_int64), ("ldaux", c_int64), ("drop_ld", c_int64), ("seed", c_uint64),
        ("alpha", c_float), ("beta", c_float), ("drop_p", c_float), ("aux_scale", c_float),
        ("act", ctypes.c_int32), ("c_dtype", ctypes.c_int32), ("rows_per_scale", ctypes.c_int32),
        ("drop_stream", c_uint32),
        ("split_k", ctypes.c_int32),
        ("c_scale", c_void_p),
    ]


class LstmDesc(ctypes.Structure):
    _fields_ = [(n, ctypes.c_int32) for n in ("dtype", "B", "P", "E", "A", "D", "M", "T")] + [
        (n, c_void_p) for n in ("w_hcat", "b_hcat", "w_ih", "w_f", "enc", "att1", "xe", "c0", "dl", "g1", "alphas",
                                "awe", "zs", "gates", "cs", "hs", "hprev", "w_zh_t", "w_att_t", "dhs", "dalpha",
                                "dcat", "dz", "ws_y", "y_cnt", "dh", "dc", "de", "datt1", "dwf", "dbea")] + [
        ("x_slices", ctypes.c_int32), ("y_slices", ctypes.c_int32), ("dawe", c_void_p), ("sync", c_void_p),
        ("sync_words", ctypes.c_int32), ("row_groups", ctypes.c_int32)]


class MhaDesc(ctypes.Structure):
    _fields_ = [(n, ctypes.c_int32) for n in ("dtype", "B", "H", "Lq", "Lk", "dh", "causal")] + [
        ("pad_id", c_int64), ("ldq", c_int64), ("ldk", c_int64), ("ldv", c_int64), ("ldo", c_int64),
        ("q", c_void_p), ("k", c_void_p), ("v", c_void_p), ("o", c_void_p), ("lse", c_void_p),
        ("key_ids", c_void_p), ("scale", c_float), ("drop_p", c_float), ("seed", c_uint64),
        ("drop_stream", c_uint32), ("dout", c_void_p), ("lddo", c_int64), ("dq", c_void_p), ("dk", c_void_p),
        ("dv", c_void_p), ("lddq", c_int64), ("lddk", c_int64), ("lddv", c_int64), ("kv_rows", c_int64),
        ("probs", c_void_p)]


class GemmProblem(ctypes.Structure):
    _fields_ = [("A", c_void_p), ("B", c_void_p), ("C", c_void_p), ("lda", c_int64), ("ldb", c_int64),
                ("ldc", c_int64), ("M", ctypes.c_int32), ("N", ctypes.c_int32), ("K", ctypes.c_int32),
                ("alpha", c_float), ("beta", c_float)]


class ColsumItem(ctypes.Structure):
    _fields_ = [("x", c_void_p), ("out", c_void_p), ("ld", c_int64), ("rows", ctypes.c_int32),
                ("cols", ctypes.c_int32), ("dtype", ctypes.c_int32), ("vec_ok", ctypes.c_int32),
                ("beta", c_float)]


# name -> argtypes  (every entry point declared in include/imgcap_abi.h)
_SIGS = {
    "imgcap_version": [],
    "imgcap_set_seed_counter": [c_void_p],
    "imgcap_gemm_plan": [c_int] * 6 + [c_int64, c_int64, c_int, c_int, c_void_p],
    "imgcap_gemm_plan_ep": [c_int] * 6 + [c_int64, c_int64, c_int, c_void_p, c_void_p],
    "imgcap_gemm_set_pt": [c_int],
    "imgcap_gemm_get_pt": [],
    "imgcap_gemm_set_ws": [c_int],
    "imgcap_gemm_get_ws": [],
    "imgcap_dwconv7": [c_int] * 5 + [c_void_p] * 5,
    "imgcap_cnblock_mlp": [c_int, c_int] + [c_void_p] * 9 + [c_int, c_void_p, c_void_p],
    "imgcap_stochastic_depth_scales": [c_int, c_int, c_void_p, c_uint64, c_uint32, c_void_p, c_void_p],
    "imgcap_gemm": [c_int, c_int, c_int, c_int, c_int, c_int, c_void_p, c_int64, c_int64, c_void_p, c_int64,
                    c_int64, c_void_p, c_int64, c_int64, c_int, ctypes.POINTER(Epilogue), c_void_p],
    "imgcap_transpose": [c_int, c_int, c_int, c_void_p, c_int64, c_void_p, c_int64, c_void_p],
    "imgcap_colsum": [c_int, c_int, c_int, c_void_p, c_int64, c_void_p, c_float, c_void_p],
    "imgcap_add_layernorm_fwd": [c_int, c_int, c_int, c_void_p, c_void_p, c_float, c_uint64, c_uint32, c_void_p,
                                 c_void_p, c_float, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p],
    "imgcap_add_layernorm_bwd": [c_int, c_int, c_int, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_float,
                                 c_uint64, c_uint32, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p],
    "imgcap_add_layernorm_bwd_blocks": [c_int],
    "imgcap_convnext_stem": [c_int, c_int, c_int, c_int, c_int, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p,
                             c_void_p, c_void_p],
    "imgcap_convnext_stem_u8": [c_int, c_int, c_int, c_int, c_int] + [c_void_p] * 9,
    "imgcap_dwconv7_ln": [c_int, c_int, c_int, c_int, c_int, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p,
                          c_void_p, c_void_p],
    "imgcap_ln_patchify2": [c_int, c_int, c_int, c_int, c_int, c_void_p, c_void_p, c_void_p, c_int, c_void_p,
                            c_void_p],
    "imgcap_adaptive_pool_nhwc": [c_int, c_int, c_int, c_int, c_int, c_int, c_int, c_void_p, c_void_p, c_void_p],
    "imgcap_embedding_fwd": [c_int, c_int, c_int, c_void_p, c_void_p, c_void_p, c_int, c_float, c_uint64, c_uint32,
                             c_void_p, c_void_p],
    "imgcap_embedding_bwd": [c_int, c_int, c_int, c_void_p, c_void_p, c_float, c_uint64, c_uint32, c_void_p,
                             c_void_p],
    "imgcap_ce_fwd": [c_int, c_int, c_int, c_void_p, c_int64, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p],
    "imgcap_ce_bwd": [c_int, c_int, c_int, c_void_p, c_int64, c_void_p, c_void_p, c_void_p, c_void_p, c_int64,
                      c_void_p],
    "imgcap_ce_fused": [c_int, c_int, c_int, c_void_p, c_int64, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p,
                        c_void_p, c_int64, c_void_p],
    "imgcap_clamp_adam": [c_int64, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_float, c_float, c_float,
                          c_float, c_int, c_float, c_float, c_void_p, c_void_p],
    "imgcap_lstm_tf_fwd": [ctypes.POINTER(LstmDesc), c_void_p],
    "imgcap_lstm_tf_bwd": [ctypes.POINTER(LstmDesc), c_void_p],
    "imgcap_lstm_sync_words": [ctypes.POINTER(LstmDesc)],
    "imgcap_mha_fwd": [ctypes.POINTER(MhaDesc), c_void_p],
    "imgcap_mha_bwd": [ctypes.POINTER(MhaDesc), c_void_p],
    "imgcap_attn_reg": [c_int, c_int, c_int, c_void_p, c_void_p, c_float, c_void_p, c_void_p, c_void_p, c_void_p],
    "imgcap_dropout": [c_int, c_int64, c_void_p, c_float, c_uint64, c_uint32, c_void_p, c_void_p],
    "imgcap_loss_finalize": [c_int, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p],
    "imgcap_tf_targets": [c_int, c_int, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_int, c_void_p],
    "imgcap_mean_mid": [c_int, c_int, c_int, c_int, c_void_p, c_void_p, c_void_p],
    "imgcap_sort_gather_rows": [c_int] * 5 + [c_void_p] * 9,
    "imgcap_cast": [c_int, c_int, c_int64, c_void_p, c_void_p, c_void_p],
    "imgcap_fill": [c_int, c_int64, c_float, c_void_p, c_void_p],
    "imgcap_dwconv7_bwd_data": [c_int] * 5 + [c_void_p] * 5,
    "imgcap_dwconv7_wgrad": [c_int] * 5 + [c_void_p] * 5,
    "imgcap_layer_scale_grad": [c_int, c_int, c_int] + [c_void_p] * 10,
    "imgcap_rowscale": [c_int, c_int64, c_int, c_void_p, c_void_p, c_int, c_void_p, c_void_p],
    "imgcap_ln_patchify2_bwd": [c_int] * 5 + [c_void_p] * 3 + [c_int] + [c_void_p] * 4,
    "imgcap_adaptive_pool_bwd_nhwc": [c_int] * 7 + [c_void_p] * 3,
    "imgcap_lstm_denc": [c_int] * 4 + [c_void_p] * 6,
    "imgcap_gemm_set_policy": [c_int],
    "imgcap_workspace_slot": [c_int],
    "imgcap_workspace_attach": [c_int, c_void_p, c_uint64],
    "imgcap_workspace_needed": [c_int, ctypes.POINTER(c_uint64)],
    "imgcap_colsum_multi": [c_int, c_void_p, c_void_p],
    "imgcap_colsum_multi_part": [c_int, c_void_p, c_void_p, c_int64, c_void_p],
    "imgcap_gemm_grouped": [c_int, c_int, c_int, c_void_p, c_void_p],
    "imgcap_gemm_mx": [c_int, c_int, c_int, c_void_p, c_int64, c_void_p, c_void_p, c_int64, c_void_p, c_void_p,
                       c_int64, ctypes.POINTER(Epilogue), c_void_p],
    "imgcap_mx_quant_rows": [c_int, c_int, c_int, c_void_p, c_int64, c_void_p, c_void_p, c_float, c_void_p, c_void_p,
                             c_void_p],
    "imgcap_greedy_select": [c_int, c_int, c_int, c_void_p, c_int64, c_int, c_int, c_int64, c_void_p, c_void_p,
                             c_void_p, c_void_p, c_void_p, c_void_p, c_int, c_void_p],
    "imgcap_slice_reduce": [c_int64, c_int, c_void_p, c_int64, c_float, c_int64, c_void_p, c_void_p, c_void_p],
}

_lib = None
# include/imgcap_abi.h IMGCAP_ABI_VERSION (tests/test_abi_cpu.py checks the two agree)
ABI_VERSION = 6


def lib():
    """Load (once) and return the shared library; raises if it is missing."""
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise RuntimeError(f"{LIB_PATH} not built: run __graft_entry__.build() (hipcc gfx950). "
                               "There is no CPU/eager fallback for the HIP path.")
        L = ctypes.CDLL(LIB_PATH)
        L.imgcap_last_error_string.restype = ctypes.c_char_p
        L.imgcap_last_error_string.argtypes = []
        for name, argt in _SIGS.items():
            fn = getattr(L, name)
            fn.argtypes = argt
            fn.restype = c_int
        if L.imgcap_version() != ABI_VERSION:
            raise RuntimeError(f"{LIB_PATH}: ABI revision {L.imgcap_version()}, this binding expects "
                               f"{ABI_VERSION} (include/imgcap_abi.h IMGCAP_ABI_VERSION): rebuild the library")
        _lib = L
    return _lib


def exported_symbols():
    return ["imgcap_last_error_string"] + list(_SIGS)


IMGCAP_EWORKSPACE = -3
# caller-owned split-reduction scratch (imgcap_workspace_attach): {(device, slot): uint8 tensor}
# from the PyTorch caching allocator; superseded buffers stay referenced (a captured graph may
# still point at them)
_ws = {}
_ws_old = []
_WS_INITIAL = 32 << 20


def _attach(dev, slot, nbytes):
    import torch
    nbytes = (int(nbytes) + (1 << 20) - 1) >> 20 << 20
    t = torch.empty(nbytes, dtype=torch.uint8, device=torch.device("cuda", dev))
    if (dev, slot) in _ws:
        _ws_old.append(_ws[(dev, slot)])
    _ws[(dev, slot)] = t
    rc = lib().imgcap_workspace_attach(slot, t.data_ptr(), nbytes)
    if rc != 0:
        raise RuntimeError("imgcap_workspace_attach: " + lib().imgcap_last_error_string().decode(errors="replace"))


def _grow_workspaces(dev):
    need = c_uint64(0)
    for slot in (0, 1, 2):
        lib().imgcap_workspace_needed(slot, ctypes.byref(need))
        if need.value > _ws[(dev, slot)].numel():
            _attach(dev, slot, need.value * 5 // 4)


def call(name, *args):
    import torch
    dev = torch.cuda.current_device() if torch.cuda.is_available() else None
    if dev is not None and (dev, 0) not in _ws:
        _attach(dev, 0, _WS_INITIAL)
        _attach(dev, 1, _WS_INITIAL)
        _attach(dev, 2, _WS_INITIAL // 4)
    rc = getattr(lib(), name)(*args)
    if rc == IMGCAP_EWORKSPACE and dev is not None:  # nothing was enqueued: grow, then retry once
        _grow_workspaces(dev)
        rc = getattr(lib(), name)(*args)
    if rc != 0:
        msg = lib().imgcap_last_error_string().decode(errors="replace")
        raise RuntimeError(f"{name} failed (rc={rc}): {msg}")

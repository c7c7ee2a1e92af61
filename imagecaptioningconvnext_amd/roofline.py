"""Live roofline of the bench step's dominant kernel (bench.py ``roofline`` field).

Every library call of one train step is timed where it runs: the step is launched eagerly (the
sequential schedule: encoder forward, decoder forward + loss, backward, clamp + Adam) and each
``imgcap_*`` call is bracketed by two HIP events on the stream it is launched on, with a short
device-side sleep queued in front of the first event so that the GPU runs behind the host and the
events bracket only that call's kernels (no host launch gap inside the interval).  Three such
steps; the median per call.  Calls are grouped by the kernel symbol rocprofv3 lists for them
(GEMMs by the kernel ``imgcap_gemm_plan`` picks; the persistent LSTM recurrences, the attention,
the fused MLP, the depthwise conv, CE, LayerNorm, Adam ... by their own symbols) and ranked by
time per step; the top group is the step's dominant kernel.  Its algorithmic work per launch
(DESIGN.md §5 lists the per-call formulas: 2*M*N*K for GEMMs, the recurrences' MACs per row and
step, bytes read + written once for the HBM-bound kernels) over its average launch duration is
reported against the MI355X peak (bf16 dense MFMA 2.5 PFLOP/s, MX-FP8 5 PFLOP/s, fp32 157 TF/s,
HBM 8 TB/s; MI355X_MICROARCH.md).
"""
import collections
import json
import os
import statistics

import torch

from . import _abi
from . import kernels as K

PEAK_HBM_GBS = 8000.0
PEAK_BF16_TFLOPS = 2500.0
PEAK_FP8_TFLOPS = 5000.0  # dense block-scaled (MX) e4m3 MFMA
PEAK_F32_TFLOPS = 157.3   # f32 MFMA = f32 vector rate
SLEEP_CYCLES = 400_000    # device sleep in front of each timed call (> the host's launch time)

_KIND_NAME = {1: "gemm_skinny_kernel", 2: "gemm_kernel<64,64,64>", 3: "gemm_kernel<128,128,64>",
              4: "gemm_glds_kernel<128,128>", 5: "gemm256_kernel<256,256>", 6: "gemm_glds_kernel<64,64>",
              7: "gemm_glds_kernel<128,64>", 8: "gemm_pt_kernel<256,128>", 9: "gemm_pt_kernel<128,256>",
              10: "gemm_pt_kernel<128,128>", 11: "gemm_pt_kernel<128,192>", 12: "gemm_pt_kernel<128,128,4w>",
              13: "gemm_pt_kernel<128,128,k128>"}

# calls that launch nothing
_NO_KERNEL = {"imgcap_workspace_slot", "imgcap_set_seed_counter", "imgcap_gemm_set_policy", "imgcap_workspace_attach",
              "imgcap_workspace_needed", "imgcap_version"}

# ABI entry point -> the kernel symbol rocprofv3 reports for it (substring)
_SYMBOL = {
    "imgcap_lstm_tf_fwd": "lstm_fwd_persist_kernel", "imgcap_lstm_tf_bwd": "lstm_bwd_persist_kernel",
    "imgcap_mha_fwd": "mha_fwd_kernel", "imgcap_mha_bwd": "mha_bwd_kernel",
    "imgcap_dwconv7": "dwconv7_kernel", "imgcap_dwconv7_ln": "dwconv7_ln_kernel",
    "imgcap_dwconv7_bwd_data": "dwconv7_kernel", "imgcap_dwconv7_wgrad": "dwconv7_wgrad_kernel",
    "imgcap_ce_fused": "ce_fused_kernel", "imgcap_ce_fwd": "ce_fwd_kernel", "imgcap_ce_bwd": "ce_bwd_kernel",
    "imgcap_add_layernorm_fwd": "add_ln_fwd_kernel", "imgcap_add_layernorm_bwd": "add_ln_bwd_kernel",
    "imgcap_clamp_adam": "clamp_adam_kernel", "imgcap_convnext_stem": "stem_kernel",
    "imgcap_convnext_stem_u8": "stem_kernel", "imgcap_ln_patchify2": "ln_patchify2_kernel",
    "imgcap_ln_patchify2_bwd": "ln_patchify2_bwd_kernel", "imgcap_transpose": "transpose_kernel",
    "imgcap_embedding_fwd": "embedding_fwd_kernel", "imgcap_embedding_bwd": "emb_segsum_kernel",
    "imgcap_colsum_multi": "colsum_multi_kernel", "imgcap_colsum": "colsum_kernel",
    "imgcap_mx_quant_rows": "mx_quant_rows_kernel", "imgcap_sort_gather_rows": "sort_gather_kernel",
    "imgcap_dropout": "dropout_kernel", "imgcap_cast": "cast_kernel", "imgcap_rowscale": "rowscale_kernel",
    "imgcap_layer_scale_grad": "layer_scale_grad_kernel", "imgcap_lstm_denc": "lstm_denc_kernel",
    "imgcap_attn_reg": "attn_reg_kernel", "imgcap_loss_finalize": "loss_finalize_kernel",
    "imgcap_stochastic_depth_scales": "sd_scales_kernel", "imgcap_adaptive_pool_nhwc": "adaptive_pool_kernel",
    "imgcap_adaptive_pool_bwd_nhwc": "adaptive_pool_bwd_kernel", "imgcap_mean_mid": "mean_mid_kernel",
    "imgcap_fill": "fill_kernel", "imgcap_slice_reduce": "slice_reduce_kernel",
}


def _dw_symbol(fn, dtype_id, W, C):
    """The kernel convnext.hip's depthwise dispatch launches (dw_cp_fits, dwconv7_launch)."""
    bf = dtype_id == _abi.BF16
    ln = fn == "imgcap_dwconv7_ln"
    if bf and os.environ.get("IMGCAP_DW_CP", "") != "0" and W in (7, 14) and C % 128 == 0 and (not ln or C <= 1024):
        return "dwconv7_cp_kernel"
    if ln:
        return "dwconv7_ln_kernel"
    return "dwconv7_roll_kernel" if W in (56, 28, 14, 7, 64, 32, 16, 8) else "dwconv7_kernel"


def _esz(dtype_id):
    return 4 if dtype_id == _abi.F32 else 2


def _mfma_peak(dtype_id):
    return PEAK_BF16_TFLOPS if dtype_id == _abi.BF16 else PEAK_F32_TFLOPS


def _gemm_group(a):
    dtype, ak, bk, M, N, K_ = a[0], a[1], a[2], a[3], a[4], a[5]
    lda, ldb, ep = a[7], a[10], a[16]._obj
    kind, splits = K.gemm_plan(dtype, ak, bk, M, N, K_, lda, ldb, a[15], ep.split_k, ep=ep)
    name = _KIND_NAME.get(kind, f"gemm kind {kind}")
    if kind in (2, 3, 4, 5, 6, 7, 8, 9, 10, 11, 12, 13):
        name += f"<ak={ak},bk={bk}>" + (" (split-K)" if splits > 1 else "")
    tf = lambda v: "true" if v else "false"  # noqa: E731
    sym = {4: f"gemm_glds_kernel<128, 128, {tf(ak)}, {tf(bk)}, ",  # any stage count
           5: f"gemm256_kernel<64, 2, {tf(ak)}, {tf(bk)}>",
           6: f"gemm_glds_kernel<64, 64, {tf(ak)}, {tf(bk)}, ",
           7: f"gemm_glds_kernel<128, 64, {tf(ak)}, {tf(bk)}, ",
           8: "gemm_pt_kernel<256, 128, 4, 2, 3, " + f"{tf(ak)}, {tf(bk)}, ",
           9: "gemm_pt_kernel<128, 256, 2, 4, 3, " + f"{tf(ak)}, {tf(bk)}, ",
           10: "gemm_pt_kernel<128, 128, 2, 4, 4, " + f"{tf(ak)}, {tf(bk)}, ",
           11: "gemm_pt_kernel<128, 192, 2, 4, 3, " + f"{tf(ak)}, {tf(bk)}, ",
           12: "gemm_pt_kernel<128, 128, 2, 2, 2, " + f"{tf(ak)}, {tf(bk)}, ",
           13: "gemm_pt_kernel<128, 128, 2, 4, 2, " + f"{tf(ak)}, {tf(bk)}, "}.get(kind, _KIND_NAME.get(kind, ""))
    return name, sym


def _work(fn, a):
    """(group key, symbol, bound, work, peak, shape) of one call: work in FLOP (bound "mfma") or
    bytes read + written once (bound "hbm"); work None = no model (ranked by time only)."""
    sym = _SYMBOL.get(fn, fn)
    if fn == "imgcap_gemm":
        name, gsym = _gemm_group(a)
        M, N, K_, batch = a[3], a[4], a[5], a[15]
        return name, gsym, "mfma", 2.0 * M * N * K_ * batch, _mfma_peak(a[0]), (M, N, K_)
    if fn == "imgcap_gemm_grouped":
        arr = (_abi.GemmProblem * a[2]).from_address(a[3].value)
        f = sum(2.0 * p.M * p.N * p.K for p in arr)
        ak, bk = a[0], a[1]
        nm = f"gemm_glds_grouped_kernel<{'true' if ak else 'false'}, {'true' if bk else 'false'}>"
        return nm, nm, "mfma", f, PEAK_BF16_TFLOPS, (a[2], "problems")
    if fn == "imgcap_gemm_mx":
        M, N, K_ = a[0], a[1], a[2]
        return "gemm_mx_kernel (MX-FP8)", "gemm_mx", "mfma", 2.0 * M * N * K_, PEAK_FP8_TFLOPS, (M, N, K_)
    if fn in ("imgcap_lstm_tf_fwd", "imgcap_lstm_tf_bwd"):
        d = a[0]._obj
        B, P, E, A, D, T = d.B, d.P, d.E, d.A, d.D, d.T
        if fn.endswith("fwd"):  # G: h [W_da; W_fb]; U: [z | h] [W_ih_z | W_hh]^T; R: scores + context
            macs = D * (A + E) + (E + D) * 4 * D + P * A + P * E
        else:  # U: dgates W_hh + d att [W_da; W_fb]; X: dgates W_ih_z; R: d alpha, d att1 / de
            macs = 4 * D * D + (A + E) * D + 4 * D * E + P * E + 2 * P * A
        return sym, sym, "mfma", 2.0 * B * T * macs, _mfma_peak(d.dtype), (B, T, E, D)
    if fn in ("imgcap_mha_fwd", "imgcap_mha_bwd"):
        m = a[0]._obj
        if m.dtype == _abi.BF16:  # mha.hip dispatch: the bf16 kernels (natural LDS images)
            sym = sym.replace("_kernel", "_bf16_kernel")
        f = 2.0 * m.B * m.H * m.Lq * m.Lk * m.dh * (2 if fn.endswith("fwd") else 5)
        if m.causal:
            f *= 0.5
        return sym, sym, "mfma", f, _mfma_peak(m.dtype), (m.B, m.H, m.Lq, m.Lk)
    if fn == "imgcap_cnblock_mlp":
        M, C = a[0], a[1]
        nm = f"cnblock_mlp_{'res' if C == 96 else 'str'}_kernel<{C}>"
        return nm, nm, "mfma", 16.0 * M * C * C, PEAK_BF16_TFLOPS, (M, C)
    if fn in ("imgcap_dwconv7", "imgcap_dwconv7_ln", "imgcap_dwconv7_wgrad"):
        e = _esz(a[0])
        if fn != "imgcap_dwconv7_wgrad":
            sym = _dw_symbol(fn, a[0], a[3], a[4])
        n = a[1] * a[2] * a[3] * a[4]
        return sym, sym, "hbm", 2.0 * n * e + 50 * a[4] * 4, PEAK_HBM_GBS, (a[1], a[2], a[3], a[4])
    if fn == "imgcap_dwconv7_bwd_data":
        e = _esz(a[0])
        n = a[1] * a[2] * a[3] * a[4]
        res = a[7] is not None and a[7] != 0
        return sym, sym, "hbm", (3.0 if res else 2.0) * n * e + 49 * a[4] * 4, PEAK_HBM_GBS, (a[1], a[2], a[3], a[4])
    if fn in ("imgcap_ce_fused", "imgcap_ce_bwd"):
        return sym, sym, "hbm", 2.0 * a[1] * a[2] * _esz(a[0]), PEAK_HBM_GBS, (a[1], a[2])
    if fn == "imgcap_ce_fwd":
        return sym, sym, "hbm", 1.0 * a[1] * a[2] * _esz(a[0]), PEAK_HBM_GBS, (a[1], a[2])
    if fn == "imgcap_add_layernorm_fwd":  # x (+ r) read, y (+ s_out) written
        n = a[1] * a[2] * _esz(a[0])
        return sym, sym, "hbm", n * (2 + (a[4] is not None) + (a[11] is not None)), PEAK_HBM_GBS, (a[1], a[2])
    if fn == "imgcap_add_layernorm_bwd":  # dy, s read, dx (+ dr) written (+ the per-block partials)
        n = a[1] * a[2]
        part = 0
        if a[15] is not None:  # [nblk][2][cols] fp32 gamma / beta partials (the caller's column sums)
            part = _abi.lib().imgcap_add_layernorm_bwd_blocks(a[1]) * 2 * a[2] * 4
        b = n * _esz(a[0]) * (3 + (a[12] is not None)) + part
        return sym, sym, "hbm", b, PEAK_HBM_GBS, (a[1], a[2])
    if fn == "imgcap_clamp_adam":  # p, g, m, v read; p, m, v written (fp32) + bf16 shadow written
        n = a[0]
        return sym, sym, "hbm", n * (7 * 4 + (2 if a[5] is not None else 0)), PEAK_HBM_GBS, (n,)
    if fn in ("imgcap_convnext_stem", "imgcap_convnext_stem_u8"):
        B, H, W, C0 = a[1], a[2], a[3], a[4]
        src = 1 if fn.endswith("u8") else 4
        return sym, sym, "hbm", B * 3 * H * W * src + B * (H // 4) * (W // 4) * C0 * _esz(a[0]), PEAK_HBM_GBS, \
            (B, H, W, C0)
    if fn in ("imgcap_ln_patchify2", "imgcap_ln_patchify2_bwd"):
        n = a[1] * a[2] * a[3] * a[4]
        return sym, sym, "hbm", (2.0 if fn == "imgcap_ln_patchify2" else 3.0) * n * _esz(a[0]), PEAK_HBM_GBS, \
            (a[1], a[2], a[3], a[4])
    if fn == "imgcap_transpose":
        return sym, sym, "hbm", 2.0 * a[1] * a[2] * _esz(a[0]), PEAK_HBM_GBS, (a[1], a[2])
    if fn == "imgcap_embedding_fwd":
        return sym, sym, "hbm", a[1] * a[2] * (4.0 + _esz(a[0])), PEAK_HBM_GBS, (a[1], a[2])
    if fn == "imgcap_embedding_bwd":
        return sym, sym, "hbm", a[1] * a[2] * (4.0 + _esz(a[0])), PEAK_HBM_GBS, (a[1], a[2])
    if fn == "imgcap_colsum_multi":
        arr = (_abi.ColsumItem * a[0]).from_address(a[1].value)
        return sym, sym, "hbm", float(sum(it.rows * it.cols * _esz(it.dtype) for it in arr)), PEAK_HBM_GBS, \
            (a[0], "items")
    if fn == "imgcap_mx_quant_rows":
        return sym, sym, "hbm", a[1] * a[2] * (_esz(a[0]) + 1 + 1 / 32), PEAK_HBM_GBS, (a[1], a[2])
    if fn == "imgcap_sort_gather_rows":
        return sym, sym, "hbm", 2.0 * a[1] * a[2] * a[3] * _esz(a[0]), PEAK_HBM_GBS, (a[1], a[2], a[3])
    if fn == "imgcap_dropout":
        return sym, sym, "hbm", 2.0 * a[1] * _esz(a[0]), PEAK_HBM_GBS, (a[1],)
    if fn == "imgcap_cast":
        return sym, sym, "hbm", a[2] * (_esz(a[0]) + _esz(a[1])), PEAK_HBM_GBS, (a[2],)
    return sym, sym, "latency", None, None, ()


def _timed_step(trainer, batch):
    """[(fn, args, seconds)] of every library call of one eager sequential train step."""
    rec = []
    orig = _abi.call

    def call(fn, *a):
        if fn in _NO_KERNEL:
            return orig(fn, *a)
        st = torch.cuda.current_stream()
        torch.cuda._sleep(SLEEP_CYCLES)  # the device waits here while the host queues the call
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(st)
        r = orig(fn, *a)
        e1.record(st)
        rec.append((fn, a, e0, e1))
        return r

    _abi.call = call
    try:
        trainer._fwd_bwd(*batch)
        # clip + Adam (the collectives of _update are left out: rank 0 alone runs this)
        trainer.eng.fp.adam_step(trainer.decoder_lr, trainer.grad_clip)
        if trainer.enc_eng is not None:
            trainer.enc_eng.fp.adam_step(trainer.encoder_lr, trainer.grad_clip)
    finally:
        _abi.call = orig
    torch.cuda.synchronize()
    return [(fn, a, e0.elapsed_time(e1) * 1e-3) for fn, a, e0, e1 in rec]


def kernel_table(trainer, batch, passes=3):
    """Per-kernel-symbol rows of one train step, ranked by time per step."""
    runs = [_timed_step(trainer, batch) for _ in range(passes)]
    base = runs[0]
    if any(len(r) != len(base) or any(x[0] != y[0] for x, y in zip(r, base)) for r in runs):
        raise RuntimeError("roofline: the step's library calls differ between passes")
    groups = collections.OrderedDict()
    for i, (fn, a, _) in enumerate(base):
        t = statistics.median(r[i][2] for r in runs)
        key, sym, bound, work, peak, shape = _work(fn, a)
        g = groups.setdefault(key, dict(name=key, symbol=sym, bound=bound, peak=peak, t=0.0, work=0.0, n=0,
                                         shapes=set(), fns=set()))
        g["t"] += t
        g["n"] += 1
        g["fns"].add(fn)
        if work is None or g["work"] is None:
            g["work"] = None
        else:
            g["work"] += work
        if len(g["shapes"]) < 8:
            g["shapes"].add(shape)
    rows = sorted(groups.values(), key=lambda g: -g["t"])
    step_t = sum(g["t"] for g in rows)
    for g in rows:
        g["share"] = g["t"] / step_t if step_t else 0.0
        if g["work"] is not None and g["t"] > 0:
            g["achieved"] = g["work"] / g["t"] / (1e9 if g["bound"] == "hbm" else 1e12)
            g["frac"] = g["achieved"] / g["peak"]
    return rows, step_t


def pmc_traffic(symbol, cfgname):
    """HBM bytes per launch of ``symbol`` from the committed rocprofv3 FETCH_SIZE / WRITE_SIZE
    summary of this config's bench run (profiles/*_<cfg>_pmc.json, tools/pmc_summary.py:
    gfx950-corrected, averaged over the kernel's dispatches), or None."""
    import glob
    import json
    import os
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    files = sorted(glob.glob(os.path.join(root, "profiles", f"*_{cfgname}_pmc.json")))
    if not files or not symbol:
        return None
    data = json.load(open(files[-1]))
    hits = [v for k, v in data.items() if symbol in k]
    if not hits:
        return None
    n = sum(h["dispatches"] for h in hits)
    return sum(h["traffic_bytes"] * h["dispatches"] for h in hits) / max(n, 1)


def pmc_sq(symbol, cfgname):
    """SQ counters of ``symbol`` from the committed rocprofv3 summary of this config's bench run
    (profiles/*_<cfg>_sq.json, tools/sq_summary.py): {mfma_busy, wait_frac, ...} or None."""
    import glob
    import json
    import os
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    files = sorted(glob.glob(os.path.join(root, "profiles", f"*_{cfgname}_sq.json")))
    if not files or not symbol:
        return None
    data = json.load(open(files[-1]))
    hits = [v for k, v in data.items() if symbol in k and "mfma_busy" in v]
    if not hits:
        return None
    n = sum(h["dispatches"] for h in hits)
    out = {"source": os.path.relpath(files[-1], root)}
    for key in ("mfma_busy", "wait_frac", "lds_conflict_per_inst"):
        if all(key in h for h in hits):
            out[key] = round(sum(h[key] * h["dispatches"] for h in hits) / max(n, 1), 4)
    return out


def measure(cfg, trainer, batch, cfgname=None):
    rows, step_t = kernel_table(trainer, batch)
    dump = os.environ.get("IMGCAP_ROOFLINE_TABLE")
    if dump:  # the whole ranked table (profiles/*_kernel_table.json)
        with open(dump, "w") as f:
            json.dump([{k: (sorted(map(str, v)) if isinstance(v, set) else v) for k, v in g.items()} for g in rows],
                      f, indent=1)
    modelled = [g for g in rows if g["work"] is not None]
    best = rows[0] if rows[0]["work"] is not None else modelled[0]
    t = best["t"] / best["n"]
    unit = "GB/s" if best["bound"] == "hbm" else "TFLOP/s"
    traffic = pmc_traffic(best["symbol"], cfgname) if cfgname else None
    return {"bound": best["bound"], "achieved": round(best["achieved"], 2), "peak": best["peak"], "unit": unit,
            "frac": round(best["frac"], 4), "traffic": None if traffic is None else round(traffic),
            "traffic_unit": "bytes/launch (rocprofv3 FETCH_SIZE x2 + WRITE_SIZE, profiles/)",
            "algorithmic": round(best["work"] / best["n"]),
            "algorithmic_unit": "bytes/launch" if best["bound"] == "hbm" else "FLOP/launch",
            "kernel": best["name"], "symbol": best["symbol"],
            "sq": pmc_sq(best["symbol"], cfgname) if cfgname else None,
            "avg_launch_us": round(t * 1e6, 2), "launches_per_step": best["n"],
            "share_of_kernel_time": round(best["share"], 4),
            "shape": f"{best['n']} launches/step, shapes {sorted(best['shapes'], key=str)[:6]}",
            "method": "every library call of one eager sequential step between HIP events on its own stream "
                      "(median of 3 steps), grouped by kernel symbol, ranked by time per step",
            "kernel_time_per_step_us": round(step_t * 1e6, 1),
            "ranked_us_per_step": {g["name"]: [round(g["t"] * 1e6, 1)] +
                                   ([round(g["frac"], 4)] if "frac" in g else []) for g in rows[:12]}}

"""Live roofline of the bench step's dominant kernel (bench.py ``roofline`` field).

Candidates are timed on the current HIP stream with HIP events around back-to-back launches
replayed from a HIP graph (so host launch cost does not hide short kernels), each with its
algorithmic work per launch:

  * every GEMM of one train step: the step runs once eagerly with ``kernels.record_gemms``
    collecting each ``imgcap_gemm`` call; the calls are grouped by the kernel that serves them
    (``imgcap_gemm_plan``: one group per kernel symbol, as rocprofv3 lists them) and each call
    is re-timed in isolation.  Work = 2*M*N*K per call; a group's achieved rate is
    sum(work) / sum(time), i.e. its average launch's work over its average launch duration.
  * the fused ConvNeXt MLP (cnblock_mlp) per stage width: 2 * 2 * M * C * 4C per launch.
  * the depthwise 7x7 per stage: HBM bytes = read x + write y (+ weights).

The dominant kernel is the group with the largest time per step; its rate is reported against
the MI355X peak (bf16 dense MFMA 2.5 PFLOP/s, HBM 8 TB/s; MI355X_MICROARCH.md).
"""
import collections

import torch

from . import kernels as K

PEAK_HBM_GBS = 8000.0
PEAK_BF16_TFLOPS = 2500.0
PEAK_FP8_TFLOPS = 5000.0  # dense block-scaled (MX) e4m3 MFMA

_KIND_NAME = {1: "gemm_skinny_kernel", 2: "gemm_kernel<64,64,64>", 3: "gemm_kernel<128,128,64>",
              4: "gemm_glds_kernel<128,128>", 5: "gemm256_kernel<256,256>", 6: "gemm_glds_kernel<64,64>",
              7: "gemm_glds_kernel<128,64>"}


def time_launch(fn, reps=50, warm=5, graph=True):
    """Seconds per launch of ``fn``, HIP events around ``reps`` back-to-back launches.  With
    graph=True the launches are captured into one HIP graph and replayed, so host launch cost
    (~10 us per ctypes call) does not hide short kernels -- the per-launch figure then matches
    the kernel durations rocprofv3 reports for the step (which also replays a graph)."""
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
    return a.elapsed_time(b) / reps * 1e-3  # seconds per launch


def _gemm_groups(trainer, batch):
    rec = []
    K.record_gemms(rec)
    try:
        trainer._fwd_bwd(*batch)
    finally:
        K.record_gemms(None)
    torch.cuda.synchronize()
    groups = collections.OrderedDict()
    for c in rec:
        if c.get("mx"):  # block-scaled fp8 (frozen encoder Linears of C5)
            g = groups.setdefault("gemm_mx_kernel (MX-FP8)", dict(name="gemm_mx_kernel (MX-FP8)", calls=[],
                                                                   bound="mfma", symbol="gemm_mx_kernel", mx=True))
            g["calls"].append(c)
            continue
        kind, splits = K.gemm_plan(c["dtype"], c["ak"], c["bk"], c["M"], c["N"], c["K"], c["lda"], c["ldb"], 1,
                                   c["split_k"])
        name = _KIND_NAME.get(kind, f"gemm kind {kind}")
        if kind in (2, 3, 4, 5, 6, 7):
            name += f"<ak={c['ak']},bk={c['bk']}>" + (" (split-K)" if splits > 1 else "")
        tf = lambda v: "true" if v else "false"  # noqa: E731
        sym = {4: f"gemm_glds_kernel<128, 128, {tf(c['ak'])}, {tf(c['bk'])}, ",  # any stage count
               5: f"gemm256_kernel<64, 2, {tf(c['ak'])}, {tf(c['bk'])}>",
               6: f"gemm_glds_kernel<64, 64, {tf(c['ak'])}, {tf(c['bk'])}, ",
               7: f"gemm_glds_kernel<128, 64, {tf(c['ak'])}, {tf(c['bk'])}, "}.get(kind, _KIND_NAME.get(kind, ""))
        g = groups.setdefault(name, dict(name=name, calls=[], bound="mfma", symbol=sym))
        g["calls"].append(c)
    out = []
    for g in groups.values():
        t_tot, f_tot, b_tot = 0.0, 0.0, 0.0
        for c in g["calls"]:
            t_tot += time_launch(c["call"], reps=20, warm=2)
            f_tot += 2.0 * c["M"] * c["N"] * c["K"]
            ct = c["keep"][-1].c_dtype
            cb = 4 if ct == 0 else 2 if ct == 1 else 1 + 1 / 32
            ab = (1 + 1 / 32) if c.get("mx") else 2.0  # operand bytes per element (MX: + its scale)
            b_tot += ab * (c["M"] + c["N"]) * c["K"] + cb * c["M"] * c["N"]  # A + B read, C written once
        n = len(g["calls"])
        shapes = sorted({(c["M"], c["N"], c["K"]) for c in g["calls"]})
        out.append(dict(name=g["name"], bound="mfma", per_step=n, t=t_tot / n, flops=f_tot / n, symbol=g["symbol"],
                        bytes=b_tot / n, peak=PEAK_FP8_TFLOPS if g.get("mx") else PEAK_BF16_TFLOPS,
                        note=f"{n} launches/step, shapes (M,N,K) {shapes[:6]}{' ...' if len(shapes) > 6 else ''}"))
    return out


def _encoder_groups(trainer, B, dev):
    enc = trainer.encoder
    if enc.compute_dtype != torch.bfloat16:
        return []
    pk = enc._pack()
    out = []
    hw = 56
    for st, (blocks, _) in enumerate(pk["stages"]):
        blk = blocks[0]
        C = blk["w1"].shape[1]
        M = B * hw * hw
        x = torch.randn(B, hw, hw, C, device=dev).to(torch.bfloat16)
        y = torch.empty_like(x)
        if C in K.CNBLOCK_MLP_CHANNELS:
            x2 = x.view(M, C)
            z = y.view(M, C)

            def mlp(blk=blk, z=z, x2=x2):
                K.cnblock_mlp(z, blk["w1"], blk["b1"], blk["w2"], blk["b2"], blk["gamma"], x2, ln_w=blk["lnw"],
                              ln_b=blk["lnb"])
            kname = "cnblock_mlp_res_kernel" if C == 96 else "cnblock_mlp_str_kernel"  # csrc/cnblock_mlp.hip
            out.append(dict(name=f"{kname}<{C}> (stage {st + 1} fused MLP)", bound="mfma",
                            symbol=f"{kname}<{C}>", bytes=3.0 * M * C * 2 + 2 * 4 * C * C * 2,
                            per_step=len(blocks), t=time_launch(mlp, reps=20), flops=2.0 * 2 * M * C * 4 * C,
                            note=f"M={M} C={C}: LN + Linear C->4C + GELU + Linear 4C->C + scale + residual"))
        if hw <= 64:
            def dw(blk=blk, x=x, y=y):
                K.dwconv7(x, blk["w49"], blk["dwb"], y)
            out.append(dict(name=f"dwconv7_kernel (stage {st + 1}, C={C})", bound="hbm", per_step=len(blocks),
                            symbol="dwconv7_kernel",
                            t=time_launch(dw, reps=20), bytes=2.0 * M * C * 2 + 49 * C * 4,
                            note=f"B*H*W={M} C={C}: read x + write y (bf16)"))
        hw //= 2
    return out


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
    dev = batch[0].device
    B = batch[0].shape[0]
    cands = _gemm_groups(trainer, batch) + _encoder_groups(trainer, B, dev)
    for c in cands:
        c["share"] = c["t"] * c["per_step"]
    best = max(cands, key=lambda c: c["share"])
    t = best["t"]
    if best["bound"] == "hbm":
        achieved = best["bytes"] / t / 1e9
        peak, unit = PEAK_HBM_GBS, "GB/s"
    else:
        achieved = best["flops"] / t / 1e12
        peak, unit = best.get("peak", PEAK_BF16_TFLOPS), "TFLOP/s"
    ranked = sorted(cands, key=lambda c: -c["share"])
    traffic = pmc_traffic(best.get("symbol"), cfgname) if cfgname else None
    return {"bound": best["bound"], "achieved": round(achieved, 2), "peak": peak, "unit": unit,
            "frac": round(achieved / peak, 4), "traffic": None if traffic is None else round(traffic),
            "traffic_unit": "bytes/launch (rocprofv3 FETCH_SIZE x2 + WRITE_SIZE, profiles/)",
            "algorithmic_bytes": round(best["bytes"]) if "bytes" in best else None,
            "kernel": best["name"],
            # SIMD-cycle share of the matrix pipe while the kernel ran (rocprofv3 SQ counters)
            "sq": pmc_sq(best.get("symbol"), cfgname) if cfgname else None,
            "avg_launch_us": round(t * 1e6, 2), "launches_per_step": best["per_step"], "shape": best["note"],
            "others_us_per_step": {c["name"]: round(c["share"] * 1e6, 1) for c in ranked[1:8]}}

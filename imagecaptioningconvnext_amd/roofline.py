"""Live roofline of the bench step's dominant kernel (bench.py ``roofline`` field).

Each candidate below replays ONE kernel launch of the step with the step's own shapes on the
current HIP stream, timed with HIP events over ``reps`` back-to-back launches; its algorithmic
traffic/work per launch is stated next to it.  The dominant kernel is the
candidate with the largest (avg launch time x launches per step); its achieved rate is reported
against the MI355X peak (HBM 8 TB/s, bf16 MFMA 2.5 PF/s dense).
"""
import torch

from . import kernels as K

PEAK_HBM_GBS = 8000.0
PEAK_BF16_TFLOPS = 2500.0


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


def _candidates_lstm(trainer, B, dev):
    eng = trainer.eng
    E, A, D, W3 = eng.E, eng.A, eng.D, eng.W3
    w = eng.weights()
    ct = eng.ct
    es = 2 if ct == torch.bfloat16 else 4
    h = torch.randn(B, D, device=dev).to(ct)
    g1 = torch.empty(B, W3, device=dev)
    cands = []

    def g1_gemm():
        K.gemm(h, w["hcat"], trans_b=True, bias=w["bhcat"], out=g1)

    cands.append(dict(name="gemm_skinny (LSTM step: h_{t-1} -> [att2|gate|hh])", fn=g1_gemm, per_step=51,
                      bound="hbm", bytes=W3 * D * es + B * D * es + B * W3 * 4,
                      note=f"M={B} N={W3} K={D}: weight stream W3*D*2 B + A + fp32 C per launch"))
    return cands


def _candidates_encoder(trainer, B, dev):
    enc = trainer.encoder
    pk = enc._pack()
    blk = pk["stages"][0][0][0]
    C = blk["w1"].shape[1]
    Mrows = B * 56 * 56
    z = torch.randn(Mrows, C, device=dev).to(enc.compute_dtype)
    hid = torch.empty(Mrows, 4 * C, device=dev, dtype=enc.compute_dtype)
    x = torch.randn(B, 56, 56, C, device=dev).to(enc.compute_dtype)
    y = torch.empty_like(x)
    cands = []

    def pw1():
        K.gemm(z, blk["w1"], trans_b=True, bias=blk["b1"], act=K.ACT_GELU, out=hid)

    cands.append(dict(name="gemm_kernel 128x128 (ConvNeXt stage-1 pointwise Linear C->4C + GELU)", fn=pw1,
                      per_step=3, bound="mfma", flops=2 * Mrows * C * 4 * C,
                      note=f"M={Mrows} N={4 * C} K={C}"))

    def dw():
        K.dwconv7_ln(x, blk["w49"], blk["dwb"], blk["lnw"], blk["lnb"], y)

    es = 2 if enc.compute_dtype == torch.bfloat16 else 4
    cands.append(dict(name="dwconv7_ln (ConvNeXt stage-1 depthwise 7x7 + LayerNorm)", fn=dw, per_step=3,
                      bound="hbm", bytes=2 * Mrows * C * es + 49 * C * 4,
                      note=f"B*H*W={Mrows} C={C}: read x + write y"))
    return cands


def measure(cfg, trainer, batch):
    dev = batch[0].device
    B = batch[0].shape[0]
    cands = _candidates_encoder(trainer, B, dev)
    if cfg["decoder"] == "lstm":
        cands += _candidates_lstm(trainer, B, dev)
    best = None
    for c in cands:
        t = time_launch(c["fn"])
        c["t"] = t
        c["share"] = t * c["per_step"]
        if best is None or c["share"] > best["share"]:
            best = c
    t = best["t"]
    if best["bound"] == "hbm":
        achieved = best["bytes"] / t / 1e9
        peak, unit = PEAK_HBM_GBS, "GB/s"
    else:
        achieved = best["flops"] / t / 1e12
        peak, unit = PEAK_BF16_TFLOPS, "TFLOP/s"
    return {"bound": best["bound"], "achieved": round(achieved, 2), "peak": peak, "unit": unit,
            "frac": round(achieved / peak, 4), "traffic": None, "kernel": best["name"],
            "avg_launch_us": round(t * 1e6, 2), "launches_per_step": best["per_step"], "shape": best["note"],
            "others": {c["name"]: round(c["t"] * 1e6, 2) for c in cands if c is not best}}

"""Teacher-forced train-step throughput (images/sec) on MI355X — BASELINE.json's metric.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--config C2|C3|C4|C5]
    python -m torch.distributed.run --nproc-per-node N --master-addr 127.0.0.1 ... bench.py --gpus N

``--gpus N`` without a launcher (no WORLD_SIZE in the environment) starts the N rank processes
itself, before anything touches the GPU, and exits with their status.

Default workload = BASELINE.json configs[2] (C3), the largest single-GPU configuration (the
metric names no config): ConvNeXt-Tiny encoder (frozen, train mode) + Transformer decoder,
teacher forced, 64 images per GPU, 224x224x3, captions of length 52, vocab 9490, bf16 compute /
fp32 master weights + Adam.  --config C2 (Tiny + LSTM, B=32), C4, C5 select the others.  One step =
the full train.py:251-299 body (encoder fwd, decoder fwd, CE + alpha reg, backward, RCCL grad
all-reduce when N > 1, clip + Adam, metrics).  Synthetic data, pre-generated in HBM; weights
randomly initialised (no network).  Per-GPU work is fixed as N grows ("scaling": "weak").
Rank 0 prints ONE JSON line.
"""
import argparse
import json
import math
import os
import sys
import time

import torch
import torch.distributed as dist

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

V = 9490
CAPLEN = 52
CONFIGS = {
    "C2": dict(encoder="tiny", decoder="lstm", batch=32),
    "C3": dict(encoder="tiny", decoder="transformer", batch=64),
    "C4": dict(encoder="base", decoder="transformer", batch=32),
    # ConvNeXt-Large + Transformer, encoder fine-tuned from startingLayer=7 (stage 4 trains)
    "C5": dict(encoder="large", decoder="transformer", batch=64, starting_layer=7, frozen_fp8=True),
}
PEAK_BF16_TFLOPS = 2500.0   # MI355X dense bf16 MFMA (MI355X_MICROARCH.md)
PEAK_FP8_TFLOPS = 5000.0    # dense block-scaled e4m3 MFMA
PEAK_HBM_GBS = 8000.0       # HBM3E spec


def parse(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--warmup", type=int, default=10)
    ap.add_argument("--config", default="C3", choices=sorted(CONFIGS))
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-graph", action="store_true", help="launch eagerly instead of replaying a HIP graph")
    ap.add_argument("--cpu-seconds", type=float, default=15.0)
    ap.add_argument("--no-pipeline", action="store_true",
                    help="run encoder and decoder of a step back to back (no two-stream overlap)")
    ap.add_argument("--no-fp8", action="store_true", help="C5: frozen encoder GEMMs in bf16 instead of MX-FP8")
    ap.add_argument("--lengths", choices=("full", "coco"), default="full",
                    help="caption lengths of the synthetic batches: all 52 (default) or COCO-like")
    ap.add_argument("--no-len-buckets", action="store_true",
                    help="LSTM: always run L - 1 steps (no length buckets)")
    ap.add_argument("--no-roofline", action="store_true",
                    help="skip the per-call roofline pass (profiling the replays alone); roofline is then null")
    ap.add_argument("--launch-selftest", action="store_true",
                    help="launcher check on CPU: gloo ranks time an empty step (tests/test_bench_cpu.py); "
                         "prints the rank layout, not a measurement")
    return ap.parse_args(argv)


def spawn_ranks(n, argv):
    """One process per GPU (rank r on GPU r), the torchrun environment set by hand; returns the
    first non-zero exit status (the other ranks are terminated then) or 0."""
    import socket
    import subprocess
    with socket.socket() as sk:
        sk.bind(("127.0.0.1", 0))
        port = sk.getsockname()[1]
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + list(argv), env=env))
    rc = 0
    pending = list(procs)
    while pending:
        for p in list(pending):
            code = p.poll()
            if code is None:
                continue
            pending.remove(p)
            if code != 0 and rc == 0:
                rc = code
                for q in pending:  # a dead rank would leave the others blocked in a collective
                    q.terminate()
        time.sleep(0.05)
    return rc


def synthetic_batch(B, rank, step, device, lengths="full"):
    """U[0,1) images ImageNet-normalised; caps <start> w.. <end>, caplen 52.
    lengths="coco": caption lengths drawn like COCO's (about 10.5 +- 2.5 words + <start>/<end>,
    clipped to [8, 52]; padded with 0 past the length, as dataLoader.py's encoded captions).
    Returns (img, caps, caplens, max_caplen) -- the last known on the host."""
    g = torch.Generator(device="cpu").manual_seed(1234 + 7919 * rank + step)
    img = torch.rand(B, 3, 224, 224, generator=g)
    mean = torch.tensor([0.485, 0.456, 0.406]).view(1, 3, 1, 1)
    std = torch.tensor([0.229, 0.224, 0.225]).view(1, 3, 1, 1)
    img = (img - mean) / std
    caps = torch.randint(1, V - 3, (B, CAPLEN), generator=g)
    caps[:, 0] = V - 2
    if lengths == "coco":
        lens = (torch.randn(B, generator=g) * 2.5 + 12.5).round().clamp(8, CAPLEN).long()
    else:
        lens = torch.full((B,), CAPLEN, dtype=torch.int64)
    for b in range(B):
        caps[b, lens[b] - 1] = V - 1
        caps[b, lens[b]:] = 0
    caplens = lens.view(B, 1)
    return img.to(device), caps.to(device), caplens.to(device), int(lens.max())


def build(cfg, device):
    from imagecaptioningconvnext_amd.models.decoder import DecoderWithAttention
    from imagecaptioningconvnext_amd.models.encoder import Encoder
    enc = Encoder(variant=cfg["encoder"], compute_dtype=torch.bfloat16, frozen_fp8=cfg.get("frozen_fp8", False))
    enc = enc.to(device)
    if "starting_layer" in cfg:
        enc.fine_tune(True, startingLayer=cfg["starting_layer"])
    else:
        enc.fine_tune(False)
    E = enc.encoder_dim
    if cfg["decoder"] == "lstm":
        dec = DecoderWithAttention(attention_dim=512, embed_dim=512, decoder_dim=512, vocab_size=V, device=device,
                                   encoder_dim=E, dropout=0.5, compute_dtype=torch.bfloat16).to(device)
    else:
        from imagecaptioningconvnext_amd.models.transformerDecoder import TransformerDecoder
        dec = TransformerDecoder(embed_dim=512, decoder_dim=512, vocab_size=V, maxLen=CAPLEN, device=device,
                                 wordMap=None, pretrained_embeddings_path=None, fine_tune_embeddings=True,
                                 dropout=0.5, encoder_dim=E, compute_dtype=torch.bfloat16).to(device)
    return enc, dec


def fp8_flops_per_image(cfg, enc):
    """FLOPs per image of the frozen CNBlock Linears that run in MX-FP8 (the rest is bf16)."""
    if not enc.frozen_fp8:
        return 0
    from imagecaptioningconvnext_amd.models.encoder import VARIANTS
    chans, depths, _ = VARIANTS[cfg["encoder"]]
    start = cfg.get("starting_layer", 8)
    f, h = 0, 56
    for st in range(4):
        C = chans[st]
        if 1 + 2 * st < start and enc._mx_stage(C):
            f += 2 * depths[st] * 2 * h * h * C * 4 * C
        h //= 2
    return f


def flops_per_image(cfg, enc):
    """Algorithmic FLOPs per image: encoder fwd (+ 2x fwd for the fine-tuned
    children's backward) + 3x decoder fwd."""
    enc_macs = enc.macs_per_image(224)
    if "starting_layer" in cfg:
        enc_macs += 2 * enc.macs_per_image(224, start=cfg["starting_layer"])
    T, E, A, D, M = CAPLEN - 1, enc.encoder_dim, 512, 512, 512
    if cfg["decoder"] == "lstm":
        P = 49
        dec_macs = (P * E * A                      # att1 (hoisted)
                    + T * (D * (A + E + 4 * D)     # h -> [att2 | gate | hh]
                           + P * A + P * E         # scores + context
                           + E * 4 * D + M * 4 * D  # LSTMCell input GEMMs
                           + D * V)                # fc
                    + E * 2 * D)                   # init_h / init_c
    else:
        L, d, ff, layers, P = CAPLEN, 512, 512, 6, 49
        per_layer = L * (3 * d * d + d * d) + L * L * d * 2 + L * d * d + P * d * 2 * d + L * P * d * 2 \
            + L * d * d + 2 * L * d * ff
        dec_macs = P * E * d + layers * per_layer + L * d * V
    return 2 * enc_macs + 3 * 2 * dec_macs


def cpu_model():
    """The host CPU's model name (lscpu's "Model name", read from /proc/cpuinfo)."""
    try:
        with open("/proc/cpuinfo") as f:
            for ln in f:
                if ln.startswith("model name"):
                    return ln.split(":", 1)[1].strip()
    except OSError:
        pass
    import platform
    return platform.processor() or None


def physical_cores():
    """Physical cores this process may run on: distinct (package, core) pairs of the CPUs in its
    affinity mask (/proc/cpuinfo), capped by the cgroup CPU quota (cpu.max) when one is set --
    the GPU box grants each GPU a share of a larger host.  Returns (cores, detail)."""
    cpus = sorted(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else list(range(os.cpu_count() or 1))
    pairs, cur = {}, {}
    try:
        with open("/proc/cpuinfo") as f:
            for ln in f:
                if ":" not in ln:
                    if "processor" in cur:
                        pairs[cur["processor"]] = (cur.get("physical id", "0"), cur.get("core id", cur["processor"]))
                    cur = {}
                    continue
                k, v = (s.strip() for s in ln.split(":", 1))
                cur[k] = v
        if "processor" in cur:
            pairs[cur["processor"]] = (cur.get("physical id", "0"), cur.get("core id", cur["processor"]))
    except OSError:
        pass
    phys = len({pairs.get(str(c), (None, c)) for c in cpus}) or len(cpus)
    quota = None
    try:
        with open("/sys/fs/cgroup/cpu.max") as f:
            q, p = f.read().split()[:2]
            if q != "max":
                quota = max(1, int(int(q) / int(p)))
    except (OSError, ValueError):
        pass
    cores = min(phys, quota) if quota else phys
    return cores, f"{phys} physical cores in the affinity mask ({len(cpus)} logical)" + (
        f", cgroup quota {quota} CPUs" if quota else "")


def cpu_baseline(seconds):
    """Oracle (plain PyTorch CPU restatement) of the C1 train step: Tiny + LSTM, B=4, fp32."""
    from oracle import convnext, decoders, shapes, train_step
    nthreads, core_detail = physical_cores()
    torch.set_num_threads(nthreads)
    B, E = 4, 768
    sd = convnext.init_params("tiny")
    g = torch.Generator().manual_seed(0)
    p = {k: (torch.rand(s, generator=g) * 0.2 - 0.1) for k, s in shapes.lstm_decoder_shapes(E, 512, 512, 512, V).items()}
    state = {}
    img, caps, caplens, _ = synthetic_batch(B, 0, 0, "cpu")
    t_steps, n = 0.0, 0
    step = 0
    while True:
        t0 = time.perf_counter()
        with torch.no_grad():
            feats = convnext.encoder_forward(sd, "tiny", img)
        pr = {k: v.clone().requires_grad_(True) for k, v in p.items()}
        preds, cs, dls, al, _ = decoders.lstm_tf_forward(pr, feats, caps, caplens)
        loss, _, _ = train_step.lstm_loss(preds, cs, dls, al)
        loss.backward()
        step += 1
        p = train_step.adam_step(p, train_step.clip_gradient({k: v.grad for k, v in pr.items()}, 5.0), state,
                                 1e-4, step)
        dt = time.perf_counter() - t0
        if step > 1:  # first step is warm-up
            t_steps += dt
            n += 1
        if (t_steps >= seconds and n >= 2) or step >= 50:
            break
    return dict(value=round(B * n / t_steps, 3), unit="images/s", cores=nthreads, cores_detail=core_detail,
                kind="port", cpu=cpu_model(),
                sample=f"oracle C1 train step (ConvNeXt-Tiny + LSTM-attention, B=4, fp32, 224x224, L=52, "
                       f"V={V}), {n} timed steps after 1 warm-up, {t_steps:.1f} s")


def launch_selftest(args, rank, world):
    """The bench's rank/timing protocol around an empty step (gloo, CPU)."""
    dist.barrier()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        pass
    dist.barrier()
    t = torch.tensor([time.perf_counter() - t0], dtype=torch.float64)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    if rank == 0:
        print(json.dumps({"launch_selftest": True, "n_gpus": dist.get_world_size(), "steps": args.steps,
                          "max_elapsed_s": t.item()}), flush=True)
    dist.barrier()
    dist.destroy_process_group()


def main(argv=None):
    raw = sys.argv[1:] if argv is None else list(argv)
    args = parse(raw)
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(spawn_ranks(args.gpus, raw))
    cfg = dict(CONFIGS[args.config])
    if args.no_fp8:
        cfg["frozen_fp8"] = False
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus and rank == 0:
        print(f"bench.py: --gpus {args.gpus} but WORLD_SIZE={world}; running {world} ranks", file=sys.stderr)
    if args.launch_selftest:
        dist.init_process_group("gloo", init_method="env://", world_size=world, rank=rank)
        return launch_selftest(args, rank, world)
    if world > 1:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        torch.cuda.set_device(local)
        dist.init_process_group("nccl", init_method="env://", world_size=world, rank=rank,
                                device_id=torch.device("cuda", local))
        world = dist.get_world_size()
    device = torch.device("cuda", local)
    torch.manual_seed(42 + rank)
    from imagecaptioningconvnext_amd.train_step import TeacherForcedTrainer
    enc, dec = build(cfg, device)
    # frozen encoder: its forward for batch i+1 overlaps the decoder step of batch i (two
    # streams in one graph); every timed step still does one encoder + one decoder pass
    pipeline = not args.no_pipeline and "starting_layer" not in cfg
    trainer = TeacherForcedTrainer(enc, dec, lstm=cfg["decoder"] == "lstm", graph=not args.no_graph,
                                   pipeline=pipeline, len_buckets=not args.no_len_buckets)
    B = cfg["batch"]
    batches = [synthetic_batch(B, rank, i, device, args.lengths) for i in range(4)]
    for i in range(args.warmup):
        trainer.step(*batches[i % 4][:3], max_caplen=batches[i % 4][3])
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    progress = os.environ.get("IMGCAP_BENCH_PROGRESS") == "1"  # diagnostics: a synchronised mark per 10 steps
    t0 = time.perf_counter()
    for i in range(args.steps):
        trainer.step(*batches[i % 4][:3], max_caplen=batches[i % 4][3])
        if progress and i % 10 == 9:
            torch.cuda.synchronize()
            print(f"[bench] step {i + 1}/{args.steps}", file=sys.stderr, flush=True)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([elapsed], device=device, dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = t.item()
    metrics = trainer.drain_metrics()
    ms = elapsed / args.steps * 1e3
    imgs_per_s = B * world * args.steps / elapsed
    fpi = flops_per_image(cfg, enc)
    fp8_fpi = fp8_flops_per_image(cfg, enc)
    if rank == 0:
        from imagecaptioningconvnext_amd import roofline
        if progress:
            print("[bench] roofline", file=sys.stderr, flush=True)
        roof = None if args.no_roofline else roofline.measure(cfg, trainer, batches[0][:3], cfgname=args.config)
        if progress:
            print("[bench] roofline done", file=sys.stderr, flush=True)
        out = {
            "metric": "images/sec (train step, teacher-forced)",
            "value": round(imgs_per_s, 2),
            "unit": "images/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(ms, 3),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "bf16" + (" + MX-FP8 (e4m3, 32-element E8M0 block scales) frozen encoder Linears"
                               if fp8_fpi else ""),
            "pipeline": "encoder(batch i+1) || decoder fwd/bwd(batch i), two HIP streams in one graph"
                        if pipeline else "sequential",
            "data": "synthetic (224x224x3 U[0,1) ImageNet-normalised, random captions " +
                    ("len 52" if args.lengths == "full" else "of COCO-like lengths (12.5 +- 2.5 tokens, <= 52)") +
                    "), random-init weights",
            "config": {"workload": f"{args.config}: ConvNeXt-{cfg['encoder'].capitalize()} "
                                   f"({'fine-tuned from child %d' % cfg['starting_layer'] if 'starting_layer' in cfg else 'frozen'}) + "
                                   f"{'LSTM-attention' if cfg['decoder'] == 'lstm' else 'Transformer'} decoder, "
                                   f"teacher-forced train step",
                       "per_gpu_batch": B, "global_batch": B * world, "image": 224, "caption_len": CAPLEN,
                       "vocab": V, "parallelism": f"dp{world}"},
            "step_flops_per_image": fpi,
            # mixed peak for fp8 configs: ideal = F_fp8 / 5 PF + F_bf16 / 2.5 PF
            "step_mfma_frac": round(imgs_per_s * (fp8_fpi / PEAK_FP8_TFLOPS + (fpi - fp8_fpi) / PEAK_BF16_TFLOPS)
                                    / (world * 1e12), 5),
            "last_loss": round(metrics[-1][0], 5) if metrics else None,
            "last_top5": round(metrics[-1][2], 4) if metrics else None,
            "roofline": roof,
        }
        if not args.no_cpu_baseline and world == 1:
            out["cpu_baseline"] = cpu_baseline(args.cpu_seconds)
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()

"""Two-rank DDP train step with the Transformer decoder and a trainable encoder
(trainMultiGPU.py:233-235 decoder DDP, :256 encoder DDP once fine-tuning, :384-394 backward ->
averaged gradients -> clip -> both Adams), driven through TeacherForcedTrainer.

mode "oracle" (CPU, gloo): the engines are CPU stand-ins whose forward / backward / Adam are the
oracle's (test infrastructure only): the Transformer decoder of oracle/decoders.py and a
per-channel affine "encoder" (feats = x * w + b: trainable parameters with their own flat
buffer, Adam at encoder_lr, gradient from the decoder's dL/d encoder_out) -- exercises the
trainer's broadcasts, the per-layer decoder buckets, the decoder's rest reduced before the encoder backward,
the encoder's bucket reduced inside its backward, the unbucketed rest and grad_div.  ``expected`` is the oracle's single-process averaged step.
mode "hip" (GPU box): ConvNeXt-Tiny with children[7:] trainable + the HIP Transformer engine,
both ranks on the one GPU, gloo carrying the all-reduces.
"""
import os

import torch
import torch.distributed as dist
from safetensors.torch import load_file, save_file

from golden_util import make_captions, make_features, make_params

CFG = dict(E=32, d=16, ff=32, V=60, layers=2, H=2, L=10, B=3)
LR_DEC, LR_ENC, CLIP = 1e-3, 2e-3, 5.0


def shard(rank):
    """Rank r's batch: encoder inputs [B, 7, 7, E] (the affine encoder's x), captions, lengths."""
    c = CFG
    x = make_features((c["B"], 7, 7, c["E"]), 300 + rank)
    lens = [[10, 7, 4], [9, 9, 6]][rank]
    caps, caplens = make_captions(c["B"], c["L"], lens, c["V"], 310 + rank)
    return x, caps, caplens


def init_params(rank):
    from oracle import shapes
    c = CFG
    dec = make_params(shapes.transformer_decoder_shapes(c["E"], c["d"], c["ff"], c["V"], c["layers"]), 320)
    g = torch.Generator().manual_seed(330)
    enc = {"w": 1.0 + 0.2 * torch.rand(c["E"], generator=g), "b": 0.1 * torch.rand(c["E"], generator=g)}
    if rank:  # rank 1 starts elsewhere: the trainer must broadcast rank 0's weights (DDP init)
        dec = {k: v + 0.25 for k, v in dec.items()}
        enc = {k: v - 0.5 for k, v in enc.items()}
    return dec, enc


def _loss(dp, ep, x, caps, caplens):
    from oracle import decoders, train_step
    c = CFG
    feats = x * ep["w"] + ep["b"]
    preds, cs, dls = decoders.transformer_tf_forward(dp, feats, caps, caplens, caps == 0, c["H"], c["layers"])
    loss, scores, targets = train_step.transformer_loss(preds, cs, dls)
    return loss, scores, targets, dls


class _OracleFlat:
    def __init__(self, params):
        self.names = list(params)
        self.shapes = {n: params[n].shape for n in self.names}
        self.flat = torch.cat([params[n].reshape(-1) for n in self.names]).clone()
        self.grad = torch.zeros_like(self.flat)
        self.state, self.t = {}, 0

    def views(self, buf):
        out, o = {}, 0
        for n in self.names:
            k = self.shapes[n].numel()
            out[n] = buf[o:o + k].view(self.shapes[n])
            o += k
        return out

    def refresh_shadow(self):
        pass

    def adam_step(self, lr, clip, grad_div=1.0, skip=None):
        from oracle import train_step
        self.t += 1
        if skip is not None and float(skip.reshape(-1)[0]) != 0.0:  # FlatParams.adam_step's gate
            return
        g = {n: v / grad_div for n, v in self.views(self.grad).items()}
        p = {n: v.clone() for n, v in self.views(self.flat).items()}
        new = train_step.adam_step(p, train_step.clip_gradient(g, clip), self.state, lr, self.t)
        for n, v in self.views(self.flat).items():
            v.copy_(new[n])


class _OracleTransformerEngine:
    def __init__(self, params):
        self.fp = _OracleFlat(params)

    def forward(self, feats, caps, caplens, pad_id=0):
        from oracle import decoders, train_step
        c = CFG
        pr = {n: v.clone().requires_grad_(True) for n, v in self.fp.views(self.fp.flat).items()}
        f = feats.detach().clone().requires_grad_(True)
        preds, cs, dls = decoders.transformer_tf_forward(pr, f, caps, caplens, caps == pad_id, c["H"], c["layers"])
        loss, scores, targets = train_step.transformer_loss(preds, cs, dls)
        hits = float(train_step.top5_correct(scores, targets))
        return dict(loss=loss, pr=pr, feats=f, metrics=torch.tensor([loss.item(), float(sum(dls)), hits]))

    def early_bucket(self):  # the embedding's range (as the HIP engine's)
        fp = self.fp
        lo = 0
        for n in fp.names:
            if n == "embedding.weight":
                return lo, lo + fp.shapes[n].numel()
            lo += fp.shapes[n].numel()
        raise KeyError("embedding.weight")

    def grad_buckets(self):  # one per layer, the last first (as the HIP engine's)
        fp, out = self.fp, []
        for i in reversed(range(CFG["layers"])):
            pre, lo, span = f"transformer_decoder.layers.{i}.", 0, []
            for n in fp.names:
                k = fp.shapes[n].numel()
                if n.startswith(pre):
                    span.append((lo, lo + k))
                lo += k
            out.append((span[0][0], span[-1][1]))
        return out

    def backward(self, s, want_denc=False, bucket_hook=None):
        s["loss"].backward()
        for n, v in self.fp.views(self.fp.grad).items():
            v.copy_(s["pr"][n].grad)
        s["denc"] = s["feats"].grad if want_denc else None
        if bucket_hook is not None:
            for _ in range(CFG["layers"]):
                bucket_hook()


class _OracleDecoder(torch.nn.Module):
    def __init__(self, params):
        super().__init__()
        self._eng = _OracleTransformerEngine(params)

    def engine(self):
        return self._eng


class _AffineEngine:
    def __init__(self, enc):
        self.enc = enc
        self.fp = _OracleFlat({"w": enc.w.data, "b": enc.b.data})

    def forward(self, x):
        v = self.fp.views(self.fp.flat)
        return x * v["w"] + v["b"], dict(x=x)

    def grad_buckets(self):  # "b" (final first); "w" is left to the trainer's update
        E = self.fp.shapes["w"].numel()
        return [(E, E + self.fp.shapes["b"].numel())]

    def backward(self, saved, dfeat, bucket_hook=None):
        g = self.fp.views(self.fp.grad)
        x = saved["x"]
        g["b"].copy_(dfeat.reshape(-1, x.shape[-1]).sum(0))
        if bucket_hook is not None:
            bucket_hook()
        g["w"].copy_((dfeat * x).reshape(-1, x.shape[-1]).sum(0))


class _AffineEncoder(torch.nn.Module):
    """Encoder stand-in with trainable parameters (the trainer's fine-tuned-encoder surface)."""

    def __init__(self, params):
        super().__init__()
        self.w = torch.nn.Parameter(params["w"].clone())
        self.b = torch.nn.Parameter(params["b"].clone())
        self._eng = None

    def trainable(self):
        return True

    def engine(self):
        if self._eng is None:
            self._eng = _AffineEngine(self)
        return self._eng


def worker(rank, world, initfile, outdir, bucketed):
    from imagecaptioningconvnext_amd.train_step import TeacherForcedTrainer
    torch.set_num_threads(2)
    dist.init_process_group("gloo", init_method="file://" + initfile, rank=rank, world_size=world)
    dp, ep = init_params(rank)
    tr = TeacherForcedTrainer(_AffineEncoder(ep), _OracleDecoder(dp), lstm=False, decoder_lr=LR_DEC,
                              encoder_lr=LR_ENC, grad_clip=CLIP)
    # fine-tuning: one bucket per decoder layer, the decoder's rest, then the encoder's bucket
    assert [f is tr.eng.fp for f, _ in tr._buckets] == [True] * (CFG["layers"] + 1) + [False]
    if not bucketed:
        tr._buckets = None
    tr.step(*shard(rank))
    (loss, tokens, top5), = tr.drain_metrics()
    out = {"dec." + n: v.clone() for n, v in tr.eng.fp.views(tr.eng.fp.flat).items()}
    out.update({"enc." + n: v.clone() for n, v in tr.enc_eng.fp.views(tr.enc_eng.fp.flat).items()})
    out["metrics"] = torch.tensor([loss, tokens, top5], dtype=torch.float64)
    save_file(out, os.path.join(outdir, f"rank{rank}.safetensors"))
    dist.barrier()
    dist.destroy_process_group()


def run(tmpdir, bucketed=True, world=2):
    import torch.multiprocessing as mp
    os.makedirs(str(tmpdir), exist_ok=True)
    initfile = os.path.join(str(tmpdir), "init")
    mp.spawn(worker, args=(world, initfile, str(tmpdir), bucketed), nprocs=world, join=True)
    return [load_file(os.path.join(str(tmpdir), f"rank{r}.safetensors")) for r in range(world)]


def expected():
    """The oracle's averaged step from rank 0's weights: mean over ranks of each rank's
    token-mean loss gradient (DDP), clip, Adam per optimizer; the reduced metrics."""
    from oracle import train_step
    dp, ep = init_params(0)
    gd, ge = {}, {}
    num, tok, hits = 0.0, 0.0, 0.0
    for r in range(2):
        d = {n: v.clone().requires_grad_(True) for n, v in dp.items()}
        e = {n: v.clone().requires_grad_(True) for n, v in ep.items()}
        loss, scores, targets, dls = _loss(d, e, *shard(r))
        loss.backward()
        for n in d:
            gd[n] = gd.get(n, 0) + d[n].grad / 2
        for n in e:
            ge[n] = ge.get(n, 0) + e[n].grad / 2
        num += loss.item() * sum(dls)
        tok += sum(dls)
        hits += train_step.top5_correct(scores, targets)
    post_d = train_step.adam_step(dp, train_step.clip_gradient(gd, CLIP), {}, LR_DEC, 1)
    post_e = train_step.adam_step(ep, train_step.clip_gradient(ge, CLIP), {}, LR_ENC, 1)
    return post_d, post_e, (num / tok, tok, hits / tok * 100.0)


def check(results, rtol=1e-5, atol=1e-6):
    r0, r1 = results
    for k in r0:
        torch.testing.assert_close(r0[k], r1[k], rtol=0, atol=0)  # the ranks agree exactly
    post_d, post_e, (loss, tokens, top5) = expected()
    for n, v in post_d.items():
        torch.testing.assert_close(r0["dec." + n], v, rtol=rtol, atol=atol)
    for n, v in post_e.items():
        torch.testing.assert_close(r0["enc." + n], v, rtol=rtol, atol=atol)
    got = r0["metrics"].tolist()
    assert abs(got[0] - loss) < 1e-5 * abs(loss) and got[1] == tokens and abs(got[2] - top5) < 1e-4


# ---- HIP (GPU box): ConvNeXt-Tiny children[7:] trainable + the HIP Transformer engine ----------
HIP_CFG = dict(d=128, ff=128, V=120, layers=2, H=2, L=16, B=2)


def hip_models(dev, rank=0, frozen=False):
    from imagecaptioningconvnext_amd.models.encoder import Encoder
    from imagecaptioningconvnext_amd.models.transformerDecoder import TransformerDecoder
    c = HIP_CFG
    torch.manual_seed(11)
    enc = Encoder(variant="tiny", compute_dtype=torch.float32)
    for m in enc.modules():  # stochastic depth off: the same computation on every rank / run
        if hasattr(m, "sd_prob"):
            m.sd_prob = 0.0
    with torch.no_grad():  # layer scale 1e-6 would hide the block branch (SURVEY.md §7 vi)
        for n, p in enc.named_parameters():
            if n.endswith("layer_scale"):
                p.fill_(0.5)
    if not frozen:
        enc.fine_tune(True, startingLayer=7)
    dec = TransformerDecoder(embed_dim=c["d"], decoder_dim=c["ff"], vocab_size=c["V"], maxLen=c["L"], device=dev,
                             wordMap=None, pretrained_embeddings_path=None, fine_tune_embeddings=True, dropout=0.0,
                             encoder_dim=768, num_heads=c["H"], num_layers=c["layers"], compute_dtype=torch.float32)
    if rank:  # other starting weights on rank 1: the trainer broadcasts rank 0's
        with torch.no_grad():
            for p in list(enc.parameters()) + list(dec.parameters()):
                p.add_(0.01)
    return enc.to(dev), dec.to(dev)


def hip_shard(rank, dev):
    c = HIP_CFG
    g = torch.Generator().manual_seed(400 + rank)
    img = torch.randn(c["B"], 3, 224, 224, generator=g)
    caps, lens = make_captions(c["B"], c["L"], [[16, 9], [12, 12]][rank], c["V"], 410 + rank)
    return img.to(dev), caps.to(dev), lens.to(dev)


def worker_hip(rank, world, initfile, outdir, graph, bucketed, steps, frozen=False):
    from imagecaptioningconvnext_amd import kernels as K
    from imagecaptioningconvnext_amd.train_step import TeacherForcedTrainer
    import faulthandler
    import sys
    faulthandler.dump_traceback_later(120, exit=True, file=sys.stderr)
    torch.set_num_threads(2)
    dist.init_process_group("gloo", init_method="file://" + initfile, rank=rank, world_size=world)
    dev = torch.device("cuda:0")
    enc, dec = hip_models(dev, rank, frozen)
    # frozen: the pipelined schedule (the encoder forward of batch i beside the decoder of i - 1)
    tr = TeacherForcedTrainer(enc, dec, lstm=False, decoder_lr=LR_DEC, encoder_lr=LR_ENC, grad_clip=CLIP,
                              graph=graph, pipeline=frozen)
    if not bucketed:
        tr._buckets = None
    for _ in range(steps):
        tr.step(*hip_shard(rank, dev))
    tr.flush()
    torch.cuda.synchronize()
    K.set_seed_counter(None)
    save_file({"dec": tr.eng.fp.flat.cpu(), "enc": (tr.enc_eng.fp.flat if tr.enc_eng else tr.eng.fp.m).cpu(),
               "metrics": torch.tensor([m for r in tr.drain_metrics() for m in r], dtype=torch.float64)},
              os.path.join(outdir, f"hip_rank{rank}.safetensors"))
    dist.barrier()
    dist.destroy_process_group()
    faulthandler.cancel_dump_traceback_later()


def run_hip(tmpdir, graph, bucketed, steps=2, world=2, frozen=False):
    import torch.multiprocessing as mp
    os.makedirs(str(tmpdir), exist_ok=True)
    initfile = os.path.join(str(tmpdir), "init")
    mp.spawn(worker_hip, args=(world, initfile, str(tmpdir), graph, bucketed, steps, frozen), nprocs=world,
             join=True)
    return [load_file(os.path.join(str(tmpdir), f"hip_rank{r}.safetensors")) for r in range(world)]


def expected_hip(dev, steps=2):
    """One process, the same HIP engines: each rank's shard forward / backward into its own
    gradient buffers, their sum (what the SUM all-reduce hands every rank), clip + Adam with
    grad_div 2 -- bitwise what the 2-rank run must produce."""
    enc, dec = hip_models(dev, 0)
    eng, eeng = dec.engine(), enc.engine()
    for _ in range(steps):
        gd = [torch.empty_like(eng.fp.grad) for _ in range(2)]
        ge = [torch.empty_like(eeng.fp.grad) for _ in range(2)]
        for r in range(2):
            img, caps, lens = hip_shard(r, dev)
            enc.train()
            dec.train()
            feats, es = eeng.forward(img)
            s = eng.forward(feats, caps, lens, pad_id=0)
            eng.backward(s, gbuf=gd[r], want_denc=True)
            eeng.backward(es, s["denc"].reshape(feats.shape), gbuf=ge[r])
        eng.fp.grad.copy_(gd[0] + gd[1])
        eeng.fp.grad.copy_(ge[0] + ge[1])
        eng.fp.adam_step(LR_DEC, CLIP, grad_div=2.0)
        eeng.fp.adam_step(LR_ENC, CLIP, grad_div=2.0)
    torch.cuda.synchronize()
    return eng.fp.flat.cpu(), eeng.fp.flat.cpu()

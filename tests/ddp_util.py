"""Two-rank DDP train step (trainMultiGPU.py:339-420) driven through TeacherForcedTrainer.

``worker`` runs one rank: it builds the LSTM decoder of the ddp2_lstm golden, steps the trainer
once on that rank's shard (pass-through encoder: the shard is already encoder features, as in
tools/gen_golden.py) and saves the post-step parameters and reduced metrics.

mode "oracle": the trainer's engine is a CPU stand-in whose forward/backward/Adam are the
oracle (test infrastructure only) -- exercises the trainer's broadcast / gradient all-reduce /
grad_div / metric reduction over gloo on CPU.  mode "hip": the real HIP engine on cuda:0 (both
ranks share the one GPU; gloo carries the all-reduce).
"""
import json
import os

import torch
import torch.distributed as dist
from safetensors.torch import load_file, save_file

from golden_util import GOLDEN_DIR


class PassThrough(torch.nn.Module):
    def forward(self, x):
        return x


class _OracleFlat:
    """FlatParams stand-in: one fp32 buffer of all parameters, oracle clip + Adam."""

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


class _OracleEngine:
    def __init__(self, params):
        self.fp = _OracleFlat(params)

    def forward(self, feats, caps, caplens, fixed_T=True, alphaC=1.0):
        from oracle import decoders, train_step
        pr = {n: v.clone().requires_grad_(True) for n, v in self.fp.views(self.fp.flat).items()}
        preds, cs, dls, al, _ = decoders.lstm_tf_forward(pr, feats, caps, caplens)
        loss, scores, targets = train_step.lstm_loss(preds, cs, dls, al, alphaC=alphaC)
        hits = float(train_step.top5_correct(scores, targets))
        return dict(loss=loss, pr=pr, metrics=torch.tensor([loss.item(), float(sum(dls)), hits]))

    def early_bucket(self):  # the last two parameters' range (the trainer's bucketed all-reduce)
        fp = self.fp
        n0 = sum(fp.shapes[n].numel() for n in fp.names[:-2])
        return n0, fp.flat.numel()

    def grad_buckets(self):
        return [self.early_bucket()]

    def backward(self, s, bucket_hook=None):
        s["loss"].backward()
        for n, v in self.fp.views(self.fp.grad).items():
            v.copy_(s["pr"][n].grad)
        if bucket_hook is not None:
            bucket_hook()


class _OracleDecoder(torch.nn.Module):
    def __init__(self, params):
        super().__init__()
        self._eng = _OracleEngine(params)

    def engine(self):
        return self._eng


def _golden():
    t = load_file(os.path.join(GOLDEN_DIR, "ddp2_lstm.safetensors"))
    s = load_file(os.path.join(GOLDEN_DIR, "lstm_tf_small.safetensors"))
    with open(os.path.join(GOLDEN_DIR, "ddp2_lstm.json")) as f:
        meta = json.load(f)
    params = {k[len("param."):]: v for k, v in s.items() if k.startswith("param.")}
    return t, meta, params


def worker(rank, world, initfile, mode, outdir, graph=False, bucketed=True):
    from imagecaptioningconvnext_amd.train_step import TeacherForcedTrainer
    torch.set_num_threads(2)
    dist.init_process_group("gloo", init_method="file://" + initfile, rank=rank, world_size=world)
    t, meta, params = _golden()
    cfg = meta["cfg"]
    if mode == "oracle":
        dev = torch.device("cpu")
        # rank 1 starts from different weights: the trainer must broadcast rank 0's (DDP init)
        dec = _OracleDecoder({n: v + 0.5 * rank for n, v in params.items()})
    else:
        from imagecaptioningconvnext_amd.models.decoder import DecoderWithAttention
        dev = torch.device("cuda:0")
        dec = DecoderWithAttention(attention_dim=cfg["A"], embed_dim=cfg["Em"], decoder_dim=cfg["D"],
                                   vocab_size=cfg["V"], device=dev, encoder_dim=cfg["E"], dropout=0.0,
                                   compute_dtype=torch.float32)
        dec.load_state_dict({n: v + 0.5 * rank for n, v in params.items()})
        dec = dec.to(dev)
    tr = TeacherForcedTrainer(PassThrough(), dec, lstm=True, decoder_lr=1e-4, grad_clip=5.0, graph=graph)
    assert tr._buckets is not None and len(tr._buckets) == 1  # early bucket (LSTM engine: embedding + fc)
    if not bucketed:
        tr._buckets = None
    tr.step(t[f"rank{rank}.enc"].to(dev), t[f"rank{rank}.caps"].to(dev), t[f"rank{rank}.caplens"].to(dev))
    (loss, tokens, top5), = tr.drain_metrics()
    fp = tr.eng.fp
    if mode == "oracle":
        post = fp.views(fp.flat)
    else:
        post = {n: p.detach() for n, p in dec.named_parameters()}
    out = {"post." + n: v.detach().float().cpu().contiguous() for n, v in post.items()}
    out["metrics"] = torch.tensor([loss, tokens, top5], dtype=torch.float64)
    save_file(out, os.path.join(outdir, f"rank{rank}.safetensors"))
    dist.barrier()
    dist.destroy_process_group()


def run(mode, tmpdir, world=2, graph=False, bucketed=True):
    import torch.multiprocessing as mp
    initfile = os.path.join(str(tmpdir), "init")
    mp.spawn(worker, args=(world, initfile, mode, str(tmpdir), graph, bucketed), nprocs=world, join=True)
    return [load_file(os.path.join(str(tmpdir), f"rank{r}.safetensors")) for r in range(world)]


def check(results, rtol=1e-5, atol=1e-6, lr=1e-4):
    """Both ranks hold identical weights equal to the reference's post-step weights (entries
    whose averaged gradient is round-off noise agree within 2*lr, see test_oracle_golden), and
    the reduced metrics equal reduceLossAndTokens / the top-5 all-reduce."""
    t, meta, params = _golden()
    r0, r1 = results
    for k in r0:
        torch.testing.assert_close(r0[k], r1[k], rtol=0, atol=0)
    for n in params:
        got, ref = r0["post." + n], t["post." + n]
        moved = (ref - params[n]).abs()
        # Adam step 1 moves an entry by lr*g/(|g|+eps): ~lr wherever |g| >> eps; entries moved
        # visibly less have a gradient near round-off, where only the 2*lr bound is meaningful
        sure = moved > 0.999 * lr
        torch.testing.assert_close(got[sure], ref[sure], rtol=rtol, atol=atol)
        assert (got - ref).abs().max().item() <= 2 * lr * 1.0001, n
    loss, tokens, top5 = r0["metrics"].tolist()
    assert abs(loss - float(t["ref_loss"])) < 1e-5
    assert abs(top5 - float(t["ref_top5"])) < 1e-4
    assert tokens == sum(c - 1 for caps in meta["caplens"] for c in caps)


def worker_steps(rank, world, initfile, outdir, pipeline, graph, bucketed, steps):
    """Several steps of the HIP trainer on this rank's golden shard (same batch each step):
    the flat parameters after the last update, for bucketed-vs-unbucketed comparisons."""
    from imagecaptioningconvnext_amd import kernels as K
    from imagecaptioningconvnext_amd.models.decoder import DecoderWithAttention
    from imagecaptioningconvnext_amd.train_step import TeacherForcedTrainer
    import faulthandler
    import sys
    faulthandler.dump_traceback_later(60, exit=True, file=sys.stderr)  # a hang names its line
    torch.set_num_threads(2)
    dist.init_process_group("gloo", init_method="file://" + initfile, rank=rank, world_size=world)
    t, meta, params = _golden()
    cfg = meta["cfg"]
    dev = torch.device("cuda:0")
    dec = DecoderWithAttention(attention_dim=cfg["A"], embed_dim=cfg["Em"], decoder_dim=cfg["D"],
                               vocab_size=cfg["V"], device=dev, encoder_dim=cfg["E"], dropout=0.0,
                               compute_dtype=torch.float32)
    dec.load_state_dict(params)
    dec = dec.to(dev)
    tr = TeacherForcedTrainer(PassThrough(), dec, lstm=True, decoder_lr=1e-3, grad_clip=5.0, graph=graph,
                              pipeline=pipeline)
    if not bucketed:
        tr._buckets = None
    batch = (t[f"rank{rank}.enc"].to(dev), t[f"rank{rank}.caps"].to(dev), t[f"rank{rank}.caplens"].to(dev))
    for _ in range(steps):
        tr.step(*batch)
    tr.flush()
    K.set_seed_counter(None)
    save_file({"flat": tr.eng.fp.flat.cpu(), "metrics": torch.tensor([m for r in tr.drain_metrics() for m in r],
                                                                   dtype=torch.float64)},
              os.path.join(outdir, f"steps_rank{rank}.safetensors"))
    dist.barrier()
    dist.destroy_process_group()
    faulthandler.cancel_dump_traceback_later()


def run_steps(tmpdir, pipeline, graph, bucketed, steps=4, world=2):
    import torch.multiprocessing as mp
    os.makedirs(str(tmpdir), exist_ok=True)
    initfile = os.path.join(str(tmpdir), "init")
    mp.spawn(worker_steps, args=(world, initfile, str(tmpdir), pipeline, graph, bucketed, steps), nprocs=world,
             join=True)
    return [load_file(os.path.join(str(tmpdir), f"steps_rank{r}.safetensors")) for r in range(world)]

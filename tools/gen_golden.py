"""Generate golden vectors from the REAL reference code (this container only).

    python tools/gen_golden.py            # writes tests/golden/*.safetensors + *.json

Runs the reference's own ``DecoderWithAttention`` / ``TransformerDecoder`` modules and its own
``train.trainWithTeacherForcing`` / ``trainMultiGPU.trainWithTeacherForcing`` functions (imported
from /root/reference with placeholder modules for the absent torchvision/gensim/h5py/nltk
names, see tools/ref_import.py) on deterministic inputs from tests/golden_util.py, and stores
inputs + outputs as data fixtures.  Reference source never leaves /root/reference.

Fixtures:
  lstm_tf_small       decoder.py:69-113 + train.py:240-302 (LSTM, 1 step, clip 5, Adam 1e-4)
  transformer_tf_small transformerDecoder.py:88-108 + train.py:270-302 (key-padding mask)
  ddp2_lstm            trainMultiGPU.py:339-420, 2-rank gloo DDP, different shard per rank
  lstm_full_spot / transformer_full_spot   full-size dims (E=768, V=9490, L=52), B=2:
                       loss + sampled logits; weights regenerated from the recipe at test time
"""
import copy
import json
import os
import sys
import tempfile

import torch
import torch.multiprocessing as mp
from safetensors.torch import save_file

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
sys.path.insert(0, os.path.join(HERE, "..", "tests"))
import ref_import  # noqa: E402
from golden_util import GOLDEN_DIR, make_captions, make_features, make_params, word_map  # noqa: E402

torch.set_num_threads(8)
torch.use_deterministic_algorithms(True)

LSTM_SMALL = dict(B=3, L=14, caplens=[12, 9, 6], V=50, E=32, A=16, D=16, Em=16, S=2, seed=11)
TRF_SMALL = dict(B=3, L=12, caplens=[12, 7, 9], V=50, E=48, d=32, ff=64, H=4, layers=2, S=2, seed=22)
LSTM_FULL = dict(B=2, L=52, caplens=[52, 40], V=9490, E=768, A=512, D=512, Em=512, S=7, seed=33)
TRF_FULL = dict(B=2, L=52, caplens=[52, 37], V=9490, E=768, d=512, ff=512, H=8, layers=6, S=7, seed=44)


class PassThroughEncoder(torch.nn.Module):
    """Stands in for Encoder: the 'images' handed to the train function are already features."""

    def forward(self, x):
        return x


def _train_module(lstm):
    tr = ref_import.load("train.py", "ref_train", argv=["train.py", "--teacherForcing"])
    tr.lstmDecoder = lstm
    return tr


def _named_shapes(module):
    return {n: tuple(p.shape) for n, p in module.named_parameters()}


def _grads(module):
    return {"grad." + n: p.grad.detach().clone() for n, p in module.named_parameters() if p.grad is not None}


def _lstm_decoder(cfg):
    _train_module(True)
    dec_mod = sys.modules["models.decoder"]
    dec = dec_mod.DecoderWithAttention(attention_dim=cfg["A"], embed_dim=cfg["Em"], decoder_dim=cfg["D"],
                                       vocab_size=cfg["V"], device="cpu", encoder_dim=cfg["E"], dropout=0.0)
    dec.load_state_dict(make_params(_named_shapes(dec), cfg["seed"]))
    return dec


def _transformer_decoder(cfg):
    _train_module(False)
    tmod = sys.modules["models.transformerDecoder"]
    dec = tmod.TransformerDecoder(embed_dim=cfg["d"], decoder_dim=cfg["ff"], vocab_size=cfg["V"], maxLen=cfg["L"],
                                  device="cpu", wordMap=None, pretrained_embeddings_path=None,
                                  fine_tune_embeddings=True, dropout=0.0, encoder_dim=cfg["E"],
                                  num_heads=cfg["H"], num_layers=cfg["layers"])
    sd = dict(dec.state_dict())
    sd.update(make_params(_named_shapes(dec), cfg["seed"]))
    dec.load_state_dict(sd)
    return dec


def _inputs(cfg):
    enc = make_features((cfg["B"], cfg["S"], cfg["S"], cfg["E"]), cfg["seed"] + 1)
    caps, caplens = make_captions(cfg["B"], cfg["L"], cfg["caplens"], cfg["V"], cfg["seed"] + 2)
    return enc, caps, caplens


def lstm_loss(dec, enc, caps, caplens, alphaC=1.0):
    """train.py:263-269 verbatim in behaviour (packing + CE + doubly-stochastic reg)."""
    from torch.nn.utils.rnn import pack_padded_sequence
    scores, caps_sorted, dls, alphas, sort_ind = dec(teacherForcing=True, encoder_out=enc,
                                                     encoded_captions=caps, caption_lengths=caplens)
    targets = caps_sorted[:, 1:]
    packed = pack_padded_sequence(scores, dls, batch_first=True).data
    tpacked = pack_padded_sequence(targets, dls, batch_first=True).data
    ce = torch.nn.CrossEntropyLoss()(packed, tpacked)
    reg = alphaC * ((1.0 - alphas.sum(dim=1)) ** 2).mean()
    return dict(scores=scores, caps_sorted=caps_sorted, dls=dls, alphas=alphas, sort_ind=sort_ind,
                packed=packed, tpacked=tpacked, ce=ce, loss=ce + reg)


def transformer_loss(dec, enc, caps, caplens):
    """train.py:271-276 in behaviour."""
    from torch.nn.utils.rnn import pack_padded_sequence
    mask = caps == 0
    scores, caps_out, dls = dec(teacherForcing=True, encoder_out=enc, encoded_captions=caps,
                                caption_lengths=caplens, tgt_key_padding_mask=mask)
    targets = caps_out[:, 1:]
    packed = pack_padded_sequence(scores, dls, batch_first=True, enforce_sorted=False).data
    tpacked = pack_padded_sequence(targets, dls, batch_first=True, enforce_sorted=False).data
    loss = torch.nn.CrossEntropyLoss()(packed, tpacked)
    return dict(scores=scores, dls=dls, packed=packed, tpacked=tpacked, loss=loss)


def _run_ref_train_step(tr, dec, enc, caps, caplens, lstm):
    """One call of the reference's own train.trainWithTeacherForcing over a one-batch loader."""
    opt = torch.optim.Adam(params=filter(lambda p: p.requires_grad, dec.parameters()), lr=tr.decoderLr)
    crit = torch.nn.CrossEntropyLoss()
    out = tr.trainWithTeacherForcing(trainDataLoader=[(enc, caps, caplens)], encoder=PassThroughEncoder(),
                                     decoder=dec, criterion=crit, encoderOptimizer=None,
                                     decoderOptimizer=opt, epoch=0, device="cpu")
    return out, {"post." + n: p.detach().clone() for n, p in dec.named_parameters()}


def gen_lstm_small():
    cfg = LSTM_SMALL
    dec = _lstm_decoder(cfg)
    enc, caps, caplens = _inputs(cfg)
    params = {"param." + n: p.detach().clone() for n, p in dec.named_parameters()}
    r = lstm_loss(dec, enc, caps, caplens)
    r["loss"].backward()
    grads = _grads(dec)
    tr = _train_module(True)
    dec2 = _lstm_decoder(cfg)
    (loss_avg, top5, _, _), post = _run_ref_train_step(tr, dec2, enc, caps, caplens, True)
    t = dict(enc=enc, caps=caps, caplens=caplens, predictions=r["scores"].detach(), alphas=r["alphas"].detach(),
             caps_sorted=r["caps_sorted"], sort_ind=r["sort_ind"], packed_scores=r["packed"].detach(),
             packed_targets=r["tpacked"], loss=r["loss"].detach().view(1), ce=r["ce"].detach().view(1),
             ref_step_loss=torch.tensor([loss_avg]), ref_step_top5=torch.tensor([top5]))
    t.update(params)
    t.update(grads)
    t.update(post)
    meta = dict(cfg=cfg, decode_lengths=r["dls"], source="decoder.py:69-113; train.py:240-302")
    return "lstm_tf_small", t, meta


def gen_transformer_small():
    cfg = TRF_SMALL
    dec = _transformer_decoder(cfg)
    enc, caps, caplens = _inputs(cfg)
    params = {"param." + n: p.detach().clone() for n, p in dec.named_parameters()}
    r = transformer_loss(dec, enc, caps, caplens)
    r["loss"].backward()
    grads = _grads(dec)
    tr = _train_module(False)
    tr.wordMap = word_map(cfg["V"])
    dec2 = _transformer_decoder(cfg)
    (loss_avg, top5, _, _), post = _run_ref_train_step(tr, dec2, enc, caps, caplens, False)
    t = dict(enc=enc, caps=caps, caplens=caplens, predictions=r["scores"].detach(),
             packed_scores=r["packed"].detach(), packed_targets=r["tpacked"], loss=r["loss"].detach().view(1),
             pe=dec.pos_encoding.pe.detach().clone(),
             ref_step_loss=torch.tensor([loss_avg]), ref_step_top5=torch.tensor([top5]))
    t.update(params)
    t.update(grads)
    t.update(post)
    meta = dict(cfg=cfg, decode_lengths=r["dls"], source="transformerDecoder.py:88-108; train.py:240-302")
    return "transformer_tf_small", t, meta


def _ddp_worker(rank, world, initfile, outdir):
    import torch.distributed as dist
    from torch.nn.parallel import DistributedDataParallel as DDP
    torch.set_num_threads(2)
    dist.init_process_group("gloo", init_method="file://" + initfile, rank=rank, world_size=world)
    tm = ref_import.load("trainMultiGPU.py", "ref_trainMultiGPU", argv=["trainMultiGPU.py", "--teacherForcing"])
    tm.lstmDecoder = True
    cfg = LSTM_SMALL
    dec = _lstm_decoder(cfg)  # identical init on both ranks (recipe), like a rank-0 broadcast
    # different shard per rank
    enc = make_features((cfg["B"], cfg["S"], cfg["S"], cfg["E"]), 100 + rank)
    caps, caplens = make_captions(cfg["B"], cfg["L"], [[12, 9, 6], [10, 11, 5]][rank], cfg["V"], 200 + rank)
    ddp = DDP(dec)
    opt = torch.optim.Adam(params=filter(lambda p: p.requires_grad, ddp.parameters()), lr=tm.decoderLr)
    out = tm.trainWithTeacherForcing([(enc, caps, caplens)], PassThroughEncoder(), ddp, torch.nn.CrossEntropyLoss(),
                                     None, opt, 0, "cpu", world)
    t = {f"rank{rank}.enc": enc, f"rank{rank}.caps": caps, f"rank{rank}.caplens": caplens}
    if rank == 0:
        t.update({"post." + n: p.detach().clone() for n, p in dec.named_parameters()})
        t["ref_loss"] = torch.tensor([out[0]])
        t["ref_top5"] = torch.tensor([out[1]])
    save_file({k: v.contiguous() for k, v in t.items()}, os.path.join(outdir, f"r{rank}.safetensors"))
    dist.destroy_process_group()


def gen_ddp2():
    from safetensors.torch import load_file
    with tempfile.TemporaryDirectory() as td:
        initfile = os.path.join(td, "init")
        mp.spawn(_ddp_worker, args=(2, initfile, td), nprocs=2, join=True)
        t = {}
        for r in range(2):
            t.update(load_file(os.path.join(td, f"r{r}.safetensors")))
    meta = dict(cfg=LSTM_SMALL, world_size=2, caplens=[[12, 9, 6], [10, 11, 5]],
                source="trainMultiGPU.py:96-108,339-420 under 2-rank gloo DDP")
    return "ddp2_lstm", t, meta


def _spot_indices(n_rows, V, k, seed):
    g = torch.Generator().manual_seed(seed)
    return torch.randint(0, n_rows, (k,), generator=g), torch.randint(0, V, (k,), generator=g)


def gen_lstm_full():
    cfg = LSTM_FULL
    dec = _lstm_decoder(cfg)
    enc, caps, caplens = _inputs(cfg)
    with torch.no_grad():
        r = lstm_loss(dec, enc, caps, caplens)
    ri, vi = _spot_indices(r["packed"].shape[0], cfg["V"], 256, 5)
    t = dict(loss=r["loss"].view(1), ce=r["ce"].view(1), rows=ri, cols=vi, values=r["packed"][ri, vi],
             alphas=r["alphas"], sort_ind=r["sort_ind"])
    meta = dict(cfg=cfg, decode_lengths=r["dls"], torch=torch.__version__,
                note="weights: tests/golden_util.make_params(named_shapes, cfg.seed); not stored")
    return "lstm_full_spot", t, meta


def gen_transformer_full():
    cfg = TRF_FULL
    dec = _transformer_decoder(cfg)
    enc, caps, caplens = _inputs(cfg)
    with torch.no_grad():
        r = transformer_loss(dec, enc, caps, caplens)
    ri, vi = _spot_indices(r["packed"].shape[0], cfg["V"], 256, 6)
    t = dict(loss=r["loss"].view(1), rows=ri, cols=vi, values=r["packed"][ri, vi])
    meta = dict(cfg=cfg, decode_lengths=r["dls"], torch=torch.__version__,
                note="weights: tests/golden_util.make_params(named_shapes, cfg.seed); not stored")
    return "transformer_full_spot", t, meta


def main():
    os.makedirs(GOLDEN_DIR, exist_ok=True)
    for fn in (gen_lstm_small, gen_transformer_small, gen_ddp2, gen_lstm_full, gen_transformer_full,
               gen_transformer_h64):
        name, tensors, meta = fn()
        save_file({k: v.detach().contiguous() for k, v in tensors.items()},
                  os.path.join(GOLDEN_DIR, name + ".safetensors"))
        with open(os.path.join(GOLDEN_DIR, name + ".json"), "w") as f:
            json.dump(meta, f, indent=1)
        print("wrote", name, sum(v.numel() for v in tensors.values()), "values")




TRF_H64 = dict(B=3, L=12, caplens=[12, 7, 9], V=50, E=48, d=64, ff=32, H=1, layers=2, S=2, seed=55)


def gen_transformer_h64():
    """Head dim 64 (the HIP attention kernel's tile); params regenerated from the recipe at test time."""
    cfg = TRF_H64
    dec = _transformer_decoder(cfg)
    enc, caps, caplens = _inputs(cfg)
    r = transformer_loss(dec, enc, caps, caplens)
    r["loss"].backward()
    grads = _grads(dec)
    tr = _train_module(False)
    tr.wordMap = word_map(cfg["V"])
    dec2 = _transformer_decoder(cfg)
    (loss_avg, top5, _, _), post = _run_ref_train_step(tr, dec2, enc, caps, caplens, False)
    t = dict(enc=enc, caps=caps, caplens=caplens, predictions=r["scores"].detach(), loss=r["loss"].detach().view(1),
             ref_step_loss=torch.tensor([loss_avg]), ref_step_top5=torch.tensor([top5]))
    t.update(grads)
    t.update(post)
    meta = dict(cfg=cfg, decode_lengths=r["dls"], source="transformerDecoder.py:88-108; train.py:240-302",
                note="params: tests/golden_util.make_params(named_shapes, cfg.seed); not stored")
    return "transformer_tf_h64", t, meta


def _gen_ckpt(lstm):
    """Resume fixture: one reference train step, the checkpoint the
    reference's own utils.save_checkpoint writes after it, then a second step on the same
    batch (its post-step parameters and clamped gradients).  encoderSaved is None: the
    reference Encoder needs torchvision (§8c), and the encoder keys are checked separately."""
    import shutil
    import tempfile
    cfg = LSTM_SMALL if lstm else TRF_H64  # head dim 64: the HIP attention kernel's tile
    tr = _train_module(lstm)
    if not lstm:
        tr.wordMap = word_map(cfg["V"])
    dec = _lstm_decoder(cfg) if lstm else _transformer_decoder(cfg)
    enc, caps, caplens = _inputs(cfg)
    opt = torch.optim.Adam(params=filter(lambda p: p.requires_grad, dec.parameters()), lr=tr.decoderLr)
    crit = torch.nn.CrossEntropyLoss()

    def step():
        return tr.trainWithTeacherForcing(trainDataLoader=[(enc, caps, caplens)], encoder=PassThroughEncoder(),
                                          decoder=dec, criterion=crit, encoderOptimizer=None,
                                          decoderOptimizer=opt, epoch=0, device="cpu")
    step()
    utils_mod = sys.modules["utils.utils"]
    name = "ckpt_lstm_small" if lstm else "ckpt_transformer_small"
    cwd = os.getcwd()
    tmp = tempfile.mkdtemp()
    try:
        os.chdir(tmp)
        utils_mod.save_checkpoint("coco_5_cap_per_img_5_min_word_freq", 0, 0, None, dec.state_dict(), None, opt,
                                  0.0, False, [], lstm, 5, 1e-4, None if lstm else "none")
        (written,) = os.listdir(tmp)
        shutil.copy(written, os.path.join(GOLDEN_DIR, name + ".pth.tar"))
    finally:
        os.chdir(cwd)
        shutil.rmtree(tmp)
    loss2, top5_2, _, _ = step()
    t = dict(enc=enc, caps=caps, caplens=caplens, ref_step2_loss=torch.tensor([loss2]))
    t.update({"post2." + n: p.detach().clone() for n, p in dec.named_parameters()})
    t.update({"grad2." + n: p.grad.detach().clone() for n, p in dec.named_parameters() if p.grad is not None})
    meta = dict(cfg=cfg, filename=written, param_order=[n for n, p in dec.named_parameters() if p.requires_grad],
                source="utils.py:195-224 (save_checkpoint), train.py:118-147 (resume), train.py:240-302")
    return name, t, meta


def gen_ckpt_lstm():
    return _gen_ckpt(True)


def gen_ckpt_transformer():
    return _gen_ckpt(False)


def gen_greedy():
    """forwardWithoutTeacherForcing (decoder.py:119-163, transformerDecoder.py:110-160) of the
    reference in eval mode: predictions, alphas (LSTM), sequences, for a maxDecodeLen run."""
    t, meta = {}, {}
    for name, cfg, lstm in (("lstm", LSTM_SMALL, True), ("trf", TRF_H64, False)):
        for variant in ("", "_end"):
            dec = _lstm_decoder(cfg) if lstm else _transformer_decoder(cfg)
            dec.eval()
            enc, _, _ = _inputs(cfg)
            wm = word_map(cfg["V"])
            fc = dec.fc if lstm else dec.fc_out
            end_bias = 0.0
            if variant:  # raise <end>'s bias until rows finish at different steps (the finished logic)
                for end_bias in [0.05 * k for k in range(1, 200)]:
                    with torch.no_grad():
                        fc.bias[wm["<end>"]] += 0.05
                        out = dec(teacherForcing=False, encoder_out=enc, wordMap=wm, maxDecodeLen=10)
                    first = [(row == wm["<end>"]).nonzero()[:1].flatten().tolist() for row in out[-1]]
                    stops = {f[0] if f else 99 for f in first}
                    if len(stops) >= 2 and 99 not in stops or len(stops) >= 3:
                        break
            with torch.no_grad():
                out = dec(teacherForcing=False, encoder_out=enc, wordMap=wm, maxDecodeLen=10)
            key = name + variant
            t[f"{key}.enc"] = enc
            t[f"{key}.predictions"] = out[0]
            t[f"{key}.sequences"] = out[-1]
            if lstm:
                t[f"{key}.alphas"] = out[1]
            meta[key] = dict(cfg=cfg, maxDecodeLen=10, end_bias_added=round(end_bias, 6))
    meta["source"] = "decoder.py:119-163; transformerDecoder.py:110-160 (eval, greedy)"
    meta["note"] = "params: tests/golden_util.make_params(named_shapes, cfg.seed) (the same recipe as *_tf_*)"
    return "greedy_small", t, meta


def gen_beam():
    """caption.py:39-155 / :160-255 (the reference's own beam-search functions) on a temp PNG with a
    stand-in encoder that returns fixed features (the reference Encoder needs torchvision, §8c):
    the returned word ids (and LSTM alphas) for beam sizes 3 and 5.  <end>'s fc bias is raised
    (recorded) so that beams complete at different steps."""
    import numpy as np
    from PIL import Image
    if "skimage" not in sys.modules:
        ref_import._stub("skimage")
        ref_import._stub("skimage.transform")
    cap = ref_import.load("caption.py", "ref_caption", argv=["caption.py"])
    cap.device = torch.device("cpu")
    import types  # the image transform only feeds the stand-in encoder, which ignores it

    def _normalize(mean, std):
        m, s = torch.tensor(mean).view(-1, 1, 1), torch.tensor(std).view(-1, 1, 1)
        return lambda x: (x - m) / s
    cap.transforms = types.SimpleNamespace(Normalize=_normalize,
                                           Compose=lambda fs: (lambda x: fs[0](x)))
    tmp = tempfile.mkdtemp()
    png = os.path.join(tmp, "img.png")
    Image.fromarray(np.random.default_rng(0).integers(0, 256, size=(40, 30, 3), dtype=np.uint8)).save(png)

    class FixedEncoder(torch.nn.Module):
        def __init__(self, feats):
            super().__init__()
            self.feats = feats

        def forward(self, image):
            return self.feats

    t, meta = {}, {}
    # the Transformer beam search decodes up to 51 positions: positional table of maxLen 52
    for name, cfg, lstm in (("lstm", LSTM_SMALL, True), ("trf", dict(TRF_H64, L=52), False)):
        feats = make_features((1, cfg["S"], cfg["S"], cfg["E"]), cfg["seed"] + 5)
        enc = FixedEncoder(feats)
        wm = word_map(cfg["V"])
        run = cap.caption_image_beam_search if lstm else cap.caption_image_beam_search_transformer
        # smallest <end> bias (steps of 0.01) at which every beam size finishes with a caption of >= 3 ids
        for bias in [0.01 * i for i in range(0, 1000)]:
            dec = _lstm_decoder(cfg) if lstm else _transformer_decoder(cfg)
            dec.eval()
            fc = dec.fc if lstm else dec.fc_out
            with torch.no_grad():
                fc.bias[wm["<end>"]] += bias
                try:
                    lens = [len(run(enc, dec, png, wm, beamSize=k)[0]) for k in (3, 5)]
                except ValueError:  # no beam completed (max() of an empty list)
                    continue
            if min(lens) >= 3:
                break
        t[f"{name}.feats"] = feats
        for k in (3, 5):
            with torch.no_grad():
                if lstm:
                    seq, alphas = cap.caption_image_beam_search(enc, dec, png, wm, beamSize=k)
                    t[f"{name}.k{k}.alphas"] = torch.tensor(alphas, dtype=torch.float32)
                else:
                    seq, _ = cap.caption_image_beam_search_transformer(enc, dec, png, wm, beamSize=k)
            t[f"{name}.k{k}.seq"] = torch.tensor(seq, dtype=torch.int64)
        meta[name] = dict(cfg=cfg, end_bias_added=round(bias, 6))
    meta["source"] = "caption.py:39-155 (LSTM), caption.py:160-255 (Transformer), run with a fixed-feature encoder"
    return "beam_small", t, meta


ATT_CFG = dict(B=3, L=12, caplens=[12, 7, 9], V=50, E=48, d=128, ff=32, H=2, layers=2, S=2, seed=66)


def _attvis_decoder(cfg):
    import importlib
    _train_module(False)  # stubs + the reference root on sys.path
    mod = importlib.import_module("models.transformerDecoderAttVis")
    dec = mod.TransformerDecoderForAttentionViz(embed_dim=cfg["d"], decoder_dim=cfg["ff"], vocab_size=cfg["V"],
                                                maxLen=cfg["L"], device="cpu", dropout=0.0, encoder_dim=cfg["E"],
                                                num_heads=cfg["H"], num_layers=cfg["layers"])
    sd = dict(dec.state_dict())
    sd.update(make_params(_named_shapes(dec), cfg["seed"]))
    dec.load_state_dict(sd)
    dec.eval()
    return dec


def gen_attvis():
    """models/transformerDecoderAttVis.py (TransformerDecoderForAttentionViz) in eval mode:
    teacher-forced predictions + alphas [H, B, P] (with a key-padding mask), greedy predictions /
    sequences / alphas (rows ending at different steps), and caption.py:260-383
    (caption_image_beam_search_transformer_attention) word ids + alphas, beam 3 and 5."""
    import numpy as np
    from PIL import Image
    t, meta = {}, {}
    cfg = ATT_CFG
    dec = _attvis_decoder(cfg)
    enc, caps, caplens = _inputs(cfg)
    with torch.no_grad():
        preds, _, dls, alphas = dec(teacherForcing=True, encoder_out=enc, encoded_captions=caps,
                                    caption_lengths=caplens, tgt_key_padding_mask=caps == 0)
    t.update({"tf.enc": enc, "tf.caps": caps, "tf.caplens": caplens, "tf.predictions": preds, "tf.alphas": alphas})
    meta["tf"] = dict(cfg=cfg, decode_lengths=dls)
    wm = word_map(cfg["V"])
    end_bias = 0.0
    for end_bias in [0.05 * k for k in range(1, 200)]:  # rows finish at different steps
        with torch.no_grad():
            dec.fc_out.bias[wm["<end>"]] += 0.05
            out = dec(teacherForcing=False, encoder_out=enc, wordMap=wm, maxDecodeLen=10)
        first = [(row == wm["<end>"]).nonzero()[:1].flatten().tolist() for row in out[1]]
        stops = {f[0] if f else 99 for f in first}
        if len(stops) >= 2 and 99 not in stops or len(stops) >= 3:
            break
    with torch.no_grad():
        gp, gs, ga = dec(teacherForcing=False, encoder_out=enc, wordMap=wm, maxDecodeLen=10)
    t.update({"greedy.predictions": gp, "greedy.sequences": gs, "greedy.alphas": ga})
    meta["greedy"] = dict(maxDecodeLen=10, end_bias_added=round(end_bias, 6))
    # beam search with attention maps (caption.py:260-383), maxLen 52 for up to 51 positions
    if "skimage" not in sys.modules:
        ref_import._stub("skimage")
        ref_import._stub("skimage.transform")
    cap = ref_import.load("caption.py", "ref_caption", argv=["caption.py"])
    cap.device = torch.device("cpu")
    import types

    def _normalize(mean, std):
        m, sd = torch.tensor(mean).view(-1, 1, 1), torch.tensor(std).view(-1, 1, 1)
        return lambda x: (x - m) / sd
    cap.transforms = types.SimpleNamespace(Normalize=_normalize, Compose=lambda fs: (lambda x: fs[0](x)))
    png = os.path.join(tempfile.mkdtemp(), "img.png")
    Image.fromarray(np.random.default_rng(0).integers(0, 256, size=(40, 30, 3), dtype=np.uint8)).save(png)

    class FixedEncoder(torch.nn.Module):
        def __init__(self, feats):
            super().__init__()
            self.feats = feats

        def forward(self, image):
            return self.feats

    bcfg = dict(cfg, L=52)
    # feature seed with the longest beam captions at the first <end> bias (steps of 0.01) at
    # which both beam sizes finish
    best = None
    for fseed in range(bcfg["seed"] + 5, bcfg["seed"] + 17):
        feats = make_features((1, bcfg["S"], bcfg["S"], bcfg["E"]), fseed)
        fenc = FixedEncoder(feats)
        for bias in [0.01 * i for i in range(0, 600)]:
            bdec = _attvis_decoder(bcfg)
            with torch.no_grad():
                bdec.fc_out.bias[wm["<end>"]] += bias
                try:
                    lens = [len(cap.caption_image_beam_search_transformer_attention(fenc, bdec, png, wm, "x",
                                                                                    beamSize=k)[0]) for k in (3, 5)]
                except ValueError:
                    continue
            if best is None or min(lens) > best[0]:
                best = (min(lens), fseed, bias)
            break
        if best is not None and best[0] >= 6:
            break
    _, fseed, bias = best
    feats = make_features((1, bcfg["S"], bcfg["S"], bcfg["E"]), fseed)
    fenc = FixedEncoder(feats)
    bdec = _attvis_decoder(bcfg)
    with torch.no_grad():
        bdec.fc_out.bias[wm["<end>"]] += bias
    bcfg["feature_seed"] = fseed
    t["beam.feats"] = feats
    for k in (3, 5):
        with torch.no_grad():
            seq, al = cap.caption_image_beam_search_transformer_attention(fenc, bdec, png, wm, "x", beamSize=k)
        t[f"beam.k{k}.seq"] = torch.tensor(seq, dtype=torch.int64)
        t[f"beam.k{k}.alphas"] = torch.tensor(al, dtype=torch.float32)
    meta["beam"] = dict(cfg=bcfg, end_bias_added=round(bias, 6))
    meta["source"] = ("models/transformerDecoderAttVis.py:108-239 (eval), caption.py:260-383 with a fixed-feature "
                      "encoder; params: tests/golden_util.make_params(named_shapes, cfg.seed)")
    return "attvis_small", t, meta


if __name__ == "__main__":
    if len(sys.argv) > 1 and sys.argv[1] in ("greedy", "beam", "attvis"):
        name, tensors, meta = {"greedy": gen_greedy, "beam": gen_beam, "attvis": gen_attvis}[sys.argv[1]]()
        save_file({k: v.detach().contiguous() for k, v in tensors.items()}, os.path.join(GOLDEN_DIR, name + ".safetensors"))
        with open(os.path.join(GOLDEN_DIR, name + ".json"), "w") as f:
            json.dump(meta, f, indent=1)
        print("wrote", name, {k: tuple(v.shape) for k, v in tensors.items()})
    elif len(sys.argv) > 1 and sys.argv[1] == "ckpt":
        fns = (gen_ckpt_lstm, gen_ckpt_transformer)
        for fn in (fns[int(sys.argv[2]):int(sys.argv[2]) + 1] if len(sys.argv) > 2 else fns):
            name, tensors, meta = fn()
            save_file({k: v.detach().contiguous() for k, v in tensors.items()},
                      os.path.join(GOLDEN_DIR, name + ".safetensors"))
            with open(os.path.join(GOLDEN_DIR, name + ".json"), "w") as f:
                json.dump(meta, f, indent=1)
            print("wrote", name)
    else:
        main()

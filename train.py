"""Single-GPU teacher-forced training entry point with the reference's CLI (train.py:59-65).

    python train.py --teacherForcing [--lstmDecoder] [--startingLayer 5] [--encoderLr 1e-4]
                    [--encoder base|tiny|large] [--steps N] [--batchSize 32]

Mirrors ``train.py``'s model construction (:37-57, :95-115) and ``trainWithTeacherForcing``
(:240-302) on the MI355X path.  The COCO HDF5 pipeline (``CaptionDataset``) is outside this
build's scope and its inputs are absent here, so batches are synthetic COCO-shaped tensors
(224x224 images, length-52 captions, V = 9490) unless a loader is passed in.
"""
import argparse
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))

# model / training parameters of the reference (train.py:37-57)
embDim = 512
attentionDim = 512
decoderDim = 512
dropout = 0.5
maxLen = 52
batchSize = 32
decoderLr = 1e-4
gradClip = 5.
alphaC = 1.
VOCAB = 9490  # len(wordMap) of the Karpathy COCO split, min_word_freq 5


class AverageMeter:
    """utils.py AverageMeter: running average of a metric."""

    def __init__(self):
        self.val = self.avg = self.sum = 0.0
        self.count = 0

    def update(self, val, n=1):
        self.val = val
        self.sum += val * n
        self.count += n
        self.avg = self.sum / self.count


def make_parser(multi_gpu=False):
    """train.py:59-65 (``multi_gpu``: trainMultiGPU.py:63-70, which adds --port and fine-tunes
    from child 7 by default instead of 5)."""
    p = argparse.ArgumentParser()
    p.add_argument('--checkpoint', type=str, default=None, help='Path to checkpoint file')
    p.add_argument('--lstmDecoder', action='store_true', help='Use LSTM decoder instead of Transformer')
    if multi_gpu:
        p.add_argument('--port', type=str, default='29500', help='Master port for distributed training')
    p.add_argument('--teacherForcing', action='store_true', help='Use teacher forcing training strategy')
    p.add_argument('--startingLayer', type=int, default=7 if multi_gpu else 5,
                   help='Starting layer index for encoder fine-tuning')
    p.add_argument('--encoderLr', type=float, default=1e-4, help='Learning rate for encoder if fine-tuning')
    p.add_argument('--embeddingName', type=str, default=None, help='Pretrained embedding name from gensim')
    # additions of this build
    p.add_argument('--encoder', default='base', choices=['tiny', 'small', 'base', 'large'])
    p.add_argument('--batchSize', type=int, default=batchSize)
    p.add_argument('--steps', type=int, default=20, help='synthetic iterations per epoch')
    p.add_argument('--epochs', type=int, default=1)
    p.add_argument('--fineTuneFromEpoch', type=int, default=20,
                   help='epoch at which the encoder starts fine-tuning from --startingLayer (reference: 20)')
    p.add_argument('--saveDir', type=str, default=None,
                   help='write the reference-schema checkpoint (utils.py:195-224) here after every epoch')
    p.add_argument('--dataName', type=str, default='coco_5_cap_per_img_5_min_word_freq')
    p.add_argument('--dataFolder', type=str, default=None,
                   help="the reference's input files (train.py:35); synthetic batches when not given")
    p.add_argument('--workers', type=int, default=6)
    p.add_argument('--noPipeline', action='store_true',
                   help='frozen encoder: run encoder and decoder of a step back to back (no two-stream pipeline)')
    return p


def parse(argv=None):
    return make_parser().parse_args(argv)


def synthetic_loader(steps, B, device, rank=0, V=VOCAB, L=maxLen):
    """COCO-shaped synthetic batches: normalised U[0,1) images, <start> w.. <end>."""
    mean = torch.tensor([0.485, 0.456, 0.406]).view(1, 3, 1, 1)
    std = torch.tensor([0.229, 0.224, 0.225]).view(1, 3, 1, 1)
    for i in range(steps):
        g = torch.Generator().manual_seed(1234 + 7919 * rank + i)
        img = (torch.rand(B, 3, 224, 224, generator=g) - mean) / std
        caps = torch.randint(1, V - 3, (B, L), generator=g)
        caps[:, 0], caps[:, L - 1] = V - 2, V - 1
        yield img.to(device), caps.to(device), torch.full((B, 1), L, dtype=torch.long, device=device)


def _val_loader(args):
    """train.py:156-157: the VAL split (with its word map for <start>/<end>/<pad>), when present."""
    import json
    if not args.dataFolder:
        return None
    cap = os.path.join(args.dataFolder, 'VAL_CAPTIONS_' + args.dataName + '.json')
    if not os.path.exists(cap):
        return None
    from torch.utils.data import DataLoader
    from imagecaptioningconvnext_amd.data import CaptionDataset
    ds = CaptionDataset(args.dataFolder, args.dataName, 'VAL')
    wm_path = os.path.join(args.dataFolder, 'WORDMAP_' + args.dataName + '.json')
    if os.path.exists(wm_path):
        with open(wm_path) as f:
            ds.wordMap = json.load(f)
    else:  # SURVEY.md §8 ids: <pad>=0, <unk>=V-3, <start>=V-2, <end>=V-1
        ds.wordMap = {'<pad>': 0, '<unk>': VOCAB - 3, '<start>': VOCAB - 2, '<end>': VOCAB - 1}
    return DataLoader(ds, batch_size=args.batchSize, shuffle=True, num_workers=args.workers, pin_memory=True)


def data_loader(args, device, epoch, rank=0, world=1):
    """train.py:154-155 (trainMultiGPU.py:240: DistributedSampler, seed 42) over the reference's files;
    items stay uint8 (normalised in the stem kernel), batches go to the GPU as bytes.  --steps
    caps the iterations per epoch (0: the whole split)."""
    from torch.utils.data import DataLoader
    from torch.utils.data.distributed import DistributedSampler
    from imagecaptioningconvnext_amd.data import CaptionDataset
    ds = CaptionDataset(args.dataFolder, args.dataName, 'TRAIN')
    sampler = DistributedSampler(ds, num_replicas=world, rank=rank, shuffle=True, seed=42) if world > 1 else None
    if sampler is not None:
        sampler.set_epoch(epoch)
    dl = DataLoader(ds, batch_size=args.batchSize, shuffle=sampler is None, sampler=sampler,
                    num_workers=args.workers, pin_memory=True, persistent_workers=args.workers > 0)
    for i, (imgs, caps, caplens) in enumerate(dl):
        if args.steps and i >= args.steps:
            break
        # the batch's longest caption, read on the host before the copy: the trainer's LSTM
        # length bucket (TeacherForcedTrainer.bucket_T) without a device sync
        yield (imgs.to(device, non_blocking=True), caps.to(device, non_blocking=True),
               caplens.to(device, non_blocking=True), int(caplens.max()))


def build_models(args, device):
    """train.py:100-115: decoder + Adam lr, frozen encoder (fine_tune(False))."""
    from imagecaptioningconvnext_amd.models.decoder import DecoderWithAttention
    from imagecaptioningconvnext_amd.models.encoder import Encoder
    from imagecaptioningconvnext_amd.models.transformerDecoder import TransformerDecoder
    if args.embeddingName:
        raise NotImplementedError("gensim pre-trained embeddings are outside the accelerated path")
    encoder = Encoder(variant=args.encoder).to(device)
    encoder.fine_tune(fine_tune=False)
    E = encoder.encoder_dim
    if args.lstmDecoder:
        decoder = DecoderWithAttention(attention_dim=attentionDim, embed_dim=embDim, decoder_dim=decoderDim,
                                       vocab_size=VOCAB, dropout=dropout, device=device, encoder_dim=E)
    else:
        decoder = TransformerDecoder(embed_dim=embDim, decoder_dim=decoderDim, vocab_size=VOCAB, maxLen=maxLen,
                                     dropout=dropout, device=device, wordMap=None, pretrained_embeddings_path=None,
                                     fine_tune_embeddings=True, encoder_dim=E)
    ck = None
    if args.checkpoint:  # train.py:125-147 (weights here; optimizer state once the trainer exists)
        from imagecaptioningconvnext_amd.checkpoint import load_checkpoint
        ck = load_checkpoint(args.checkpoint, map_location=device)
        if ck['encoder'] is not None:
            encoder.load_state_dict(ck['encoder'])
        decoder.load_state_dict(ck['decoder'])
    return encoder, decoder.to(device), ck


def trainWithTeacherForcing(trainDataLoader, encoder, decoder, trainer, epoch, lstm, log=print):
    """train.py:240-302 on the fused MI355X step: returns (loss avg, top-5 avg, batch time avg,
    data time avg) like the reference.  Metrics are read back once per epoch (no per-step sync)."""
    encoder.train()
    decoder.train()
    batchTime, dataTime, losses, top5accs = AverageMeter(), AverageMeter(), AverageMeter(), AverageMeter()
    start = time.time()
    n = 0
    for i, (imgs, caps, caplens, *host) in enumerate(trainDataLoader):
        dataTime.update(time.time() - start)
        if i % 100 == 0:
            log(f"TF, Epoch {epoch}, Batch {i + 1}", flush=True)
        trainer.step(imgs, caps, caplens, max_caplen=host[0] if host else None)
        n += 1
        batchTime.update(time.time() - start)
        start = time.time()
    trainer.flush()  # pipelined schedule: the last batch of the epoch is still in flight
    if torch.cuda.is_initialized():
        torch.cuda.synchronize()
    for loss, tokens, top5 in trainer.drain_metrics():
        losses.update(loss, tokens)
        top5accs.update(top5, tokens)
    log(f"TF, Epoch {epoch}: Training Loss = {losses.avg:.4f}, Top-5 Accuracy = {top5accs.avg:.4f}", flush=True)
    return losses.avg, top5accs.avg, batchTime.avg, dataTime.avg


def _bcast_from_rank0(values, device):
    """trainMultiGPU.py:332-334: rank 0 owns the validation bookkeeping; every rank takes its
    numbers so the lr decays and the early stop happen on all ranks together."""
    import torch.distributed as dist
    t = torch.tensor([float(v) for v in values], dtype=torch.float64, device=device)
    dist.broadcast(t, src=0)
    return t.tolist()


def run_epochs(args, encoder, decoder, trainer, ck, device, rank=0, log=print, world=1, early_stop=20,
               val=_val_loader, validate_fn=None):
    """The epoch loop of train.py:159-229 / trainMultiGPU.py:247-334: resume (train.py:130-147)
    from ``ck``, fine-tune from --fineTuneFromEpoch, lr decay x0.8 every 8 epochs without a BLEU-4
    improvement, early stop after ``early_stop`` of them (20 in train.py:168, 40 in
    trainMultiGPU.py:259), checkpoint every epoch (rank 0) when --saveDir.  With world > 1 rank 0
    validates and broadcasts epochsSinceImprovement / bestBleu4 (trainMultiGPU.py:332-334).
    ``val`` (a loader factory) and ``validate_fn`` exist for tests."""
    startEpoch, epochsSinceImprovement, results = 0, 0, []
    if ck is not None:  # train.py:130-147
        startEpoch = ck['epoch'] + 1
        if startEpoch > args.fineTuneFromEpoch:
            trainer.enable_encoder_finetune(args.startingLayer)
        trainer.load_optimizers(ck['decoderOptimizer'],
                                ck['encoderOptimizer'] if trainer.enc_eng is not None else None)
        epochsSinceImprovement, results = ck['epochsSinceImprovement'], ck['results']
    bestBleu4 = ck['bleu-4'] if ck is not None else 0.0
    val = val(args) if (rank == 0 and val is not None) else None
    if validate_fn is None:
        from imagecaptioningconvnext_amd.metrics import validate as validate_fn
    for epoch in range(startEpoch, startEpoch + args.epochs):
        if epoch == args.fineTuneFromEpoch:  # train.py:160-166: a new encoder Adam at encoderLr
            trainer.enable_encoder_finetune(args.startingLayer)
            trainer.encoder_lr = args.encoderLr
            log(f"Fine-tuning encoder from epoch {epoch} onwards (starting from layer {args.startingLayer})",
                flush=True)
        if epochsSinceImprovement == early_stop:  # train.py:168-169 / trainMultiGPU.py:259-260
            break
        if epochsSinceImprovement > 0 and epochsSinceImprovement % 8 == 0:  # train.py:170-173
            trainer.decoder_lr *= 0.8
            if trainer.enc_eng is not None:  # only an existing encoder optimizer decays
                trainer.encoder_lr *= 0.8
        loader = (data_loader(args, device, epoch, rank, world) if args.dataFolder else
                  synthetic_loader(args.steps, args.batchSize, device, rank=rank))
        out = trainWithTeacherForcing(loader, encoder, decoder, trainer, epoch, args.lstmDecoder, log=log)
        log(f"epoch {epoch}: loss {out[0]:.4f} top5 {out[1]:.2f} batch {out[2] * 1e3:.2f} ms ({world} GPUs)",
            flush=True)
        rec = {'epoch': epoch, 'trainLoss': out[0], 'trainTop5Acc': out[1], 'trainBatchTime': out[2],
               'trainDataTime': out[3]}
        recentBleu4, isBest = 0.0, False
        if val is not None:  # train.py:190-222: greedy validation, BLEU, improvement bookkeeping
            vl, vt, b1, b2, b3, recentBleu4 = validate_fn(val, encoder, decoder, val.dataset.wordMap,
                                                          args.lstmDecoder, device, alphaC=alphaC, log=log)
            rec.update(valLoss=vl, valTop5Acc=vt, bleu1=b1, bleu2=b2, bleu3=b3, bleu4=recentBleu4)
            isBest = recentBleu4 > bestBleu4
            bestBleu4 = max(recentBleu4, bestBleu4)
            epochsSinceImprovement = 0 if isBest else epochsSinceImprovement + 1
            encoder.train()
            decoder.train()
        if world > 1:
            epochsSinceImprovement, bestBleu4 = _bcast_from_rank0((epochsSinceImprovement, bestBleu4), device)
            epochsSinceImprovement = int(epochsSinceImprovement)
        results.append(rec)
        if args.saveDir and rank == 0:  # train.py:224-229
            from imagecaptioningconvnext_amd.checkpoint import save_checkpoint
            encOpt, decOpt = trainer.optimizers()
            path = save_checkpoint(args.dataName, epoch, epochsSinceImprovement, encoder.state_dict(),
                                   decoder.state_dict(), encOpt, decOpt, recentBleu4, isBest, results,
                                   args.lstmDecoder, args.startingLayer, args.encoderLr, args.embeddingName,
                                   directory=args.saveDir)
            log(f"saved {path}", flush=True)
    return epochsSinceImprovement, results


def main(argv=None):
    args = parse(argv)
    if not args.teacherForcing:
        raise NotImplementedError("non-teacher-forced training is outside the accelerated path (SURVEY.md §8f)")
    torch.manual_seed(42)
    device = torch.device("cuda")
    from imagecaptioningconvnext_amd.train_step import TeacherForcedTrainer
    encoder, decoder, ck = build_models(args, device)
    # pipeline: while the encoder is frozen its forward of batch i+1 runs beside the decoder step of
    # batch i (the schedule bench.py measures; parameter updates identical to the sequential one)
    trainer = TeacherForcedTrainer(encoder, decoder, lstm=args.lstmDecoder, decoder_lr=decoderLr,
                                   encoder_lr=args.encoderLr, grad_clip=gradClip, alphaC=alphaC, graph=True,
                                   pipeline=not args.noPipeline)
    run_epochs(args, encoder, decoder, trainer, ck, device)


if __name__ == '__main__':
    main()

"""Evaluation entry point: the reference's ``test.py`` on the MI355X path.

Same CLI (test.py:63-68: ``--checkpoint``, ``--lstmDecoder``, ``--startingLayer``,
``--embeddingName``) plus the data / model knobs ``train.py`` here takes (``--dataFolder``,
``--dataName``, ``--encoder``, ``--batchSize``, ``--workers``).  ``main`` follows test.py:86-135:
load the checkpoint (safe loader, ``checkpoint.load_checkpoint``), build the decoder for
``len(wordMap)``, run ``test`` over the TEST split and write the reference's results CSV
(``results/test-...csv``).  ``test`` follows test.py:144-215: greedy decoding through
``forwardWithoutTeacherForcing`` on the HIP engines, ``preprocessDecoderOutputForMetrics``
loss / top-5 on device, corpus BLEU-1..4 (``metrics.validate`` with ``label="Test"``).
"""
import argparse
import csv
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))

embDim = 512  # test.py:47-51
attentionDim = 512
decoderDim = 512
dropout = 0.5
maxLen = 52
batchSize = 32
workers = 6
alphaC = 1


def parse(argv=None):
    p = argparse.ArgumentParser()
    p.add_argument('--checkpoint', type=str, default=None, help='Path to checkpoint file')
    p.add_argument('--lstmDecoder', action='store_true', help='Use LSTM decoder instead of Transformer')
    p.add_argument('--startingLayer', type=int, default=None, help='Starting layer index for encoder fine-tuning encoder')
    p.add_argument('--embeddingName', type=str, default=None, help='Pretrained embedding name from gensim')
    # MI355X build: where the data lives and which ConvNeXt the checkpoint holds
    p.add_argument('--dataFolder', type=str, default='cocoDataset/inputFiles')
    p.add_argument('--dataName', type=str, default='coco_5_cap_per_img_5_min_word_freq')
    p.add_argument('--encoder', default='base', choices=['tiny', 'small', 'base', 'large'])
    p.add_argument('--batchSize', type=int, default=batchSize)
    p.add_argument('--workers', type=int, default=workers)
    p.add_argument('--resultsDir', type=str, default='results')
    return p.parse_args(argv)


def test(testDataLoader, encoder, decoder, criterion=None, *, wordMap, lstmDecoder, device, maxDecodeLen=maxLen - 1,
         log=print):
    """test.py:144-215 -> (loss avg, top-5 avg, BLEU-1, BLEU-2, BLEU-3, BLEU-4).  ``criterion`` is
    accepted for the reference's signature; the loss is the fused cross-entropy kernel's."""
    from imagecaptioningconvnext_amd.metrics import validate
    return validate(testDataLoader, encoder, decoder, wordMap, lstmDecoder, device, maxDecodeLen=maxDecodeLen,
                    alphaC=alphaC, log=log, label="Test")


def results_name(lstmDecoder, startingLayer, embeddingName):
    """test.py:128-131."""
    if lstmDecoder:
        return f'test-lstmDecoder-TeacherForcing-Finetuning{startingLayer}.csv'
    return f'test-TransformerDecoder-TeacherForcing-Finetuning{startingLayer}-{embeddingName}.csv'


def main(argv=None):
    args = parse(argv)
    if args.embeddingName:
        raise NotImplementedError("gensim pre-trained embeddings are outside the accelerated path")
    if not args.checkpoint:
        raise SystemExit("--checkpoint is required (test.py:97)")
    from torch.utils.data import DataLoader
    from imagecaptioningconvnext_amd.checkpoint import load_checkpoint
    from imagecaptioningconvnext_amd.data import CaptionDataset
    from imagecaptioningconvnext_amd.models.decoder import DecoderWithAttention
    from imagecaptioningconvnext_amd.models.encoder import Encoder
    from imagecaptioningconvnext_amd.models.transformerDecoder import TransformerDecoder

    torch.manual_seed(42)
    device = torch.device("cuda")
    with open(os.path.join(args.dataFolder, 'WORDMAP_' + args.dataName + '.json')) as j:
        wordMap = json.load(j)
    ck = load_checkpoint(args.checkpoint, map_location=device)
    encoder = Encoder(variant=args.encoder)
    E = encoder.encoder_dim
    if args.lstmDecoder:
        decoder = DecoderWithAttention(attention_dim=attentionDim, embed_dim=embDim, decoder_dim=decoderDim,
                                       vocab_size=len(wordMap), dropout=dropout, device=device, encoder_dim=E)
    else:
        decoder = TransformerDecoder(embed_dim=embDim, decoder_dim=decoderDim, vocab_size=len(wordMap), maxLen=maxLen,
                                     dropout=dropout, device=device, wordMap=wordMap, pretrained_embeddings_path=None,
                                     fine_tune_embeddings=True, encoder_dim=E)
    encoder.load_state_dict(ck['encoder'])
    decoder.load_state_dict(ck['decoder'])
    encoder = encoder.to(device)
    decoder = decoder.to(device)
    ds = CaptionDataset(args.dataFolder, args.dataName, 'TEST')
    loader = DataLoader(ds, batch_size=args.batchSize, shuffle=False, num_workers=args.workers, pin_memory=True)
    row = dict(zip(('testLoss', 'testTop5Acc', 'bleu1', 'bleu2', 'bleu3', 'bleu4'),
                   test(loader, encoder, decoder, wordMap=wordMap, lstmDecoder=args.lstmDecoder, device=device)))
    os.makedirs(args.resultsDir, exist_ok=True)
    path = os.path.join(args.resultsDir, results_name(args.lstmDecoder, args.startingLayer, args.embeddingName))
    with open(path, 'w', newline='') as f:
        w = csv.DictWriter(f, fieldnames=list(row))
        w.writeheader()
        w.writerow(row)
    print(f"wrote {path}")
    return row


if __name__ == '__main__':
    main()

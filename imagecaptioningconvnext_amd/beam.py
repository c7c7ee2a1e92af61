"""Beam-search captioning of one image (caption.py:39-255) on the HIP path.

``caption_image_beam_search`` (LSTM-attention) and ``caption_image_beam_search_transformer`` keep
the reference's arguments, control flow and results (the k-beam bookkeeping -- top-k over the
unrolled k x V log-probabilities, completed beams set aside, the beam count shrinking -- is the
reference's, on small device tensors); each decoding step runs on the engines' step-wise
primitives (``decode_step`` / ``decode_select``): the one-step LSTM recurrence kernels, and for
the Transformer the layers on the new position only over a key/value cache that is reordered
with the surviving beams (the reference re-decodes every beam's whole prefix each step).

Image input: a path (PIL read, RGB, 256x256 bicubic, as caption.py:52-58) or a [3, H, W]
tensor; the encoder normalises uint8 pixels on the GPU exactly as caption.py:59-63 does on the
host.  ``caption_image_beam_search_transformer_attention`` (caption.py:260-383, with a
``TransformerDecoderForAttentionViz``) also returns the per-step cross-attention map averaged over
layers and heads: the attention kernel writes its probabilities when asked (imgcap_mha_desc.probs).
"""
import numpy as np
import torch
import torch.nn.functional as F


def load_image(imagePath):
    """caption.py:52-58: RGB, resized to 256x256 (bicubic), [3, 256, 256] uint8 tensor."""
    from PIL import Image
    img = Image.open(imagePath).convert('RGB')
    img = img.resize((256, 256), Image.Resampling.BICUBIC)
    img = np.array(img)
    if len(img.shape) == 2:
        img = np.stack([img, img, img], axis=2)
    return torch.from_numpy(np.ascontiguousarray(img.transpose(2, 0, 1)))


def _encode(encoder, imagePath, dev):
    image = imagePath if torch.is_tensor(imagePath) else load_image(imagePath)
    with torch.no_grad():
        return encoder(image.unsqueeze(0).to(dev))  # (1, enc_image_size, enc_image_size, encoder_dim)


def caption_image_beam_search(encoder, decoder, imagePath, wordMap, beamSize=3):
    """caption.py:39-155 -> (seq: list of word ids incl. <start> / <end>, alphas: nested list
    [len(seq)][enc_image_size][enc_image_size])."""
    k = beamSize
    vocabSize = len(wordMap)
    dev = decoder.fc.weight.device
    encoderOut = _encode(encoder, imagePath, dev)
    encImageSize = encoderOut.size(1)
    encoderDim = encoderOut.size(3)
    encoderOut = encoderOut.reshape(1, -1, encoderDim).expand(k, -1, encoderDim)
    eng = decoder.engine()
    start, end = wordMap['<start>'], wordMap['<end>']
    with torch.no_grad():
        st = eng.decode_init(encoderOut)                                    # caption.py:86
        kPrevWords = torch.full((k,), start, dtype=torch.long, device=dev)
        seqs = kPrevWords.view(k, 1)
        topKScores = torch.zeros(k, 1, device=dev)
        seqsAlpha = torch.ones(k, 1, encImageSize, encImageSize, device=dev)
        completeSeqs, completeSeqsAlpha, completeSeqsScores = [], [], []
        step = 1
        while True:
            logits, alpha = eng.decode_step(st, kPrevWords)                  # caption.py:89-96
            alpha = alpha.view(-1, encImageSize, encImageSize)
            scores = F.log_softmax(logits[:, :vocabSize].float(), dim=1)
            scores = topKScores.expand_as(scores) + scores
            if step == 1:  # all k beams are the same <start> beam
                topKScores, topKWords = scores[0].topk(k, 0, True, True)
            else:
                topKScores, topKWords = scores.view(-1).topk(k, 0, True, True)
            prevWordInds = torch.div(topKWords, vocabSize, rounding_mode='floor')
            nextWordInds = topKWords % vocabSize
            seqs = torch.cat([seqs[prevWordInds], nextWordInds.unsqueeze(1)], dim=1)
            seqsAlpha = torch.cat([seqsAlpha[prevWordInds], alpha[prevWordInds].unsqueeze(1)], dim=1)
            nxt = nextWordInds.tolist()
            incompleteInds = [ind for ind, w in enumerate(nxt) if w != end]
            completeInds = sorted(set(range(len(nxt))) - set(incompleteInds))
            if completeInds:
                completeSeqs.extend(seqs[completeInds].tolist())
                completeSeqsAlpha.extend(seqsAlpha[completeInds].tolist())
                completeSeqsScores.extend(topKScores[completeInds].tolist())
            k -= len(completeInds)
            if k == 0:
                break
            keep = torch.tensor(incompleteInds, device=dev, dtype=torch.long)
            seqs = seqs[keep]
            seqsAlpha = seqsAlpha[keep]
            eng.decode_select(st, prevWordInds[keep])                       # h, c (and rows) of the kept beams
            topKScores = topKScores[keep].unsqueeze(1)
            kPrevWords = nextWordInds[keep]
            if step > 50:
                break
            step += 1
    if not completeSeqsScores:
        raise ValueError("beam search: no beam reached <end> within 51 steps (caption.py:151 would fail too)")
    i = completeSeqsScores.index(max(completeSeqsScores))
    return completeSeqs[i], completeSeqsAlpha[i]


def caption_image_beam_search_transformer(encoder, decoder, imagePath, wordMap, beamSize=3, max_decode_len=51):
    """caption.py:160-255 -> (seq: list of word ids incl. <start> / <end>, None)."""
    return _transformer_beam(encoder, decoder, imagePath, wordMap, beamSize, max_decode_len, False)


def caption_image_beam_search_transformer_attention(encoder, decoder, imagePath, wordMap, filename, beamSize=3,
                                                    max_decode_len=51):
    """caption.py:260-383 -> (seq, alphas: [max_decode_len][num_pixels] nested list, the cross-
    attention of each emitted word averaged over layers and heads, zero past the caption).
    ``filename`` is unused, as in the reference."""
    return _transformer_beam(encoder, decoder, imagePath, wordMap, beamSize, max_decode_len, True)


def _transformer_beam(encoder, decoder, imagePath, wordMap, beamSize, max_decode_len, with_alphas):
    k = beamSize
    vocab_size = len(wordMap)
    end_token_idx = wordMap['<end>']
    dev = decoder.fc_out.weight.device
    encoderOut = _encode(encoder, imagePath, dev)
    encoderDim = encoderOut.size(3)
    eng = decoder.engine()
    try:
        with torch.no_grad():
            st = eng.decode_init(encoderOut.reshape(1, -1, encoderDim).expand(k, -1, encoderDim), max_decode_len)
            num_pixels = st["P"]
            kPrevWords = torch.full((k, 1), wordMap['<start>'], dtype=torch.long, device=dev)
            topKScores = torch.zeros(k, 1, device=dev)
            seqsAlphas = torch.zeros(k, max_decode_len, num_pixels, device=dev) if with_alphas else None
            completeSeqs, completeSeqsScores, completeSeqsAlphas = [], [], []
            step = 0
            while True:
                if with_alphas:
                    eng.cross_probs = []
                logits = eng.decode_step(st, kPrevWords[:, -1].contiguous())    # caption.py:202-216
                scoresActive = F.log_softmax(logits[:, :vocab_size].float(), dim=1)
                scoresActive = topKScores.expand_as(scoresActive) + scoresActive
                if step == 0:
                    topKScoresNew, topKUnrolledIndices = scoresActive[0].topk(k, 0, True, True)
                else:
                    topKScoresNew, topKUnrolledIndices = scoresActive.view(-1).topk(k, 0, True, True)
                prevWordActiveIndices = torch.div(topKUnrolledIndices, vocab_size, rounding_mode='floor')
                nextWordsIds = topKUnrolledIndices % vocab_size
                newKPrevWordsIds = torch.cat([kPrevWords[prevWordActiveIndices], nextWordsIds.unsqueeze(1)], dim=1)
                newTopKScores = topKScoresNew.unsqueeze(1)
                justCompletedMask = nextWordsIds == end_token_idx
                justCompletedIndices = torch.nonzero(justCompletedMask, as_tuple=False).squeeze(1)
                if with_alphas:                                                   # caption.py:332-345
                    # [layers, k, H, 1, P] -> this word's map averaged over layers and heads
                    avg = torch.stack(eng.cross_probs, dim=0)[:, :, :, -1, :].mean(dim=(0, 2))
                    newSeqsAlphas = torch.zeros(k, max_decode_len, num_pixels, device=dev)
                    if step > 0:
                        newSeqsAlphas[:, :step, :] = seqsAlphas[prevWordActiveIndices, :step, :]
                    newSeqsAlphas[:, step, :] = avg[prevWordActiveIndices]
                if len(justCompletedIndices) > 0:
                    completeSeqs.extend(newKPrevWordsIds[justCompletedIndices].tolist())
                    if with_alphas:
                        completeSeqsAlphas.extend(newSeqsAlphas[justCompletedIndices].tolist())
                    completeSeqsScores.extend(newTopKScores[justCompletedIndices].squeeze(1).tolist())
                incompleteIndices = torch.nonzero(~justCompletedMask, as_tuple=False).squeeze(1)
                k -= len(justCompletedIndices)
                if k == 0:
                    break
                kPrevWords = newKPrevWordsIds[incompleteIndices]
                topKScores = newTopKScores[incompleteIndices]
                if with_alphas:
                    seqsAlphas = newSeqsAlphas[incompleteIndices]
                eng.decode_select(st, prevWordActiveIndices[incompleteIndices])  # caches follow their beams
                if step + 1 >= max_decode_len:
                    break
                step += 1
    finally:
        eng.cross_probs = None
    if not completeSeqsScores:
        raise ValueError("beam search: no beam reached <end> within max_decode_len steps")
    i = completeSeqsScores.index(max(completeSeqsScores))
    return completeSeqs[i], (completeSeqsAlphas[i] if with_alphas else None)

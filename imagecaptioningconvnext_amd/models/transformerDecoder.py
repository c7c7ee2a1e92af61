"""Transformer decoder with the reference's class surface (models/transformerDecoder.py:14-168).

``TransformerDecoder`` keeps the constructor signature, submodules (embedding, pos_encoding,
dropout, transformer_decoder = nn.TransformerDecoder of 6 post-norm nn.TransformerDecoderLayer,
fc_out, encoder_proj) and state-dict keys, so reference checkpoints load.  forward(
teacherForcing=True, ...) returns ``(predictions[B, L, V], encoded_captions, decode_lengths)``
and is differentiable; the compute runs on the HIP engine (transformer_engine.py).

Out of the accelerated path: gensim pre-trained embeddings
(loadPretrainedWordEmbeddings, transformerDecoder.py:29-42 — the word2vec variant also forces
6 heads of dim 50, which the head-dim-64 attention kernel does not take) and greedy
non-teacher-forced decoding (:110-160).
"""
import math

import torch
from torch import nn


class PositionalEncoding(nn.Module):
    """Sinusoidal table, buffer ``pe`` [1, maxLen, embed_dim] (transformerDecoder.py:14-27)."""

    def __init__(self, embed_dim, maxLen):
        super().__init__()
        pos = torch.arange(maxLen, dtype=torch.float32)[:, None]
        inv = torch.exp(torch.arange(0, embed_dim, 2, dtype=torch.float32) * (-math.log(10000.0) / embed_dim))
        table = torch.zeros(maxLen, embed_dim)
        table[:, 0::2] = torch.sin(pos * inv)
        table[:, 1::2] = torch.cos(pos * inv)
        self.register_buffer("pe", table[None])

    def forward(self, x):
        return x + self.pe[:, : x.size(1)]


class _TransformerTF(torch.autograd.Function):
    @staticmethod
    def forward(ctx, engine, encoder_out, caps, caplens, key_ids, pad_id, *params):
        s = engine.forward(encoder_out, caps, caplens, key_ids=key_ids, pad_id=pad_id, loss=False)
        ctx.engine, ctx.s = engine, s
        ctx.enc_shape, ctx.enc_dtype = encoder_out.shape, encoder_out.dtype
        return engine.predictions(s)

    @staticmethod
    def backward(ctx, dpred):
        eng, s = ctx.engine, ctx.s
        B, L, V = dpred.shape
        dl = torch.zeros(B * L, eng.Vpad, device=dpred.device, dtype=eng.ct)
        dl[:, :V] = dpred.reshape(B * L, V).to(eng.ct)
        gbuf = torch.empty_like(eng.fp.grad)
        eng.backward(s, dlogits=dl, gbuf=gbuf, want_denc=bool(ctx.needs_input_grad[1]))
        denc = s["denc"].reshape(ctx.enc_shape).to(ctx.enc_dtype) if s["denc"] is not None else None
        grads = tuple(eng.fp.g(n, buf=gbuf) for n in eng.fp.params)
        return (None, denc, None, None, None, None) + grads


class TransformerDecoder(nn.Module):
    def __init__(self, embed_dim, decoder_dim, vocab_size, maxLen, device, wordMap, pretrained_embeddings_path,
                 fine_tune_embeddings, dropout=0.5, encoder_dim=1024, num_heads=8, num_layers=6,
                 compute_dtype=torch.bfloat16):
        super().__init__()
        if pretrained_embeddings_path:
            raise NotImplementedError("gensim pre-trained embeddings are outside the accelerated path")
        self.encoder_dim = encoder_dim
        self.decoder_dim = decoder_dim
        self.embed_dim = embed_dim
        self.vocab_size = vocab_size
        self.num_heads = num_heads
        self.num_layers = num_layers
        self.dropout_p = dropout
        self.embedding = nn.Embedding(vocab_size, embed_dim)
        self.pos_encoding = PositionalEncoding(embed_dim, maxLen)
        self.dropout = nn.Dropout(p=dropout)
        layer = nn.TransformerDecoderLayer(d_model=embed_dim, nhead=num_heads, dim_feedforward=decoder_dim,
                                           dropout=dropout)
        self.transformer_decoder = nn.TransformerDecoder(layer, num_layers=num_layers)
        self.fc_out = nn.Linear(embed_dim, vocab_size)
        self.encoder_proj = nn.Linear(encoder_dim, embed_dim) if encoder_dim != embed_dim else nn.Identity()
        self.device = device
        self.wordMap = wordMap
        self.compute_dtype = compute_dtype
        self._engine = None

    def engine(self):
        from ..transformer_engine import TransformerEngine
        dev = self.fc_out.weight.device
        if dev.type != "cuda":
            raise RuntimeError("TransformerDecoder runs on the HIP kernels; move it to the GPU first")
        if self._engine is None or not self._engine.fp.check_bound():
            self._engine = TransformerEngine(self, dev, self.compute_dtype)
        return self._engine

    def forwardWithTeacherForcing(self, encoder_out, encoded_captions, caption_lengths, tgt_key_padding_mask):
        eng = self.engine()
        decode_lengths = (caption_lengths.squeeze(1) - 1).tolist()  # transformerDecoder.py:92
        if tgt_key_padding_mask is None:
            key_ids, pad_id = None, -1  # no padding mask (-1 never matches a token id)
            key_ids = torch.zeros_like(encoded_captions)
            pad_id = 1
        else:
            key_ids, pad_id = tgt_key_padding_mask.to(torch.int64).contiguous(), 1
        preds = _TransformerTF.apply(eng, encoder_out, encoded_captions, caption_lengths, key_ids, pad_id,
                                     *eng.fp.params.values())
        return preds, encoded_captions, decode_lengths

    def forwardWithoutTeacherForcing(self, encoder_out, wordMap, maxDecodeLen):
        """transformerDecoder.py:110-160: greedy decoding -> (predictions [B, maxDecodeLen, V] f32,
        sequences [B, maxDecodeLen] int64); TransformerEngine.greedy (key/value cache instead of
        re-decoding the prefix).  Not differentiable."""
        with torch.no_grad():
            return self.engine().greedy(encoder_out, wordMap['<start>'], wordMap['<end>'], maxDecodeLen)

    def forward(self, teacherForcing, encoder_out, encoded_captions=None, caption_lengths=None,
                tgt_key_padding_mask=None, wordMap=None, maxDecodeLen=None):
        if teacherForcing is True:
            return self.forwardWithTeacherForcing(encoder_out, encoded_captions, caption_lengths,
                                                  tgt_key_padding_mask)
        return self.forwardWithoutTeacherForcing(encoder_out, wordMap, maxDecodeLen)

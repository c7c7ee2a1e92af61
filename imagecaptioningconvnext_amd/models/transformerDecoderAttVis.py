"""Attention-visualisation Transformer decoder with the reference's class surface
(models/transformerDecoderAttVis.py:40-239).

``TransformerDecoderForAttentionViz`` keeps the constructor signature, submodule names and
state-dict keys (``decoder_layers.{i}.self_attn.in_proj_weight`` ..., so its checkpoints and the
``remap_transformer_decoder_keys`` output of caption.py:418 load) and the forward return tuples:
teacher forcing -> ``(predictions [B, L, V], encoded_captions, decode_lengths, alphas [H, B, P])``
and greedy -> ``(predictions, sequences, alphas [B, maxDecodeLen, P])``.  The layers are the
post-norm ReLU decoder layers of transformerDecoder.py with the same arithmetic, so they run on
the same HIP engine (transformer_engine.py); the cross-attention probabilities the reference gets
from ``nn.MultiheadAttention(need_weights=True, average_attn_weights=False)`` are written by the
attention kernel itself (``imgcap_mha_desc.probs``) and averaged as the reference averages them.
"""
import torch
from torch import nn

from .transformerDecoder import PositionalEncoding, _TransformerTF


class CustomTransformerDecoderLayer(nn.Module):
    """Parameter holder with transformerDecoderAttVis.py:40-62's submodules.  The engine runs
    its forward (post-norm, ReLU: the configuration TransformerDecoderForAttentionViz builds)."""

    def __init__(self, d_model, nhead, dim_feedforward=2048, dropout=0.1, activation="relu", layer_norm_eps=1e-5,
                 batch_first=False, norm_first=False, device=None, dtype=None):
        super().__init__()
        if activation != "relu" or norm_first or batch_first or layer_norm_eps != 1e-5:
            raise NotImplementedError("the HIP decoder layer is post-norm, ReLU, seq-first, eps 1e-5")
        kw = {'device': device, 'dtype': dtype}
        self.self_attn = nn.MultiheadAttention(d_model, nhead, dropout=dropout, batch_first=batch_first, **kw)
        self.multihead_attn = nn.MultiheadAttention(d_model, nhead, dropout=dropout, batch_first=batch_first, **kw)
        self.linear1 = nn.Linear(d_model, dim_feedforward, **kw)
        self.dropout_ffn = nn.Dropout(dropout)
        self.linear2 = nn.Linear(dim_feedforward, d_model, **kw)
        self.norm1 = nn.LayerNorm(d_model, eps=layer_norm_eps, **kw)
        self.norm2 = nn.LayerNorm(d_model, eps=layer_norm_eps, **kw)
        self.norm3 = nn.LayerNorm(d_model, eps=layer_norm_eps, **kw)
        self.dropout1 = nn.Dropout(dropout)
        self.dropout2 = nn.Dropout(dropout)
        self.dropout3 = nn.Dropout(dropout)
        self.norm_first = norm_first
        self.batch_first = batch_first


class TransformerDecoderForAttentionViz(nn.Module):
    layer_prefix = "decoder_layers"  # parameter names the engine reads (transformerDecoderAttVis.py:123)

    def __init__(self, embed_dim, decoder_dim, vocab_size, maxLen, device, dropout=0.5, encoder_dim=1024,
                 num_heads=8, num_layers=6, compute_dtype=torch.bfloat16):
        super().__init__()
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
        self.decoder_layers = nn.ModuleList([
            CustomTransformerDecoderLayer(d_model=embed_dim, nhead=num_heads, dim_feedforward=decoder_dim,
                                          dropout=dropout, batch_first=False) for _ in range(num_layers)])
        self.fc_out = nn.Linear(embed_dim, vocab_size)
        self.encoder_proj = nn.Linear(encoder_dim, embed_dim) if encoder_dim != embed_dim else nn.Identity()
        self.device = device
        self.compute_dtype = compute_dtype
        self._engine = None

    def engine(self):
        from ..transformer_engine import TransformerEngine
        dev = self.fc_out.weight.device
        if dev.type != "cuda":
            raise RuntimeError("TransformerDecoderForAttentionViz runs on the HIP kernels; move it to the GPU first")
        if self._engine is None or not self._engine.fp.check_bound():
            self._engine = TransformerEngine(self, dev, self.compute_dtype)
        return self._engine

    def forwardWithTeacherForcing(self, encoder_out, encoded_captions, caption_lengths, tgt_key_padding_mask):
        """transformerDecoderAttVis.py:132-167; alphas = the layers' cross-attention probabilities
        [layers, B, H, L, P] averaged over layers and query positions, permuted to [H, B, P]."""
        eng = self.engine()
        decode_lengths = (caption_lengths.squeeze(1) - 1).tolist()
        if tgt_key_padding_mask is None:
            key_ids, pad_id = torch.zeros_like(encoded_captions), 1
        else:
            key_ids, pad_id = tgt_key_padding_mask.to(torch.int64).contiguous(), 1
        eng.cross_probs = []
        try:
            preds = _TransformerTF.apply(eng, encoder_out, encoded_captions, caption_lengths, key_ids, pad_id,
                                         *eng.fp.params.values())
            alphas = torch.stack(eng.cross_probs, dim=0).mean(dim=(0, 3)).permute(1, 0, 2)
        finally:
            eng.cross_probs = None
        return preds, encoded_captions, decode_lengths, alphas

    def forwardWithoutTeacherForcing(self, encoder_out, wordMap, maxDecodeLen):
        """transformerDecoderAttVis.py:170-229: greedy decoding with the key/value-cached step
        (TransformerEngine.decode_step); alphas[b, t] = the cross-attention of row b's word t
        averaged over layers and heads, left 0 once the row has emitted <end>."""
        eng = self.engine()
        from .. import kernels as K
        with torch.no_grad():
            st = eng.decode_init(encoder_out, maxDecodeLen)
            B, V, dev = st["B"], self.vocab_size, encoder_out.device
            preds = torch.zeros(B, maxDecodeLen, V, device=dev, dtype=torch.float32)
            seqs = torch.zeros(B, maxDecodeLen, device=dev, dtype=torch.int64)
            alphas = torch.zeros(B, maxDecodeLen, st["P"], device=dev, dtype=torch.float32)
            finished = torch.zeros(B, device=dev, dtype=torch.uint8)
            ids = torch.full((B,), wordMap['<start>'], device=dev, dtype=torch.int64)
            try:
                for t in range(maxDecodeLen):
                    eng.cross_probs = []
                    logits = eng.decode_step(st, ids)
                    avg = torch.stack(eng.cross_probs, dim=0)[:, :, :, -1, :].mean(dim=(0, 2))   # :223-225
                    # rows not yet finished: predictions, sequences and alphas[b, t] (:213-226)
                    K.greedy_select(logits, V, t, wordMap['<end>'], finished, ids, seqs, preds,
                                    alpha=avg.contiguous(), alphas=alphas)
            finally:
                eng.cross_probs = None
        return preds, seqs, alphas

    def forward(self, teacherForcing, encoder_out, encoded_captions=None, caption_lengths=None,
                tgt_key_padding_mask=None, wordMap=None, maxDecodeLen=None):
        if teacherForcing is True:
            return self.forwardWithTeacherForcing(encoder_out, encoded_captions, caption_lengths,
                                                  tgt_key_padding_mask)
        return self.forwardWithoutTeacherForcing(encoder_out, wordMap, maxDecodeLen)

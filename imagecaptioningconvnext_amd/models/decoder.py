"""LSTM + soft-attention decoder with the reference's class surface (models/decoder.py:16-172).

``Attention`` and ``DecoderWithAttention`` keep the constructor signatures, submodule names
(attention.{encoder_att,decoder_att,full_att}, embedding, dropout, decode_step, init_h,
init_c, f_beta, sigmoid, fc) and state-dict keys of the reference, so its checkpoints load.

forward(teacherForcing=True, ...) returns exactly the reference tuple
``(predictions[B,T,V] zero-filled, caps_sorted, decode_lengths(list), alphas[B,T,P], sort_ind)``
and is differentiable; it runs on the HIP engine (lstm_engine.LstmEngine).  The fused train
step (train_step.py) calls the engine directly so logits feed the CE kernel without the
[B,T,V] fp32 round trip.  Non-teacher-forced decoding is outside the hot path.
"""
import torch
from torch import nn


class Attention(nn.Module):
    """decoder.py:16-31 parameter surface; the TF hot path never calls forward (the fused
    recurrence kernel computes it); forward is provided for API completeness (beam search)."""

    def __init__(self, encoder_dim, decoder_dim, attention_dim):
        super().__init__()
        self.encoder_att = nn.Linear(encoder_dim, attention_dim)
        self.decoder_att = nn.Linear(decoder_dim, attention_dim)
        self.full_att = nn.Linear(attention_dim, 1)
        self.relu = nn.ReLU()
        self.softmax = nn.Softmax(dim=1)

    def forward(self, encoder_out, decoder_hidden):
        scores = self.full_att(self.relu(self.encoder_att(encoder_out)
                                         + self.decoder_att(decoder_hidden)[:, None, :]))[..., 0]
        weights = self.softmax(scores)
        return torch.einsum("bp,bpe->be", weights, encoder_out), weights


class _LstmTF(torch.autograd.Function):
    """Differentiable wrapper: inputs are the module's parameters (in FlatParams order) and the
    encoder output; outputs predictions and alphas like the reference.  Backward runs the HIP
    BPTT into a scratch flat buffer and hands autograd one view per parameter."""

    @staticmethod
    def forward(ctx, engine, encoder_out, caps, caplens, *params):
        s = engine.forward(encoder_out, caps, caplens, fixed_T=False, loss=False)
        preds = engine.predictions(s)
        ctx.engine, ctx.s = engine, s
        ctx.enc_shape, ctx.enc_dtype = encoder_out.shape, encoder_out.dtype
        ctx.mark_non_differentiable(s["caps_s"], s["sort_ind"])
        return preds, s["alphas"], s["caps_s"], s["sort_ind"]

    @staticmethod
    def backward(ctx, dpred, dalpha, _a, _b):
        eng, s = ctx.engine, ctx.s
        B, T, V = dpred.shape
        dl = torch.zeros(B * T, eng.Vpad, device=dpred.device, dtype=eng.ct)
        mask = s["tmask"].reshape(-1, 1)
        dl[:, :V] = (dpred.reshape(B * T, V) * mask).to(eng.ct)
        da = None if dalpha is None else (dalpha * s["tmask"][..., None]).contiguous().float()
        want = encoder_out_needs_grad(ctx)
        gbuf = torch.empty_like(eng.fp.grad)
        eng.backward(s, dlogits=dl, dalpha=da, gbuf=gbuf, want_denc=want)
        grads = tuple(eng.fp.g(n, buf=gbuf) for n in eng.fp.params)
        denc = s["denc"].view(ctx.enc_shape).to(ctx.enc_dtype) if want else None
        return (None, denc, None, None) + grads


class DecoderWithAttention(nn.Module):
    def __init__(self, attention_dim, embed_dim, decoder_dim, vocab_size, device, encoder_dim=1024, dropout=0.5,
                 compute_dtype=torch.bfloat16):
        super().__init__()
        self.encoder_dim = encoder_dim
        self.attention_dim = attention_dim
        self.embed_dim = embed_dim
        self.decoder_dim = decoder_dim
        self.vocab_size = vocab_size
        self.dropout_p = dropout
        self.attention = Attention(encoder_dim, decoder_dim, attention_dim)
        self.embedding = nn.Embedding(vocab_size, embed_dim)
        self.dropout = nn.Dropout(p=dropout)
        self.decode_step = nn.LSTMCell(embed_dim + encoder_dim, decoder_dim, bias=True)
        self.init_h = nn.Linear(encoder_dim, decoder_dim)
        self.init_c = nn.Linear(encoder_dim, decoder_dim)
        self.f_beta = nn.Linear(decoder_dim, encoder_dim)
        self.sigmoid = nn.Sigmoid()
        self.fc = nn.Linear(decoder_dim, vocab_size)
        self.init_weights()
        self.device = device
        self.compute_dtype = compute_dtype
        self._engine = None

    def init_weights(self):
        """decoder.py:58-61: U(-0.1, 0.1) embedding and fc weight, zero fc bias."""
        with torch.no_grad():
            self.embedding.weight.uniform_(-0.1, 0.1)
            self.fc.bias.zero_()
            self.fc.weight.uniform_(-0.1, 0.1)

    def init_hidden_state(self, encoder_out):
        mean_encoder_out = encoder_out.mean(dim=1)
        return self.init_h(mean_encoder_out), self.init_c(mean_encoder_out)

    def engine(self):
        """HIP engine bound to this module's parameters (flattened on first use on the GPU)."""
        from ..lstm_engine import LstmEngine
        dev = self.fc.weight.device
        if dev.type != "cuda":
            raise RuntimeError("DecoderWithAttention runs on the HIP kernels; move it to the GPU first")
        if self._engine is None or not self._engine.fp.check_bound():
            self._engine = LstmEngine(self, dev, self.compute_dtype)
        return self._engine

    def forwardWithTeacherForcing(self, encoder_out, encoded_captions, caption_lengths):
        eng = self.engine()
        preds, alphas, caps_s, sort_ind = _LstmTF.apply(eng, encoder_out, encoded_captions, caption_lengths,
                                                        *eng.fp.params.values())
        return preds, caps_s, _decode_lengths(caption_lengths), alphas, sort_ind

    def forwardWithoutTeacherForcing(self, encoder_out, wordMap, maxDecodeLen):
        """decoder.py:119-163: greedy decoding -> (predictions [B, maxDecodeLen, V] f32, alphas
        [B, maxDecodeLen, P] f32, sequences [B, maxDecodeLen] int64); LstmEngine.greedy.  Not
        differentiable (the reference's trainWithoutTeacherForcing is outside this build)."""
        with torch.no_grad():
            return self.engine().greedy(encoder_out, wordMap['<start>'], wordMap['<end>'], maxDecodeLen)

    def forward(self, teacherForcing, encoder_out, encoded_captions=None, caption_lengths=None, wordMap=None,
                maxDecodeLen=None):
        if teacherForcing is True:
            return self.forwardWithTeacherForcing(encoder_out, encoded_captions, caption_lengths)
        return self.forwardWithoutTeacherForcing(encoder_out, wordMap, maxDecodeLen)


def encoder_out_needs_grad(ctx):
    return bool(ctx.needs_input_grad[1])


def _decode_lengths(caption_lengths):
    lens = caption_lengths.reshape(-1).sort(descending=True, stable=True).values
    return (lens - 1).tolist()

"""Explicit forward/backward engine of the teacher-forced LSTM-attention decoder on HIP.

Mirrors DecoderWithAttention.forwardWithTeacherForcing (models/decoder.py:69-113) plus the
loss of train.py:263-269; the recurrence itself is one native call per direction
(imgcap_lstm_tf_fwd / _bwd, csrc/lstm.hip).  Every GEMM is imgcap_gemm; the loss is the
fused CE + top-5 kernel; parameters, grads, Adam state and the bf16 weight copy live in one
FlatParams buffer whose groups make the concatenated operands zero-copy views:

  hcat  = [attention.decoder_att.weight; f_beta.weight; decode_step.weight_hh]   [A+E+4D, D]
  bhcat = [attention.decoder_att.bias;   f_beta.bias;   decode_step.bias_hh]     [A+E+4D]
  init  = [init_h.weight; init_c.weight] [2D, E],  binit = [init_h.bias; init_c.bias]
"""
import ctypes
import os

import torch

from . import _abi
from . import kernels as K
from .flat import FlatParams

# weight gradients: long-K fp32 products into the gradient buffer, K sliced over the
# grid (imgcap_epilogue.split_k)
DW = dict(split_k=-1)

_STREAM_DROPOUT_H = 11  # dropout stream id for fc(dropout(h)) (decoder.py:109)


def lstm_param_groups(dec):
    n = dict(dec.named_parameters())
    order = [
        ["attention.decoder_att.weight", "f_beta.weight", "decode_step.weight_hh"],
        ["attention.decoder_att.bias", "f_beta.bias", "decode_step.bias_hh"],
        ["init_h.weight", "init_c.weight"],
        ["init_h.bias", "init_c.bias"],
        ["decode_step.weight_ih"], ["decode_step.bias_ih"],
        ["attention.encoder_att.weight"], ["attention.encoder_att.bias"],
        ["attention.full_att.weight"], ["attention.full_att.bias"],
        ["embedding.weight"], ["fc.weight"], ["fc.bias"],
    ]
    seen = {x for g in order for x in g}
    assert seen == set(n), f"unexpected decoder parameters: {set(n) ^ seen}"
    return [[(k, n[k]) for k in g] for g in order]


class LstmEngine:
    def __init__(self, dec, device, compute_dtype=torch.bfloat16):
        self.dec = dec
        self.ct = compute_dtype
        self.fp = FlatParams(lstm_param_groups(dec), device, compute_dtype)
        self.E, self.A, self.D = dec.encoder_dim, dec.attention_dim, dec.decoder_dim
        self.M, self.V = dec.embed_dim, dec.vocab_size
        self.W3 = self.A + self.E + 4 * self.D
        self.Vpad = (self.V + 7) // 8 * 8
        self.seed = 1234
        self.step_id = 0
        self._y_cnt = None
        self._sync = None
        self._chain_sync = []
        self._retired_sync = []  # superseded hand-off word buffers (captured graphs may point at them)

    # K-slices of the backward step GEMMs (imgcap_lstm_desc.x_slices / y_slices).  Measured at
    # the C2 shape (B=32, D=512, tools/gpu/lstm_sweep.sh): x 2 / y 3 (80 x 2 and 32 x 3 blocks)
    # 24.4 us/step; the former x 3 / y 8 (more blocks, each a shorter K) 26.7; y 16 33
    X_SLICES = int(os.environ.get("IMGCAP_LSTM_XS", "2"))
    Y_SLICES = int(os.environ.get("IMGCAP_LSTM_YS", "3"))
    # The batch rows are independent sequences, so the recurrence can run as CHAINS chains of
    # B / CHAINS rows, each on its own HIP stream (forked from / joined to the caller's stream,
    # graph-capturable).  Measured on MI355X (tools/microbench.py lstm): two chains take 1.85x
    # the time of one -- the step kernels of concurrent streams do not overlap (also with 8 or
    # 16 hardware queues) -- so the default is one chain; kept as a switch (IMGCAP_LSTM_CHAINS).
    # With the persistent forward (one launch per chain, own flag words) two chains are also
    # serialised: 1.80 ms vs 0.96 ms for one (tools/gpu/lp2.sh).
    CHAINS = int(os.environ.get("IMGCAP_LSTM_CHAINS", "1"))
    # Row groups of the persistent recurrences inside their one launch (imgcap_lstm_desc.row_groups:
    # 0 = library default, 4 | mask = bit 0 forward, bit 1 backward split); the trainer picks
    # it per schedule (train_step.TeacherForcedTrainer).
    row_groups = 0

    def _per_row_bytes(self, T, P):
        """Byte stride per batch row of every row-indexed imgcap_lstm_desc pointer."""
        E, A, D, W3 = self.E, self.A, self.D, self.W3
        c = 2 if self.ct == torch.bfloat16 else 4
        npc = (P + 6) // 7
        return dict(enc=P * E * c, att1=P * A * c, xe=T * 4 * D * 4, c0=D * 4, dl=4, g1=T * W3 * 4,
                    alphas=T * P * 4, awe=T * E * 4, zs=T * E * c, gates=T * 4 * D * 4, cs=T * D * 4, hs=T * D * c,
                    hprev=T * D * c, dhs=T * D * c, dalpha=T * P * 4, dcat=T * W3 * c, dh=D * 4, dc=D * 4,
                    de=T * P * 4, datt1=P * A * c, dwf=npc * A * 4, dbea=npc * A * 4, dawe=(T + 1) * E * 4)

    def _sync_words(self, d, dev):
        """Point ``d.sync`` at the engine's hand-off flag words when the persistent forward
        recurrence covers this shape (imgcap_lstm_sync_words > 0).  Caller-owned, allocated once
        (grown during warm-up, before any graph capture)."""
        words = _abi.lib().imgcap_lstm_sync_words(ctypes.byref(d))
        if words <= 0:
            return
        if self._sync is None or self._sync.numel() < words or self._sync.device != dev:
            if self._sync is not None:  # a captured graph may still point at it: keep it alive
                self._retired_sync.append(self._sync)
            self._sync = torch.zeros(max(words + 6400, 8192), dtype=torch.int32, device=dev)  # + diagnostics stamps
        d.sync, d.sync_words = self._sync.data_ptr(), self._sync.numel()

    def sync_error(self):
        """Non-zero when the last persistent recurrence gave up on a hand-off (bounded spin)."""
        return 0 if self._sync is None else int(self._sync[0].item())

    def _fold_status(self, dst, init=False):
        """dst[0] (= / +=) the persistent recurrences' error words (word 0 of every sync buffer in
        use), on the stream: a timed-out hand-off leaves that step's outputs invalid, and the
        trainer raises on it instead of training on them (train_step._update / drain_metrics)."""
        words = [self._sync] if self._sync is not None else []
        if self.CHAINS > 1:
            words += list(self._chain_sync)
        if init and len(words) == 1:
            dst.copy_(words[0][0:1])  # one launch instead of zero + add
            return
        if init:
            dst.zero_()
        for w in words:
            dst.add_(w[0:1])

    def _chain_rows(self, B):
        n = max(1, min(self.CHAINS, B))
        return [(i * B // n, (i + 1) * B // n) for i in range(n)]

    def _launch(self, fn, d, ws=None):
        """Run imgcap_lstm_tf_fwd / _bwd over the row chains of ``d``; ws[i] = per-chain workspace
        pointers (dz, ws_y, y_cnt) for the backward."""
        rows = self._chain_rows(d.B)
        if len(rows) == 1:
            if ws:
                for k, v in ws[0].items():
                    setattr(d, k, v.data_ptr())
            _abi.call(fn, ctypes.byref(d), K.stream())
            return
        main = torch.cuda.current_stream()
        if getattr(self, "_streams", None) is None or len(self._streams) < len(rows) - 1:
            prio = int(os.environ.get("IMGCAP_LSTM_STREAM_PRIO", "0"))
            self._streams = [torch.cuda.Stream(device=main.device, priority=prio) for _ in range(len(rows) - 1)]
        per = self._per_row_bytes(d.T, d.P)
        for i, (b0, b1) in enumerate(rows):
            sd = _abi.LstmDesc()
            ctypes.memmove(ctypes.byref(sd), ctypes.byref(d), ctypes.sizeof(d))
            sd.B = b1 - b0
            for f, nb in per.items():
                v = getattr(sd, f)
                if v:
                    setattr(sd, f, v + b0 * nb)
            sd.sync, sd.sync_words = None, 0
            if d.sync:  # persistent recurrence per chain: each chain its own flag words
                words = _abi.lib().imgcap_lstm_sync_words(ctypes.byref(sd))
                if words > 0:
                    cur = self._chain_sync[i] if len(self._chain_sync) > i else None
                    if cur is None or cur.device != main.device or cur.numel() < words:
                        # grown during warm-up, before any capture (a captured graph keeps its own)
                        new = torch.zeros(max(words, 8192), dtype=torch.int32, device=main.device)
                        if cur is not None:
                            self._retired_sync.append(cur)
                        self._chain_sync = self._chain_sync[:i] + [new] + self._chain_sync[i + 1:]
                    sd.sync, sd.sync_words = self._chain_sync[i].data_ptr(), self._chain_sync[i].numel()
            if ws:
                for k, v in ws[i].items():
                    setattr(sd, k, v.data_ptr())
            st = main if i == 0 else self._streams[i - 1]
            if i:
                K.fork(st, main)
            _abi.call(fn, ctypes.byref(sd), st.cuda_stream)
        for st in self._streams[:len(rows) - 1]:
            K.join(main, st)

    # ---------------------------------------------------------------------------------------
    def _side_stream(self, dev):
        """A second stream for work off the recurrence's critical path (forked / joined with
        events, so it is captured into the step's graph like the main stream)."""
        if getattr(self, "_side", None) is None or self._side.device != dev:
            self._side = torch.cuda.Stream(device=dev)
        return self._side

    def weights(self):
        fp, A, E, D, M, V = self.fp, self.A, self.E, self.D, self.M, self.V
        return dict(
            hcat=fp.w("attention.decoder_att.weight", (self.W3, D), self.W3 * D),
            bhcat=fp.f32("attention.decoder_att.bias", (self.W3,), self.W3),
            init=fp.w("init_h.weight", (2 * D, E), 2 * D * E),
            binit=fp.f32("init_h.bias", (2 * D,), 2 * D),
            wih=fp.w("decode_step.weight_ih"), bih=fp.f32("decode_step.bias_ih"),
            wea=fp.w("attention.encoder_att.weight"), bea=fp.f32("attention.encoder_att.bias"),
            wf=fp.f32("attention.full_att.weight", (A,)),
            emb=fp.f32("embedding.weight"),
            wfc=fp.w("fc.weight"), bfc=fp.f32("fc.bias"),
        )

    def forward(self, encoder_out, encoded_captions, caption_lengths, *, fixed_T=False, dropout=None, loss=True,
                alphaC=1.0):
        """Runs decoder.py:69-113 (+ the train.py:265-269 loss when ``loss``).

        fixed_T: run T = L-1 steps (True) or the given number of steps (an int >= every decode
        length: the trainer's length buckets) without reading decode lengths on the host (no sync;
        rows are masked on device).  Otherwise T = max(decode_lengths) exactly as the reference.
        Returns a dict of saved buffers (``s``) used by backward()."""
        ct, dev = self.ct, encoder_out.device
        A, E, D, M, V, W3 = self.A, self.E, self.D, self.M, self.V, self.W3
        p_drop = self.dec.dropout_p if (dropout is None and self.dec.training) else (dropout or 0.0)
        w = self.weights()
        B = encoder_out.size(0)
        enc = encoder_out.reshape(B, -1, E)
        P = enc.size(1)
        L = encoded_captions.size(1)
        lens = caption_lengths.reshape(-1)
        mean = None
        if (B <= 256 and enc.dtype == ct and enc.is_contiguous() and lens.dtype == torch.int64
                and encoded_captions.dtype == torch.int64 and encoded_captions.is_contiguous()):
            # decoder.py:64,79-81 (sort, gathers, decode lengths, pixel mean) in one launch
            enc_s, mean, caps_s, sort_ind, dl = K.sort_gather_rows(lens.contiguous(), enc, encoded_captions)
        else:
            lens, sort_ind = lens.sort(dim=0, descending=True, stable=True)
            enc_s = enc.index_select(0, sort_ind).to(ct).contiguous()
            caps_s = encoded_captions.index_select(0, sort_ind)
            dl = (lens - 1).to(torch.int32)
        if fixed_T:
            # True: T = L - 1; an int: that many steps (a length bucket >= every decode length of
            # the batch -- the rows past a caption's length are masked either way)
            T = L - 1 if fixed_T is True else max(1, min(int(fixed_T), L - 1))
            dls = None
        else:
            dls = dl.tolist()  # decoder.py:91 (host list, part of the reference API)
            T = max(dls)
        s = dict(B=B, P=P, T=T, L=L, sort_ind=sort_ind, caps_s=caps_s, dl=dl, dls=dls, p_drop=p_drop,
                 seed=self.seed + self.step_id)
        self.step_id += 1
        f32 = dict(device=dev, dtype=torch.float32)
        ctd = dict(device=dev, dtype=ct)
        # ---- loop-invariant precompute ------------------------------------------------------
        ids = caps_s[:, :T].contiguous()
        emb = torch.empty(B * T, M, **ctd)
        K.embedding_fwd(ids, w["emb"], emb)                                   # decoder.py:84
        if mean is None:
            mean = torch.empty(B, E, **ctd)
            K.mean_mid(enc_s, mean)                                           # decoder.py:64
        main = torch.cuda.current_stream(dev)
        side = self._side_stream(dev)
        # att1 = enc W_ea (decoder.py:61, hoisted out of the loop) on the side stream, beside the
        # init_h / init_c and W_ih-embedding products (no library scratch: 64x64 tile, one pass)
        K.fork(side, main)
        with torch.cuda.stream(side):
            att1 = K.gemm(enc_s.view(B * P, E), w["wea"], trans_b=True, bias=w["bea"])
            ev_att1 = torch.cuda.Event()
            ev_att1.record(side)
        att1.record_stream(main)
        h0c0 = K.gemm(mean, w["init"], trans_b=True, bias=w["binit"], out_dtype=torch.float32)  # :100-101
        xe = K.gemm(emb, w["wih"][:, :M], trans_b=True, bias=w["bih"], out_dtype=torch.float32)  # W_ih emb half
        hprev = torch.empty(B, T, D, **ctd)
        hprev[:, 0].copy_(h0c0[:, :D])
        c0 = h0c0[:, D:].contiguous()
        g1 = torch.empty(B, T, W3, **f32)
        alphas = torch.empty(B, T, P, **f32)
        awe = torch.empty(B, T, E, **f32)
        zs = torch.empty(B, T, E, **ctd)
        gates = torch.empty(B, T, 4 * D, **f32)
        cs = torch.empty(B, T, D, **f32)
        hs = torch.empty(B, T, D, **ctd)
        d = _abi.LstmDesc()
        d.dtype, d.B, d.P, d.E, d.A, d.D, d.M, d.T = K.dt(emb), B, P, E, A, D, M, T
        for k, v in dict(w_hcat=w["hcat"], b_hcat=w["bhcat"], w_ih=w["wih"], w_f=w["wf"], enc=enc_s, att1=att1,
                         xe=xe, c0=c0, dl=dl, g1=g1, alphas=alphas, awe=awe, zs=zs, gates=gates, cs=cs, hs=hs,
                         hprev=hprev).items():
            setattr(d, k, v.data_ptr())
        d.row_groups = self.row_groups
        self._sync_words(d, dev)
        # k-major copies of the weights the backward recurrence multiplies by, made on a side
        # stream under the forward recurrence (they only depend on the weights)
        with torch.cuda.stream(side):
            wzh_t = torch.empty(E + D, 4 * D, **ctd)                  # [W_ih[:, M:] | W_hh]^T
            K.transpose(w["wih"][:, M:], out=wzh_t[:E])
            K.transpose(w["hcat"][A + E:], out=wzh_t[E:])
            watt_t = K.transpose(w["hcat"][:A + E])                    # [D, A + E] = [W_da; W_fb]^T
            # the loss rows' mask and targets only depend on the captions: built here, beside the
            # recurrence, instead of between it and the vocab projection
            tmask = torch.arange(T, device=dev).view(1, T) < dl.view(B, 1)
            if loss:
                targets = torch.where(tmask, caps_s[:, 1:T + 1],
                                      torch.full_like(caps_s[:, 1:T + 1], -1)).reshape(-1)
        main.wait_event(ev_att1)
        self._launch("imgcap_lstm_tf_fwd", d)
        K.join(main, side)
        for t_ in (wzh_t, watt_t, tmask) + ((targets,) if loss else ()):
            t_.record_stream(main)
        # ---- fc(dropout(h)) over all B*T rows (decoder.py:109) ----------------------------------
        hd = hs.view(B * T, D)
        if p_drop > 0:
            hd = K.dropout(hd, p_drop, s["seed"], _STREAM_DROPOUT_H)
        s.update(enc_s=enc_s, ids=ids, emb=emb, mean=mean, att1=att1, xe=xe, c0=c0, g1=g1, alphas=alphas, awe=awe,
                 zs=zs, gates=gates, cs=cs, hs=hs, hprev=hprev, hd=hd, tmask=tmask, desc=d, wzh_t=wzh_t,
                 watt_t=watt_t)
        if loss:
            logits = torch.empty(B * T, self.Vpad, **ctd)
            K.gemm(hd, w["wfc"], trans_b=True, bias=w["bfc"], out=logits, N=V)
            lse = torch.empty(B * T, **f32)
            lrow = torch.empty(B * T, **f32)
            hit = torch.empty(B * T, **f32)
            metrics = torch.empty(5, **f32)  # loss, tokens, top5 hits, 1/tokens, hand-off errors
            # loss, top-5 and the loss gradient in one pass over the logits (train.py:266-276);
            # backward() starts from these dlogits
            dlogits = torch.empty(B * T, self.Vpad, **ctd)
            dalpha = torch.empty(B, T, P, **f32)
            reg = torch.empty(1 + B, **f32)  # the value, then the per-row partials (no library scratch)

            # the attention regulariser (train.py:268: its value and d alpha, which the backward
            # recurrence reads) on the side stream, beside the vocab projection and the CE
            K.fork(side, main)
            with torch.cuda.stream(side):
                _abi.call("imgcap_attn_reg", B, T, P, alphas.data_ptr(), dl.data_ptr(), alphaC, dalpha.data_ptr(),
                          reg.data_ptr(), reg[1:].data_ptr(), K.stream())
                ev_reg = torch.cuda.Event()
                ev_reg.record(side)

            def finalize():
                K.join(main, side, ev_reg)
                K.loss_finalize(lrow, hit, targets, reg, metrics)
            K.ce_train(logits, targets, V, metrics, lse, lrow, hit, dlogits, finalize)
            self._fold_status(metrics[4:5], init=True)  # the forward recurrence's error word
            s.update(logits=logits, targets=targets, lse=lse, dalpha=dalpha, metrics=metrics, dlogits=dlogits)
        return s

    def greedy(self, encoder_out, start_id, end_id, maxlen):
        """decoder.py:119-163 (forwardWithoutTeacherForcing) on device: per step one embedding
        lookup + the W_ih embedding half, the recurrence kernels of one step (imgcap_lstm_tf_fwd
        with T = 1: attention, gate, LSTMCell), fc and imgcap_greedy_select.  Every row is
        computed every step and finished rows' outputs stay zero (the reference compacts to the
        active rows; same results, no host sync per step).  Returns (predictions [B, maxlen, V]
        f32, alphas [B, maxlen, P] f32, sequences [B, maxlen] int64)."""
        st = self.decode_init(encoder_out)
        B, P, V, dev = st["B"], st["P"], self.V, encoder_out.device
        f32 = dict(device=dev, dtype=torch.float32)
        preds = torch.zeros(B, maxlen, V, **f32)
        alphas = torch.zeros(B, maxlen, P, **f32)
        seqs = torch.zeros(B, maxlen, device=dev, dtype=torch.int64)
        finished = torch.zeros(B, device=dev, dtype=torch.uint8)
        ids = torch.full((B,), start_id, device=dev, dtype=torch.int64)
        for t in range(maxlen):
            logits, alpha = self.decode_step(st, ids)
            K.greedy_select(logits, V, t, end_id, finished, ids, seqs, preds, alpha=alpha, alphas=alphas)  # :150-161
        self.step_id += 1
        return preds, alphas, seqs

    # -- step-wise decoding primitives (greedy above, beam search in beam.py) ---------------
    def decode_init(self, encoder_out):
        """decoder.py:121-127 / caption.py:76-86: per-row decoding state -- the encoder rows, the
        hoisted encoder_att projection and init_hidden_state's (h, c)."""
        ct, dev = self.ct, encoder_out.device
        E, D = self.E, self.D
        w = self.weights()
        B = encoder_out.size(0)
        enc = encoder_out.reshape(B, -1, E).to(ct).contiguous()
        P = enc.size(1)
        mean = torch.empty(B, E, device=dev, dtype=ct)
        K.mean_mid(enc, mean)                                                       # decoder.py:64
        h0c0 = K.gemm(mean, w["init"], trans_b=True, bias=w["binit"], out_dtype=torch.float32)  # :100-101
        att1 = K.gemm(enc.view(B * P, E), w["wea"], trans_b=True, bias=w["bea"])    # :61, once
        h = h0c0[:, :D].to(ct).reshape(B, 1, D).contiguous()
        c = h0c0[:, D:].contiguous()
        return dict(B=B, P=P, enc=enc, att1=att1.view(B, P, self.A), h=h, c=c, w=w)

    def decode_select(self, st, idx):
        """Keep / reorder decoding rows (beam search: caption.py:140-142)."""
        for k in ("enc", "att1", "h", "c"):
            st[k] = st[k].index_select(0, idx).contiguous()
        st["B"] = idx.numel()

    def decode_step(self, st, ids):
        """One decoding step for every row of ``st`` with input words ``ids`` [B]: embedding and the
        W_ih embedding half, imgcap_lstm_tf_fwd with T = 1 (attention, gate, LSTMCell), fc.
        Updates st's (h, c); returns (logits [B, Vpad] compute dtype, alpha [B, P] fp32)."""
        ct, dev = self.ct, ids.device
        A, E, D, M, V, W3 = self.A, self.E, self.D, self.M, self.V, self.W3
        B, P, w = st["B"], st["P"], st["w"]
        f32 = dict(device=dev, dtype=torch.float32)
        ctd = dict(device=dev, dtype=ct)
        emb = torch.empty(B, M, **ctd)
        K.embedding_fwd(ids, w["emb"], emb)                                         # :130 / :158
        xe = K.gemm(emb, w["wih"][:, :M], trans_b=True, bias=w["bih"], out_dtype=torch.float32)
        bufs = dict(g1=torch.empty(B, 1, W3, **f32), alphas=torch.empty(B, 1, P, **f32),
                    awe=torch.empty(B, 1, E, **f32), zs=torch.empty(B, 1, E, **ctd),
                    gates=torch.empty(B, 1, 4 * D, **f32), cs=torch.empty(B, 1, D, **f32),
                    hs=torch.empty(B, 1, D, **ctd), dl=torch.ones(B, device=dev, dtype=torch.int32))
        d = _abi.LstmDesc()
        d.dtype, d.B, d.P, d.E, d.A, d.D, d.M, d.T = K.dt(emb), B, P, E, A, D, M, 1
        for k, v in dict(w_hcat=w["hcat"], b_hcat=w["bhcat"], w_ih=w["wih"], w_f=w["wf"], enc=st["enc"],
                         att1=st["att1"], xe=xe, c0=st["c"], hprev=st["h"], **bufs).items():
            setattr(d, k, v.data_ptr())
        self._launch("imgcap_lstm_tf_fwd", d)                                       # :141-148, one step
        hd = bufs["hs"].view(B, D)
        if self.dec.training and self.dec.dropout_p > 0:
            hd = K.dropout(hd, self.dec.dropout_p, self.seed + self.step_id, _STREAM_DROPOUT_H)
        logits = torch.empty(B, self.Vpad, **ctd)
        K.gemm(hd, w["wfc"], trans_b=True, bias=w["bfc"], out=logits, N=V)         # :149
        st["h"], st["c"] = bufs["hs"], bufs["cs"].view(B, D)
        return logits, bufs["alphas"].view(B, P)

    def predictions(self, s):
        """decoder.py:94,110: zero-filled predictions [B, T, V] (fp32) from the saved state."""
        B, T, V = s["B"], s["T"], self.V
        w = self.weights()
        out = torch.empty(B * T, V, device=s["hs"].device, dtype=torch.float32)
        K.gemm(s["hd"], w["wfc"], trans_b=True, bias=w["bfc"], out=out,
               rowscale=s["tmask"].reshape(-1).float().contiguous(), rows_per_scale=1)
        return out.view(B, T, V)

    # ---------------------------------------------------------------------------------------
    def early_bucket(self):
        """Flat range whose gradients are final when backward() calls ``bucket_hook``: the
        embedding and fc weights (64 % of the decoder at C2), reduced while the weight-gradient
        GEMMs of the rest still run (DDP-style bucketed all-reduce)."""
        return self.fp.span(["embedding.weight", "fc.weight", "fc.bias"])

    def grad_buckets(self):
        """Flat ranges in the order backward() calls ``bucket_hook``: the early bucket."""
        return [self.early_bucket()]

    def backward(self, s, dlogits=None, dalpha=None, gbuf=None, want_denc=False, bucket_hook=None):
        """Writes dL/dparams into ``gbuf`` (default: the flat grad buffer).  Default upstream:
        the fused loss of forward(loss=True); otherwise ``dlogits`` [B*T, V(pad)] (compute
        dtype) and ``dalpha`` [B, T, P] (f32).  want_denc: also dL/d encoder_out (fp32, the
        caller's batch order) into s["denc"] -- encoder fine-tuning.  ``bucket_hook`` is called
        (on the current stream's timeline) once the early_bucket() gradients are final."""
        fp, ct = self.fp, self.ct
        gbuf = fp.grad if gbuf is None else gbuf

        class _G:  # views into gbuf
            @staticmethod
            def g(name, shape=None, count=None):
                return fp.g(name, shape, count, buf=gbuf)
        B, P, T = s["B"], s["P"], s["T"]
        A, E, D, M, V, W3 = self.A, self.E, self.D, self.M, self.V, self.W3
        dev = s["hs"].device
        w = self.weights()
        cb = K.ColsumBatch()  # every bias gradient, reduced in one launch at the end
        wgb = K.GemmBatch()    # every weight gradient, grouped launches at the end
        if dlogits is None:
            dlogits = s["dlogits"]  # imgcap_ce_fused in forward(loss=True)
            dalpha = s["dalpha"]
        BT = B * T
        # fc: dh = (dlogits W_fc) * dropmask on the critical path; dW_fc = dlogits^T hd and
        # db_fc = colsum(dlogits) on a side stream beside the backward recurrence
        dhs = K.gemm(dlogits, w["wfc"], K=V, drop_p=s["p_drop"], seed=s["seed"], drop_stream=_STREAM_DROPOUT_H,
                     drop_ld=D)
        main = torch.cuda.current_stream(dev)
        side = self._side_stream(dev)
        K.fork(side, main)
        with torch.cuda.stream(side):  # no library scratch on this stream (no split-K, one-pass colsum)
            # the gradient buffer is cleared here, beside the recurrence (60 MB at C2, not on the
            # critical path); the main stream joins this stream before its first gradient write
            gbuf.zero_()
            K.gemm(dlogits, s["hd"], trans_a=True, M=V, out=_G.g("fc.weight"), out_dtype=torch.float32)
            cbs = K.ColsumBatch()
            cbs.add(dlogits, _G.g("fc.bias"), cols=V)
            cbs.run()
            ev_fc = torch.cuda.Event()  # gbuf cleared, fc dW / db written
            ev_fc.record(side)
        par_tail = bucket_hook is None and not want_denc and ct == torch.bfloat16
        f32 = dict(device=dev, dtype=torch.float32)
        dcat = torch.empty(B, T, W3, device=dev, dtype=ct)
        xs, ys = self.X_SLICES, self.Y_SLICES
        # per chain: K-slice slabs of the step GEMMs and the last-arriver counters (left at 0)
        chain_ws = []
        rows = self._chain_rows(B)
        if self._y_cnt is None or len(self._y_cnt) != len(rows) or self._y_cnt[0].device != dev:
            self._retired_sync += [c for c in (self._y_cnt or []) if c is not None]
            self._y_cnt = [None] * len(rows)
        for i, (b0, b1) in enumerate(rows):
            nrg = (b1 - b0 + 31) // 32
            if self._y_cnt[i] is None or self._y_cnt[i].numel() < nrg * (D // 16):
                if self._y_cnt[i] is not None:  # captured graphs may point at the old counters
                    self._retired_sync.append(self._y_cnt[i])
                self._y_cnt[i] = torch.zeros(nrg * (D // 16), device=dev, dtype=torch.int32)
            chain_ws.append(dict(dz=torch.empty(xs, b1 - b0, E + D, **f32),
                                 ws_y=torch.empty(ys * nrg * (D // 16) * 512, **f32), y_cnt=self._y_cnt[i]))
        dh, dc = torch.empty(B, D, **f32), torch.empty(B, D, **f32)
        de = torch.empty(B, T, P, **f32)
        datt1 = torch.empty(B * P, A, device=dev, dtype=ct)
        npc = (P + 6) // 7  # pixel chunks of attn_param_grad_kernel
        dwf, dbea = torch.empty(B * npc, A, **f32), torch.empty(B * npc, A, **f32)
        wzh_t, watt_t = s["wzh_t"], s["watt_t"]  # made under the forward recurrence
        d = s["desc"]
        bufs = dict(w_zh_t=wzh_t, w_att_t=watt_t, dhs=dhs, dalpha=dalpha, dcat=dcat, dh=dh, dc=dc, de=de,
                    datt1=datt1, dwf=dwf, dbea=dbea)
        for k, v in bufs.items():
            setattr(d, k, K.ptr(v))
        d.x_slices, d.y_slices = xs, ys
        dawe = torch.empty(B, T + 1, E, **f32) if want_denc else None
        d.dawe = K.ptr(dawe)
        bufs["dawe"] = dawe
        bufs["chain_ws"] = chain_ws
        s["bwd_bufs"] = bufs  # the descriptor points into these: keep them alive as long as `s`
        self._launch("imgcap_lstm_tf_bwd", d, chain_ws)
        dc2 = dcat.view(BT, W3)
        dgates = dc2[:, A + E:]
        # one rank, bf16, no encoder gradient: the embedding gradient (d_emb = dgates W_ih[:, :M],
        # then the rank / scatter / segmented row sums) runs on the side stream beside the grouped
        # weight-gradient GEMMs and the bias column sums (it is the only library-scratch user of
        # the two branches: the grouped GEMMs and colsum_multi take none).  With DDP the early
        # bucket's all-reduce takes that window instead (the hook after the embedding gradient).
        if par_tail:
            K.fork(side, main)
            with torch.cuda.stream(side), K.workspace_slot(2):  # its own scratch slot (library check)
                if "metrics" in s:
                    self._fold_status(s["metrics"][4:5])  # the backward recurrence's error word
                demb = K.gemm(dgates, w["wih"][:, :M], K=4 * D)
                K.embedding_bwd(s["ids"], demb, _G.g("embedding.weight"))
            main.wait_event(ev_fc)
        elif "metrics" in s:
            self._fold_status(s["metrics"][4:5])
        # W_hcat / b_hcat grads (batched over all B*T rows)
        wgb.add(dc2, s["hprev"].view(BT, D), out=_G.g("attention.decoder_att.weight", (W3, D), W3 * D), trans_a=True)
        cb.add(dc2, _G.g("attention.decoder_att.bias", (W3,), W3))
        # LSTMCell weight_ih (emb half | attention half), bias_ih
        gwih = _G.g("decode_step.weight_ih")
        wgb.add(dgates, s["emb"], out=gwih[:, :M], M=4 * D, trans_a=True)
        wgb.add(dgates, s["zs"].view(BT, E), out=gwih[:, M:], M=4 * D, trans_a=True)
        cb.add(dgates, _G.g("decode_step.bias_ih"))
        if not par_tail:
            # embedding: d_emb = dgates W_ih[:, :M]  -> scatter-add rows
            demb = K.gemm(dgates, w["wih"][:, :M], K=4 * D)
            K.join(main, side)  # gbuf cleared, fc dW / db (beside the recurrence) done
            K.embedding_bwd(s["ids"], demb, _G.g("embedding.weight"))
        # init_h / init_c from dh0, dc0
        dinit = torch.cat([dh, dc], dim=1).to(ct)
        wgb.add(dinit, s["mean"], out=_G.g("init_h.weight", (2 * D, E), 2 * D * E), trans_a=True)
        cb.add(dinit, _G.g("init_h.bias", (2 * D,), 2 * D))
        # encoder_att from the time-summed d att1
        wgb.add(datt1, s["enc_s"].view(B * P, E), out=_G.g("attention.encoder_att.weight"), trans_a=True)
        cb.add(dbea, _G.g("attention.encoder_att.bias"))
        cb.add(dwf, _G.g("attention.full_att.weight", (A,)))
        # full_att.bias: exactly zero gradient (softmax is shift-invariant) -> left at 0
        if bucket_hook is not None:
            bucket_hook()
        wgb.run()
        cb.run()
        if par_tail:
            K.join(main, side)  # the embedding gradient and the metrics' error word
        s["denc"] = None
        if want_denc:
            # decoder.py:26 (att1 = enc W_ea), :64-66 (mean -> init_h/c), :102-103 (context)
            K.gemm(dinit, w["init"], out=dawe[:, T, :])                      # dL/d mean(enc)
            base = K.gemm(datt1, w["wea"], out_dtype=torch.float32)         # [B*P, E]
            denc = torch.empty(B, P, E, **f32)
            _abi.call("imgcap_lstm_denc", B, T, P, E, s["alphas"].data_ptr(), dawe.data_ptr(), base.data_ptr(),
                      s["sort_ind"].data_ptr(), denc.data_ptr(), K.stream())
            s["denc"] = denc
        return gbuf

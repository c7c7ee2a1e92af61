"""Explicit forward/backward engine of the teacher-forced Transformer decoder on HIP.

Mirrors TransformerDecoder.forwardWithTeacherForcing (models/transformerDecoder.py:88-108)
with torch.nn.TransformerDecoderLayer's post-norm math (norm_first=False, ReLU FFN,
dropout after the embedding, on the attention probabilities, on each sublayer output and
inside the FFN), plus the packed CE of train.py:271-276.

Kernels per layer (forward): in-proj GEMM -> MHA (causal + key padding) -> out-proj GEMM ->
add+dropout+LN -> q GEMM / kv GEMM on the memory -> MHA -> out-proj -> add+LN -> FFN GEMM
(+bias, ReLU, dropout in the epilogue) -> GEMM -> add+LN.  Rows are batch-major [B*L, d]
(the reference is seq-first; the permutes at transformerDecoder.py:95,99,105 are free here).
"""
import ctypes
import math
import os

import torch

from . import _abi
from . import kernels as K
from .flat import FlatParams

# weight gradients: long-K fp32 products into the gradient buffer, K sliced over the
# grid (imgcap_epilogue.split_k)
DW = dict(split_k=-1)

# backward tail: bias-gradient column sums on a side stream beside the grouped weight-gradient
# GEMMs (IMGCAP_TF_TAIL_FORK=0: one stream)
TAIL_FORK = os.environ.get("IMGCAP_TF_TAIL_FORK", "1") != "0"

# dropout stream ids (each site gets its own counter-based mask stream)
_S_EMB = 1


def _s(layer, site):
    return 100 + 16 * layer + site


def transformer_param_groups(dec):
    n = dict(dec.named_parameters())
    groups = []
    for k in n:
        groups.append([k])
    return [[(k, n[k]) for k in g] for g in groups]


class TransformerEngine:
    def __init__(self, dec, device, compute_dtype=torch.bfloat16):
        self.dec = dec
        self.ct = compute_dtype
        self.fp = FlatParams(transformer_param_groups(dec), device, compute_dtype)
        self.d = dec.embed_dim
        self.H = dec.num_heads
        self.ff = dec.decoder_dim
        self.V = dec.vocab_size
        self.E = dec.encoder_dim
        self.layers = dec.num_layers
        self.Vpad = (self.V + 7) // 8 * 8
        self.has_proj = "encoder_proj.weight" in self.fp.params
        self.layer_prefix = getattr(dec, "layer_prefix", "transformer_decoder.layers")
        # per-layer cross-attention probabilities [B, H, Lq, P] of the last forward / decode
        # step (set to a list to record them: the attention-visualisation decoder's alphas)
        self.cross_probs = None
        if self.d // self.H != 64:
            raise NotImplementedError("the HIP attention kernel needs head dim 64 (embed_dim = 64 * num_heads)")
        self.seed = 4321
        self.step_id = 0
        # one gradient bucket for all layers instead of one per layer (set by the trainer for the
        # pipelined DDP schedule: the captured step is split at each bucket hook and the encoder
        # branch of the next batch joins at the first split, so the hook must come late)
        self.merged_layer_bucket = False

    def _lw(self, i, name):
        # nn.TransformerDecoder layers (transformerDecoder.py) or the attention-visualisation
        # decoder's ModuleList (transformerDecoderAttVis.py:123: decoder_layers.{i}.*)
        return f"{self.layer_prefix}.{i}.{name}"

    def _mha(self, *, B, Lq, Lk, q, ldq, k, ldk, v, ldv, o, ldo, lse, causal, key_ids, pad_id, p, seed, sid,
             dout=None, lddo=0, dq=None, lddq=0, dk=None, lddk=0, dv=None, lddv=0, bwd=False, kv_rows=0,
             probs=None):
        m = _abi.MhaDesc()
        m.dtype, m.B, m.H, m.Lq, m.Lk, m.dh, m.causal = K.dt(q), B, self.H, Lq, Lk, 64, int(causal)
        m.pad_id = pad_id
        m.ldq, m.ldk, m.ldv, m.ldo = ldq, ldk, ldv, ldo
        m.q, m.k, m.v, m.o, m.lse = q.data_ptr(), k.data_ptr(), v.data_ptr(), K.ptr(o), lse.data_ptr()
        m.key_ids = K.ptr(key_ids)
        m.scale = 1.0 / math.sqrt(64.0)
        m.kv_rows = kv_rows
        m.probs = K.ptr(probs)
        m.drop_p, m.seed, m.drop_stream = p, seed, sid
        if bwd:
            m.dout, m.lddo = dout.data_ptr(), lddo
            m.dq, m.dk, m.dv = dq.data_ptr(), dk.data_ptr(), dv.data_ptr()
            m.lddq, m.lddk, m.lddv = lddq, lddk, lddv
            _abi.call("imgcap_mha_bwd", ctypes.byref(m), K.stream())
        else:
            _abi.call("imgcap_mha_fwd", ctypes.byref(m), K.stream())

    # ---------------------------------------------------------------------------------------
    def forward(self, encoder_out, encoded_captions, caption_lengths, *, key_ids=None, pad_id=0, dropout=None,
                loss=True):
        fp, ct, dev = self.fp, self.ct, encoder_out.device
        d, ff, V = self.d, self.ff, self.V
        p = self.dec.dropout_p if (dropout is None and self.dec.training) else (dropout or 0.0)
        B = encoder_out.size(0)
        enc = encoder_out.reshape(B, -1, self.E).to(ct).contiguous()
        P = enc.size(1)
        L = encoded_captions.size(1)
        caps = encoded_captions.contiguous()
        if key_ids is None:
            key_ids = caps
        seed = self.seed + 7919 * self.step_id
        self.step_id += 1
        s = dict(B=B, P=P, L=L, p=p, seed=seed, enc=enc, caps=caps, key_ids=key_ids, pad_id=pad_id, layers=[])
        ctd = dict(device=dev, dtype=ct)
        f32 = dict(device=dev, dtype=torch.float32)
        BL, BP = B * L, B * P
        # memory = encoder_proj(encoder_out)                                  transformerDecoder.py:95
        if self.has_proj:
            mem = K.gemm(enc.view(BP, self.E), fp.w("encoder_proj.weight"), trans_b=True,
                         bias=fp.f32("encoder_proj.bias"))
        else:
            mem = enc.view(BP, d)
        # tgt = pos_encoding(dropout(embedding(caps)))                       :97-98
        x = torch.empty(BL, d, **ctd)
        K.embedding_fwd(caps.view(-1), fp.f32("embedding.weight"), x, pe=self.dec.pos_encoding.pe.view(-1, d)[:L]
                        .contiguous().float(), L=L, drop_p=p, seed=seed, drop_stream=_S_EMB)
        s["x0"] = x
        # the cross-attention K/V projections of all layers depend on the memory alone (:81-82,
        # nn.MultiheadAttention in_proj rows d..3d): one GEMM [B*P, 2d*layers] against the layers'
        # stacked W_kv / b_kv (copied from the bf16 weights: 2 copy launches for 6 GEMMs).  Layer i
        # reads its K/V as the column slice i of kv_all; the backward's dK/dV go to the matching
        # slices of one buffer and the memory gradient is one GEMM against the same stack.
        nkv = 2 * d * self.layers
        wkv = torch.cat([fp.w(self._lw(i, "multihead_attn.in_proj_weight"))[d:] for i in range(self.layers)])
        bkv = torch.cat([fp.f32(self._lw(i, "multihead_attn.in_proj_bias"))[d:] for i in range(self.layers)])
        kv_all = K.gemm(mem, wkv, trans_b=True, bias=bkv)
        s.update(wkv=wkv, kv_all=kv_all)
        for i in range(self.layers):
            lw = lambda n: self._lw(i, n)  # noqa: E731
            st = {"x": x}
            qkv = K.gemm(x, fp.w(lw("self_attn.in_proj_weight")), trans_b=True, bias=fp.f32(lw("self_attn.in_proj_bias")))
            o = torch.empty(BL, d, **ctd)
            lse1 = torch.empty(B, self.H, L, **f32)
            self._mha(B=B, Lq=L, Lk=L, q=qkv, ldq=3 * d, k=qkv[:, d:], ldk=3 * d, v=qkv[:, 2 * d:], ldv=3 * d, o=o,
                      ldo=d, lse=lse1, causal=True, key_ids=key_ids, pad_id=pad_id, p=p, seed=seed, sid=_s(i, 0))
            s1 = torch.empty(BL, d, **ctd)
            x1, mu1, rs1 = self._linear_add_ln(o, "self_attn.out_proj", x, "norm1", i, p, seed, _s(i, 1), s1)
            wq = fp.w(lw("multihead_attn.in_proj_weight"))
            bq = fp.f32(lw("multihead_attn.in_proj_bias"))
            q2 = K.gemm(x1, wq[:d], trans_b=True, bias=bq[:d])
            kv2 = kv_all[:, 2 * d * i:2 * d * (i + 1)]
            o2 = torch.empty(BL, d, **ctd)
            lse2 = torch.empty(B, self.H, L, **f32)
            pr = None
            if self.cross_probs is not None:
                pr = torch.empty(B, self.H, L, P, **f32)
                self.cross_probs.append(pr)
            self._mha(B=B, Lq=L, Lk=P, q=q2, ldq=d, k=kv2, ldk=nkv, v=kv2[:, d:], ldv=nkv, o=o2, ldo=d, lse=lse2,
                      causal=False, key_ids=None, pad_id=0, p=p, seed=seed, sid=_s(i, 2), probs=pr)
            s2 = torch.empty(BL, d, **ctd)
            x2, mu2, rs2 = self._linear_add_ln(o2, "multihead_attn.out_proj", x1, "norm2", i, p, seed, _s(i, 3), s2)
            hdn = K.gemm(x2, fp.w(lw("linear1.weight")), trans_b=True, bias=fp.f32(lw("linear1.bias")),
                         act=K.ACT_RELU, drop_p=p, seed=seed, drop_stream=_s(i, 4))
            s3 = torch.empty(BL, d, **ctd)
            x3, mu3, rs3 = self._linear_add_ln(hdn, "linear2", x2, "norm3", i, p, seed, _s(i, 5), s3)
            st.update(qkv=qkv, o=o, lse1=lse1, s1=s1, mu1=mu1, rs1=rs1, x1=x1, q2=q2, kv2=kv2, o2=o2, lse2=lse2,
                      s2=s2, mu2=mu2, rs2=rs2, x2=x2, hdn=hdn, s3=s3, mu3=mu3, rs3=rs3)
            s["layers"].append(st)
            x = x3
        s["mem"] = mem
        s["xL"] = x
        # the decode mask, position l's target caps[:, l+1] (-1 past the decode length) and the zeroed
        # metrics (loss, tokens, top5 hits, 1/tokens, hand-off errors: none here) in one launch
        lens = caption_lengths.reshape(-1)
        if lens.dtype != torch.int64:
            lens = lens.to(torch.int64)
        tmask, targets, metrics = K.tf_targets(caps if caps.dtype == torch.int64 else caps.to(torch.int64), lens)
        s["tmask"] = tmask
        if loss:
            logits = torch.empty(BL, self.Vpad, **ctd)
            K.gemm(x, fp.w("fc_out.weight"), trans_b=True, bias=fp.f32("fc_out.bias"), out=logits, N=V)
            lse = torch.empty(BL, **f32)
            lrow = torch.empty(BL, **f32)
            hit = torch.empty(BL, **f32)
            # loss, top-5 and the loss gradient in one pass over the logits (train.py:266-276)
            dlogits = torch.empty(BL, self.Vpad, **ctd)
            K.ce_train(logits, targets, V, metrics, lse, lrow, hit, dlogits,
                       lambda: K.loss_finalize(lrow, hit, targets, None, metrics))
            s.update(logits=logits, targets=targets, lse=lse, metrics=metrics, dlogits=dlogits)
        return s

    def _linear_add_ln(self, a, linear, x, norm, i, p, seed, sid, s_out):
        """x' = LN(x + dropout(a W^T + b)) (transformerDecoder.py:82,104, post-norm): the GEMM, then
        imgcap_add_layernorm_fwd.  (Round 5 measured a row-complete GEMM + LayerNorm kernel, 32 x
        512 tiles each streaming the whole weight: 21 us against 13.8 for the pair -- DESIGN §3d.)"""
        fp = self.fp
        w, b = fp.w(self._lw(i, f"{linear}.weight")), fp.f32(self._lw(i, f"{linear}.bias"))
        g, be = fp.f32(self._lw(i, f"{norm}.weight")), fp.f32(self._lw(i, f"{norm}.bias"))
        y = K.gemm(a, w, trans_b=True, bias=b)
        return K.add_layernorm(x, y, g, be, 1e-5, drop_p=p, seed=seed, drop_stream=sid, s_out=s_out)

    def _ln_bwd_of_product(self, a, b, res, st, k, i, p, seed, sid, G, cb):
        """The LayerNorm backward of norm{k} (layer i) on its incoming gradient a @ b + res: the
        GEMM (beta = 1 into res), then imgcap_add_layernorm_bwd; returns (dS, dY)."""
        fp = self.fp
        gam = fp.f32(self._lw(i, f"norm{k}.weight"))
        gg, gb = G(self._lw(i, f"norm{k}.weight")), G(self._lw(i, f"norm{k}.bias"))
        dy = torch.empty_like(res)
        K.gemm(a, b, out=res, beta=1.0)
        ds = K.add_layernorm_bwd(res, st[f"s{k}"], st[f"mu{k}"], st[f"rs{k}"], gam, gg, gb, drop_p=p, seed=seed,
                                 drop_stream=sid, dr=dy, cb=cb)
        return ds, dy

    def greedy(self, encoder_out, start_id, end_id, maxlen):
        """transformerDecoder.py:110-160 (forwardWithoutTeacherForcing) with a key/value cache.

        The reference re-decodes the whole prefix every step (O(T^2) per caption).  In a post-norm
        decoder with a causal mask the layer outputs at positions < t do not change when token t
        is appended, so each step here runs the 6 layers on the new position only: its self-
        attention reads the cached K/V of positions 0..t (mha kv_rows = maxlen), the cross-
        attention K/V of the memory are computed once.  Same results as the reference up to fp
        reassociation.  Returns (predictions [B, maxlen, V] f32, sequences [B, maxlen] int64)."""
        st = self.decode_init(encoder_out, maxlen)
        B, V, dev = st["B"], self.V, encoder_out.device
        preds = torch.zeros(B, maxlen, V, device=dev, dtype=torch.float32)
        seqs = torch.zeros(B, maxlen, device=dev, dtype=torch.int64)
        finished = torch.zeros(B, device=dev, dtype=torch.uint8)
        ids = torch.full((B,), start_id, device=dev, dtype=torch.int64)
        for t in range(maxlen):
            logits = self.decode_step(st, ids)
            K.greedy_select(logits, V, t, end_id, finished, ids, seqs, preds)     # :141-155
        return preds, seqs

    # -- step-wise decoding primitives (greedy above, beam search in beam.py) ---------------
    def decode_init(self, encoder_out, maxlen):
        """Decoding state: the per-layer cross-attention K/V of the projected memory (computed
        once, :112-114) and an empty per-layer cache of (q | k | v) rows for ``maxlen`` positions."""
        fp, ct, dev = self.fp, self.ct, encoder_out.device
        d = self.d
        if maxlen > 64:
            raise ValueError("step-wise decode: at most 64 positions (attention kernel tile)")
        B = encoder_out.size(0)
        enc = encoder_out.reshape(B, -1, self.E).to(ct).contiguous()
        P = enc.size(1)
        if self.has_proj:
            mem = K.gemm(enc.view(B * P, self.E), fp.w("encoder_proj.weight"), trans_b=True,
                         bias=fp.f32("encoder_proj.bias"))
        else:
            mem = enc.view(B * P, d)
        kv_mem, cache = [], []
        for i in range(self.layers):
            wq = fp.w(self._lw(i, "multihead_attn.in_proj_weight"))
            bq = fp.f32(self._lw(i, "multihead_attn.in_proj_bias"))
            kv_mem.append(K.gemm(mem, wq[d:], trans_b=True, bias=bq[d:]).view(B, P, 2 * d))
            cache.append(torch.empty(B, maxlen, 3 * d, device=dev, dtype=ct))
        seed = self.seed + 7919 * self.step_id
        self.step_id += 1
        return dict(B=B, P=P, t=0, maxlen=maxlen, kv_mem=kv_mem, cache=cache, seed=seed)

    def decode_select(self, st, idx):
        """Keep / reorder decoding rows with their caches (beam search: caption.py:229-248)."""
        st["kv_mem"] = [m.index_select(0, idx).contiguous() for m in st["kv_mem"]]
        st["cache"] = [c.index_select(0, idx).contiguous() for c in st["cache"]]
        st["B"] = idx.numel()

    def decode_step(self, st, ids):
        """Position st["t"] for every row: embedding(ids) + pe[t], the layers on that position
        only (self-attention over the cached K/V of positions 0..t), fc_out.  Returns logits
        [B, Vpad] (compute dtype) and advances t."""
        fp, ct, dev = self.fp, self.ct, ids.device
        d, V, B, P, t, maxlen = self.d, self.V, st["B"], st["P"], st["t"], st["maxlen"]
        if t >= maxlen:
            raise ValueError("decode_step: cache full")
        p = self.dec.dropout_p if self.dec.training else 0.0
        seed = st["seed"] + t
        ctd = dict(device=dev, dtype=ct)
        pe = self.dec.pos_encoding.pe.view(-1, d)[t:t + 1].float().contiguous()
        x = torch.empty(B, d, **ctd)
        o = torch.empty(B, d, **ctd)
        lse = torch.empty(B, self.H, 1, device=dev, dtype=torch.float32)
        # the new position's input: embedding(last token) + pe[t]                  :129-130
        K.embedding_fwd(ids, fp.f32("embedding.weight"), x, pe=pe, L=1, drop_p=p, seed=seed, drop_stream=_S_EMB)
        for i in range(self.layers):
            lw = lambda n: self._lw(i, n)  # noqa: E731
            c = st["cache"][i]
            K.gemm(x, fp.w(lw("self_attn.in_proj_weight")), trans_b=True, bias=fp.f32(lw("self_attn.in_proj_bias")),
                   out=c[:, t])                                                 # q, k, v of position t
            # Lq = 1: the query "row stride" ldq is the cache's batch stride
            self._mha(B=B, Lq=1, Lk=t + 1, q=c[:, t], ldq=maxlen * 3 * d, k=c[:, :, d:], ldk=3 * d, v=c[:, :, 2 * d:],
                      ldv=3 * d, o=o, ldo=d, lse=lse, causal=False, key_ids=None, pad_id=0, p=p, seed=seed,
                      sid=_s(i, 0), kv_rows=maxlen)
            y = K.gemm(o, fp.w(lw("self_attn.out_proj.weight")), trans_b=True, bias=fp.f32(lw("self_attn.out_proj.bias")))
            x1, _, _ = K.add_layernorm(x, y, fp.f32(lw("norm1.weight")), fp.f32(lw("norm1.bias")), 1e-5,
                                       drop_p=p, seed=seed, drop_stream=_s(i, 1))
            wq = fp.w(lw("multihead_attn.in_proj_weight"))
            bq = fp.f32(lw("multihead_attn.in_proj_bias"))
            q2 = K.gemm(x1, wq[:d], trans_b=True, bias=bq[:d])
            kv2 = st["kv_mem"][i].view(B * P, 2 * d)
            pr = None
            if self.cross_probs is not None:
                pr = torch.empty(B, self.H, 1, P, device=dev, dtype=torch.float32)
                self.cross_probs.append(pr)
            self._mha(B=B, Lq=1, Lk=P, q=q2, ldq=d, k=kv2, ldk=2 * d, v=kv2[:, d:], ldv=2 * d, o=o, ldo=d,
                      lse=lse, causal=False, key_ids=None, pad_id=0, p=p, seed=seed, sid=_s(i, 2), probs=pr)
            y2 = K.gemm(o, fp.w(lw("multihead_attn.out_proj.weight")), trans_b=True,
                        bias=fp.f32(lw("multihead_attn.out_proj.bias")))
            x2, _, _ = K.add_layernorm(x1, y2, fp.f32(lw("norm2.weight")), fp.f32(lw("norm2.bias")), 1e-5,
                                       drop_p=p, seed=seed, drop_stream=_s(i, 3))
            hdn = K.gemm(x2, fp.w(lw("linear1.weight")), trans_b=True, bias=fp.f32(lw("linear1.bias")),
                         act=K.ACT_RELU, drop_p=p, seed=seed, drop_stream=_s(i, 4))
            y3 = K.gemm(hdn, fp.w(lw("linear2.weight")), trans_b=True, bias=fp.f32(lw("linear2.bias")))
            x, _, _ = K.add_layernorm(x2, y3, fp.f32(lw("norm3.weight")), fp.f32(lw("norm3.bias")), 1e-5,
                                      drop_p=p, seed=seed, drop_stream=_s(i, 5))
        logits = torch.empty(B, self.Vpad, **ctd)
        K.gemm(x, fp.w("fc_out.weight"), trans_b=True, bias=fp.f32("fc_out.bias"), out=logits, N=V)  # :140
        st["t"] = t + 1
        return logits

    def predictions(self, s):
        """transformerDecoder.py:106: fc_out over all L positions -> [B, L, V] fp32."""
        B, L = s["B"], s["L"]
        out = K.gemm(s["xL"], self.fp.w("fc_out.weight"), trans_b=True, bias=self.fp.f32("fc_out.bias"),
                     out_dtype=torch.float32)
        return out.view(B, L, self.V)

    # ---------------------------------------------------------------------------------------
    def early_bucket(self):
        """Flat range of the token embedding (final once its backward scatter ran)."""
        return self.fp.span(["embedding.weight"])

    def grad_buckets(self):
        """Flat ranges in the order backward() calls ``bucket_hook``: one per decoder layer, the
        last layer first (trainMultiGPU.py:233-235: DDP all-reduces gradient buckets as the
        backward produces them), or one for all layers with ``merged_layer_bucket``.  The rest
        (fc_out, embedding, encoder_proj) is final when backward() returns."""
        if self.merged_layer_bucket:
            pre = f"{self.layer_prefix}."
            return [self.fp.span([n for n in self.fp.params if n.startswith(pre)])]
        out = []
        for i in reversed(range(self.layers)):
            pre = f"{self.layer_prefix}.{i}."
            out.append(self.fp.span([n for n in self.fp.params if n.startswith(pre)]))
        return out

    def backward(self, s, dlogits=None, gbuf=None, want_denc=False, bucket_hook=None):
        """Gradients of the step into ``gbuf`` (default fp.grad).  With ``bucket_hook`` (DDP) a
        layer's deferred weight / bias gradients run as their own grouped launches when its
        backward is done and the hook is called once per layer (grad_buckets() order), so its
        all-reduce overlaps the layers below; without it every layer's are deferred to one set of
        grouped launches at the end.  Each product / column sum is computed by the same kernel
        either way (per-problem tiles, fixed-order sums): the gradients are bitwise the same."""
        fp, ct = self.fp, self.ct
        gbuf = fp.grad if gbuf is None else gbuf
        G = lambda name, shape=None, count=None: fp.g(name, shape, count, buf=gbuf)  # noqa: E731
        B, L, P, p, seed = s["B"], s["L"], s["P"], s["p"], s["seed"]
        d, V = self.d, self.V
        BL, BP = B * L, B * P
        dev = s["xL"].device
        gbuf.zero_()
        cb = K.ColsumBatch()  # every bias gradient, reduced in one launch at the end
        wgb = K.GemmBatch()    # every weight gradient, grouped launches at the end
        if dlogits is None:
            dlogits = s["dlogits"]  # imgcap_ce_fused in forward(loss=True)
        wgb.add(dlogits, s["xL"], out=G("fc_out.weight"), M=V, trans_a=True)
        cb.add(dlogits, G("fc_out.bias"), cols=V)
        dx = K.gemm(dlogits, fp.w("fc_out.weight"), K=V)                    # [BL, d]
        nkv = 2 * d * self.layers
        dkv_all = torch.empty(BP, nkv, device=dev, dtype=ct)  # every layer's dK | dV (forward's kv_all layout)
        carry = None  # (dS3, dY3) of layer i, made at the end of layer i+1's iteration

        for i in reversed(range(self.layers)):
            lw = lambda n: self._lw(i, n)  # noqa: E731
            st = s["layers"][i]
            # x3 = LN3(x2 + drop(y3))
            if carry is None:
                dy3 = torch.empty_like(dx)
                ds3 = K.add_layernorm_bwd(dx, st["s3"], st["mu3"], st["rs3"], fp.f32(lw("norm3.weight")),
                                          G(lw("norm3.weight")), G(lw("norm3.bias")), drop_p=p, seed=seed,
                                          drop_stream=_s(i, 5), dr=dy3, cb=cb)
            else:
                ds3, dy3 = carry
            # y3 = hdn W2^T + b2 ; hdn = drop(relu(x2 W1^T + b1))
            wgb.add(dy3, st["hdn"], out=G(lw("linear2.weight")), trans_a=True)
            cb.add(dy3, G(lw("linear2.bias")))
            dpre = K.gemm(dy3, fp.w(lw("linear2.weight")), aux=st["hdn"], aux_scale=1.0 / (1.0 - p))
            wgb.add(dpre, st["x2"], out=G(lw("linear1.weight")), trans_a=True)
            cb.add(dpre, G(lw("linear1.bias")))
            # x2 = LN2(x1 + drop(y2)), on its incoming gradient dx2 = ds3 + dpre W1
            ds2, dy2 = self._ln_bwd_of_product(dpre, fp.w(lw("linear1.weight")), ds3, st, 2, i, p, seed, _s(i, 3), G, cb)
            wgb.add(dy2, st["o2"], out=G(lw("multihead_attn.out_proj.weight")), trans_a=True)
            cb.add(dy2, G(lw("multihead_attn.out_proj.bias")))
            do2 = K.gemm(dy2, fp.w(lw("multihead_attn.out_proj.weight")))
            dq2 = torch.empty(BL, d, device=dev, dtype=ct)
            dkv2 = dkv_all[:, 2 * d * i:2 * d * (i + 1)]
            self._mha(B=B, Lq=L, Lk=P, q=st["q2"], ldq=d, k=st["kv2"], ldk=nkv, v=st["kv2"][:, d:], ldv=nkv,
                      o=None, ldo=d, lse=st["lse2"], causal=False, key_ids=None, pad_id=0, p=p, seed=seed,
                      sid=_s(i, 2), dout=do2, lddo=d, dq=dq2, lddq=d, dk=dkv2, lddk=nkv, dv=dkv2[:, d:],
                      lddv=nkv, bwd=True)
            gw = G(lw("multihead_attn.in_proj_weight"))
            gb = G(lw("multihead_attn.in_proj_bias"))
            wq = fp.w(lw("multihead_attn.in_proj_weight"))
            wgb.add(dq2, st["x1"], out=gw[:d], trans_a=True)
            cb.add(dq2, gb[:d])
            wgb.add(dkv2, s["mem"], out=gw[d:], trans_a=True)
            cb.add(dkv2, gb[d:])
            # x1 = LN1(x + drop(y)), on its incoming gradient dx1 = ds2 + dq2 W_q
            ds1, dy = self._ln_bwd_of_product(dq2, wq[:d], ds2, st, 1, i, p, seed, _s(i, 1), G, cb)
            wgb.add(dy, st["o"], out=G(lw("self_attn.out_proj.weight")), trans_a=True)
            cb.add(dy, G(lw("self_attn.out_proj.bias")))
            do = K.gemm(dy, fp.w(lw("self_attn.out_proj.weight")))
            dqkv = torch.empty(BL, 3 * d, device=dev, dtype=ct)
            qkv = st["qkv"]
            self._mha(B=B, Lq=L, Lk=L, q=qkv, ldq=3 * d, k=qkv[:, d:], ldk=3 * d, v=qkv[:, 2 * d:], ldv=3 * d,
                      o=None, ldo=d, lse=st["lse1"], causal=True, key_ids=s["key_ids"], pad_id=s["pad_id"], p=p,
                      seed=seed, sid=_s(i, 0), dout=do, lddo=d, dq=dqkv, lddq=3 * d, dk=dqkv[:, d:], lddk=3 * d,
                      dv=dqkv[:, 2 * d:], lddv=3 * d, bwd=True)
            wgb.add(dqkv, st["x"], out=G(lw("self_attn.in_proj_weight")), trans_a=True)
            cb.add(dqkv, G(lw("self_attn.in_proj_bias")))
            if i > 0:
                # layer i-1's LN3 on its incoming gradient dx = ds1 + dqkv W_in
                carry = self._ln_bwd_of_product(dqkv, fp.w(lw("self_attn.in_proj_weight")), ds1, s["layers"][i - 1],
                                                3, i - 1, p, seed, _s(i - 1, 5), G, cb)
            else:
                K.gemm(dqkv, fp.w(lw("self_attn.in_proj_weight")), out=ds1, beta=1.0)  # dx = ds1 + dqkv W_in
                dx = ds1
            if bucket_hook is not None and (i == 0 or not self.merged_layer_bucket):
                # layer i's gradients final (merged: every layer's): that bucket's all-reduce
                wgb.run()
                cb.run()
                bucket_hook()
        # dmem = sum over layers of dK|dV_i W_kv_i: one GEMM over the stacked K = 2d * layers
        dmem = torch.empty(BP, d, device=dev, dtype=torch.float32)
        K.gemm(dkv_all, s["wkv"], out=dmem, split_k=-1)
        # embedding (dropout mask recomputed; PE has no parameters)
        K.embedding_bwd(s["caps"].view(-1), dx, G("embedding.weight"), drop_p=p, seed=seed, drop_stream=_S_EMB)
        denc = None
        if self.has_proj:
            dmem_c = dmem.to(ct)
            wgb.add(dmem_c, s["enc"].view(BP, self.E), out=G("encoder_proj.weight"), trans_a=True)
            cb.add(dmem, G("encoder_proj.bias"))
            if want_denc:
                denc = K.gemm(dmem_c, fp.w("encoder_proj.weight")).view(B, P, self.E)
        elif want_denc:
            denc = dmem.to(ct).view(B, P, d)
        if bucket_hook is None and TAIL_FORK and cb.items:
            # the bias-gradient column sums (one launch, ~120 us at C3, reading every dY of the
            # backward) beside the grouped weight-gradient GEMMs that read the same dY: the two
            # are independent, and the step ends with them alone on the chip
            main = torch.cuda.current_stream(dev)
            side = self._side_stream(dev)
            K.fork(side, main)
            # the operands the side stream reads were allocated on the main stream: held until the
            # join, so the caching allocator cannot hand their blocks to a main-stream allocation
            # while the column sums still read them (the round-4 side-stream drift)
            held = [it[0] for it in cb.items]
            with torch.cuda.stream(side):
                cb.run()
            wgb.run()
            K.join(main, side)
            del held
        else:
            wgb.run()
            cb.run()
        s["denc"] = denc
        return gbuf

    def _side_stream(self, dev):
        if getattr(self, "_side", None) is None or self._side.device != dev:
            self._side = torch.cuda.Stream(device=dev)
        return self._side

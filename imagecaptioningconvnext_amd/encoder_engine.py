"""Forward (with saved activations) and backward of the trainable ConvNeXt children on HIP.

``Encoder.fine_tune(fine_tune=True, startingLayer=s)`` (models/encoder.py:29-34) makes
``convnext.children()[s:]`` trainable; train.py:113-114,138-139 then give them their own Adam
(lr = encoderLr) and train.py:278-290 back-propagates the caption loss into them.  This engine
runs that encoder half of the step:

  * children < s: the frozen fast path (fused CNBlock MLP, bf16 packed weights, no saved state)
  * children >= s: per CNBlock  dwconv7 -> LayerNorm (mean/rstd saved) -> Linear+GELU (the
    pre-activation saved through the GEMM epilogue) -> Linear with layer-scale, per-sample
    stochastic depth and the residual in the epilogue (out of place: the block input is kept
    for the depthwise weight gradient); per downsample  LayerNorm2d + 2x2 patchify in the
    torch weight's (c, kh, kw) order -> GEMM with the Conv2d weight as stored
  * backward walks the same children in reverse (csrc/convnext_bwd.hip lists the math).

The trainable parameters live in one FlatParams buffer (fp32 master + bf16 shadow + grads +
Adam moments), so the encoder optimiser step is one clamp+Adam launch and the DDP gradient
average one all-reduce, exactly like the decoder's.
"""
import torch

from . import kernels as K
from .flat import FlatParams


class EncoderEngine:
    def __init__(self, enc, device):
        self.enc = enc
        self.ct = enc.compute_dtype
        children = list(enc.convnext.children())
        train = [i for i, c in enumerate(children) if any(p.requires_grad for p in c.parameters())]
        if not train:
            raise ValueError("EncoderEngine needs at least one trainable child (Encoder.fine_tune)")
        self.s0 = train[0]
        if any(i not in train for i in range(self.s0, len(children))):
            raise NotImplementedError("trainable children must be a suffix convnext.children()[startingLayer:]")
        if self.s0 == 0:
            raise NotImplementedError("fine-tuning the stem (startingLayer=0) is not supported; use startingLayer>=1")
        names = [(n, p) for n, p in enc.named_parameters() if p.requires_grad]
        self.fp = FlatParams([[np_] for np_ in names], device, self.ct)
        self.key = tuple(n for n, _ in names)

    # -- parameter views ---------------------------------------------------------------------
    def _blk(self, ci, j, gbuf=None):
        pre = f"convnext.{ci}.{j}."
        fp = self.fp
        C = fp.offsets[pre + "block.0.bias"][1][0]
        return dict(
            C=C,
            dw=fp.f32(pre + "block.0.weight", (C, 49)), dwb=fp.f32(pre + "block.0.bias"),
            lnw=fp.f32(pre + "block.2.weight"), lnb=fp.f32(pre + "block.2.bias"),
            w1=fp.w(pre + "block.3.weight"), b1=fp.f32(pre + "block.3.bias"),
            w2=fp.w(pre + "block.5.weight"), w2m=fp.f32(pre + "block.5.weight"), b2=fp.f32(pre + "block.5.bias"),
            gamma=fp.f32(pre + "layer_scale", (C,)),
            g=lambda n, shape=None: fp.g(pre + n, shape, buf=gbuf),
        )

    def _down(self, ci, gbuf=None):
        pre = f"convnext.{ci}."
        fp = self.fp
        C2, C = fp.offsets[pre + "1.weight"][1][:2]
        return dict(C=C, C2=C2, lnw=fp.f32(pre + "0.weight"), lnb=fp.f32(pre + "0.bias"),
                    w=fp.w(pre + "1.weight", (C2, 4 * C)), b=fp.f32(pre + "1.bias"),
                    g=lambda n, shape=None: fp.g(pre + n, shape, buf=gbuf))

    # -- forward -----------------------------------------------------------------------------
    def forward(self, images):
        """Encoder.forward (encoder.py:23-27) in train mode; returns (features [B,s,s,E], saved)."""
        enc, ct = self.enc, self.ct
        from .models.encoder import as_input
        images = as_input(images)
        B, _, H, W = images.shape
        dev = images.device
        sd = enc._sd_scales(B, dev) if enc.training else None
        x, bid = enc._run_frozen(images, upto=self.s0, sd=sd)
        saved = dict(B=B, sd=sd, layers=[])
        children = list(enc.convnext.children())
        for ci in range(self.s0, len(children)):
            if ci % 2 == 1:  # CNBlock stage
                blocks = []
                for j in range(len(children[ci])):
                    p = self._blk(ci, j)
                    rs = sd[bid] if (sd is not None and children[ci][j].sd_prob > 0) else None
                    x, st = self._block_fwd(x, p, rs)
                    blocks.append(st)
                    bid += 1
                saved["layers"].append(("stage", ci, blocks))
            else:            # downsample
                p = self._down(ci)
                _, h, w, C = x.shape
                patches = torch.empty(B * (h // 2) * (w // 2), 4 * C, device=dev, dtype=ct)
                K.ln_patchify2(x, p["lnw"], p["lnb"], patches, cmajor=True)
                xo = torch.empty(B, h // 2, w // 2, p["C2"], device=dev, dtype=ct)
                K.gemm(patches, p["w"], trans_b=True, bias=p["b"], out=xo.view(-1, p["C2"]))
                saved["layers"].append(("down", ci, dict(x=x, patches=patches)))
                x = xo
        saved["pre_pool"] = x
        s = enc.enc_image_size
        if x.shape[1] == s and x.shape[2] == s:
            return x, saved
        out = torch.empty(B, s, s, x.shape[3], device=dev, dtype=ct)
        return K.adaptive_pool(x, s, s, out), saved

    def _block_fwd(self, x, p, rs):
        B, h, w, C = x.shape
        M = B * h * w
        ct, dev = self.ct, x.device
        w49 = K.transpose(p["dw"])                                  # [49, C] tap-major
        z = torch.empty_like(x)
        K.dwconv7(x, w49, p["dwb"], z)
        zn, mean, rstd = K.add_layernorm(z.view(M, C), None, p["lnw"], p["lnb"], 1e-6)
        hpre = torch.empty(M, 4 * C, device=dev, dtype=ct)
        a = K.gemm(zn, p["w1"], trans_b=True, bias=p["b1"], act=K.ACT_GELU, aux=hpre)
        xo = torch.empty_like(x)
        K.gemm(a, p["w2"], trans_b=True, bias=p["b2"], colscale=p["gamma"], rowscale=rs, rows_per_scale=h * w,
               res=x.view(M, C), out=xo.view(M, C))
        return xo, dict(x=x, w49=w49, z=z, zn=zn, mean=mean, rstd=rstd, hpre=hpre, a=a, rs=rs)

    # -- gradient buckets (DDP) ----------------------------------------------------------------
    BUCKET_BYTES = 25 << 20  # torch DDP's default bucket_cap_mb (trainMultiGPU.py:233)

    def _units(self):
        """(child, block or None, flat [lo, hi)) of every trainable unit in backward order."""
        fp = self.fp
        children = list(self.enc.convnext.children())
        units = []
        for ci in range(len(children) - 1, self.s0 - 1, -1):
            if ci % 2 == 1:
                for j in range(len(children[ci]) - 1, -1, -1):
                    pre = f"convnext.{ci}.{j}."
                    units.append((ci, j, fp.span([n for n in fp.params if n.startswith(pre)])))
            else:
                pre = f"convnext.{ci}."
                units.append((ci, None, fp.span([n for n in fp.params if n.startswith(pre)])))
        return units

    def grad_buckets(self, cap_bytes=None):
        """Flat ranges in the order backward() calls ``bucket_hook``: consecutive units (CNBlocks,
        downsamples) in backward order cut once they reach ``cap_bytes`` of fp32 gradients (25 MiB:
        DDP's default bucket size, trainMultiGPU.py:233-235); the hook fires when the unit that
        completes a bucket is done, so its all-reduce overlaps the blocks below.  The last, partial
        bucket is left to the caller (final when backward() returns).  The flat buffer holds the
        units in forward order, so each bucket is one contiguous range."""
        cap = (self.BUCKET_BYTES if cap_bytes is None else cap_bytes) // 4
        out, fire = [], set()
        hi = None
        for ci, j, (lo, uhi) in self._units():
            hi = uhi if hi is None else hi
            if hi - lo >= cap:
                out.append((lo, hi))
                fire.add((ci, j))
                hi = None
        self._fire = fire
        return out

    # -- backward ----------------------------------------------------------------------------
    def backward(self, saved, dfeat, gbuf=None, bucket_hook=None):
        """dfeat: dL/d(features) [B, s, s, E] (any float dtype).  Writes the trainable
        parameters' gradients into ``gbuf`` (default ``fp.grad``; overwritten, not accumulated).
        ``bucket_hook``: called when the unit completing each grad_buckets() range is done."""
        ct = self.ct
        fire = getattr(self, "_fire", None) if bucket_hook is not None else None
        if bucket_hook is not None and fire is None:
            self.grad_buckets()
            fire = self._fire
        gbuf = self.fp.grad if gbuf is None else gbuf
        gbuf.zero_()
        x = saved["pre_pool"]
        B, h, w, C = x.shape
        if dfeat.shape[1] == h and dfeat.shape[2] == w:
            dx = dfeat.to(ct).contiguous()
        else:
            dx = torch.empty(B, h, w, C, device=x.device, dtype=ct)
            K.adaptive_pool_bwd(dfeat.to(ct).contiguous(), h, w, dx)
        layers = saved["layers"]
        for li in range(len(layers) - 1, -1, -1):
            kind, ci, st = layers[li]
            need_dx = li > 0
            if kind == "stage":
                for j in range(len(st) - 1, -1, -1):
                    dx = self._block_bwd(dx, self._blk(ci, j, gbuf), st[j], need_dx=need_dx or j > 0)
                    if fire and (ci, j) in fire:
                        bucket_hook()
            else:
                dx = self._down_bwd(dx, self._down(ci, gbuf), st, need_dx=need_dx)
                if fire and (ci, None) in fire:
                    bucket_hook()
        return gbuf

    def _block_bwd(self, dout, p, st, need_dx):
        B, h, w, C = dout.shape
        M = B * h * w
        ct, dev = self.ct, dout.device
        d2 = dout.view(M, C)
        dpr = K.rowscale(d2, st["rs"], h * w) if st["rs"] is not None else d2       # dout * sd
        G = K.gemm(dpr, st["a"], trans_a=True, out_dtype=torch.float32, split_k=-1)  # [C, 4C]
        cs = torch.empty(C, device=dev, dtype=torch.float32)
        K.colsum(dpr, cs)
        wg = torch.empty(C, 4 * C, device=dev, dtype=ct)
        K.layer_scale_grad(G, p["w2m"], p["b2"], p["gamma"], cs, p["g"]("block.5.weight"), wg,
                           p["g"]("layer_scale", (C,)), p["g"]("block.5.bias"))
        dh = K.gemm(dpr, wg, act=K.ACT_DGELU, aux=st["hpre"])                        # [M, 4C]
        K.gemm(dh, st["zn"], trans_a=True, out=p["g"]("block.3.weight"), split_k=-1)
        K.colsum(dh, p["g"]("block.3.bias"))
        dzn = K.gemm(dh, p["w1"])                                                     # [M, C]
        dz = K.add_layernorm_bwd(dzn, st["z"].view(M, C), st["mean"], st["rstd"], p["lnw"],
                                 p["g"]("block.2.weight"), p["g"]("block.2.bias"))
        dz4 = dz.view(B, h, w, C)
        K.dwconv7_wgrad(dz4, st["x"], p["g"]("block.0.weight", (C, 49)), p["g"]("block.0.bias"))
        if not need_dx:
            return None
        dx = torch.empty_like(dout)
        return K.dwconv7_bwd_data(dz4, st["w49"], dx, res=dout)

    def _down_bwd(self, dout, p, st, need_dx):
        B, ho, wo, C2 = dout.shape
        C = p["C"]
        d2 = dout.view(-1, C2)
        K.gemm(d2, st["patches"], trans_a=True, out=p["g"]("1.weight", (C2, 4 * C)), split_k=-1)
        K.colsum(d2, p["g"]("1.bias"))
        # dpatch / dx are needed even at the lowest trainable child: the LayerNorm2d weights'
        # gradients come out of the same pass
        dpatch = K.gemm(d2, p["w"])                                                   # [B*ho*wo, 4C]
        x = st["x"]
        dx = torch.empty_like(x)
        K.ln_patchify2_bwd(x, dpatch, p["lnw"], dx, p["g"]("0.weight"), p["g"]("0.bias"), cmajor=True)
        return dx

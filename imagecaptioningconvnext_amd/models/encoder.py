"""ConvNeXt encoder with the reference's class surface (models/encoder.py:14-34).

``Encoder(encoded_image_size=7)`` exposes ``.convnext`` (the 8-child ``features`` Sequential,
torchvision parameter names, so reference checkpoints' ``convnext.{i}...`` keys load
unchanged), ``.adaptive_pool``, ``.forward(images) -> [B, 7, 7, E]`` and
``.fine_tune(fine_tune, startingLayer)``.  The reference hard-codes ConvNeXt-Base with
ImageNet weights (encoder.py:18); there is no network here, so weights are randomly
initialised the torchvision way and ``variant`` selects tiny/base/large (BASELINE configs).

forward runs the NHWC trunk on the HIP kernels: stem (conv4x4+LN) -> per CNBlock
dwconv7x7+LN -> MFMA GEMM (Linear C->4C, +bias, GELU) -> MFMA GEMM (Linear 4C->C, +bias,
*layer_scale, *stochastic-depth, +residual, in place) -> downsample LN + 2x2 patch GEMM ->
adaptive pool.  With trainable children (``fine_tune(True, startingLayer)``) the trainable
suffix runs on encoder_engine.EncoderEngine (saved activations + HIP backward) and the output is
differentiable; the frozen prefix always takes the fused fast path.
"""
import math

import torch
from torch import nn

from .. import kernels as K


VARIANTS = {
    "tiny": ((96, 192, 384, 768), (3, 3, 9, 3), 0.1),
    "small": ((96, 192, 384, 768), (3, 3, 27, 3), 0.4),
    "base": ((128, 256, 512, 1024), (3, 3, 27, 3), 0.5),
    "large": ((192, 384, 768, 1536), (3, 3, 27, 3), 0.5),
}


SD_STREAM = 7  # RNG stream id of the encoder's stochastic-depth draws


class _LayerNorm2d(nn.LayerNorm):
    """Parameter holder with torchvision's LayerNorm2d names (weight, bias), eps 1e-6."""


class _Permute(nn.Module):
    def __init__(self, dims):
        super().__init__()
        self.dims = dims


IMAGENET_MEAN = (0.485, 0.456, 0.406)  # train.py:152 transforms.Normalize
IMAGENET_STD = (0.229, 0.224, 0.225)


def as_input(images):
    """Encoder input: normalised fp32 images, or the dataset's raw uint8 pixels (kept as bytes:
    the stem kernel normalises them, dataLoader.py:46 + train.py:152)."""
    return images.contiguous() if images.dtype == torch.uint8 else images.float().contiguous()


class CNBlock(nn.Module):
    """torchvision CNBlock parameter layout: block.{0: dwconv, 2: LayerNorm, 3: Linear C->4C,
    5: Linear 4C->C}, layer_scale [C,1,1]; stochastic-depth probability ``sd_prob``."""

    def __init__(self, dim, layer_scale, sd_prob):
        super().__init__()
        self.block = nn.Sequential(
            nn.Conv2d(dim, dim, kernel_size=7, padding=3, groups=dim, bias=True),
            _Permute([0, 2, 3, 1]),
            nn.LayerNorm(dim, eps=1e-6),
            nn.Linear(dim, 4 * dim, bias=True),
            nn.GELU(),
            nn.Linear(4 * dim, dim, bias=True),
            _Permute([0, 3, 1, 2]),
        )
        self.layer_scale = nn.Parameter(torch.ones(dim, 1, 1) * layer_scale)
        self.sd_prob = sd_prob


def build_features(variant):
    chans, depths, sd_max = VARIANTS[variant]
    layers = [nn.Sequential(nn.Conv2d(3, chans[0], kernel_size=4, stride=4, bias=True),
                            _LayerNorm2d(chans[0], eps=1e-6))]
    total = sum(depths)
    bid = 0
    for st in range(4):
        blocks = []
        for _ in range(depths[st]):
            blocks.append(CNBlock(chans[st], 1e-6, sd_max * bid / (total - 1.0)))
            bid += 1
        layers.append(nn.Sequential(*blocks))
        if st < 3:
            layers.append(nn.Sequential(_LayerNorm2d(chans[st], eps=1e-6),
                                        nn.Conv2d(chans[st], chans[st + 1], kernel_size=2, stride=2)))
    feats = nn.Sequential(*layers)
    for m in feats.modules():  # torchvision ConvNeXt init
        if isinstance(m, (nn.Conv2d, nn.Linear)):
            nn.init.trunc_normal_(m.weight, std=0.02)
            if m.bias is not None:
                nn.init.zeros_(m.bias)
    return feats


class _EncoderTrain(torch.autograd.Function):
    """Differentiable encoder forward over the trainable children's parameters (FlatParams
    order); backward = EncoderEngine.backward, handing autograd one grad view per parameter."""

    @staticmethod
    def forward(ctx, engine, images, *params):
        feats, saved = engine.forward(images)
        ctx.engine, ctx.saved = engine, saved
        return feats

    @staticmethod
    def backward(ctx, dfeat):
        eng = ctx.engine
        gbuf = torch.empty_like(eng.fp.grad)  # autograd accumulates the returned views into .grad
        eng.backward(ctx.saved, dfeat, gbuf=gbuf)
        grads = tuple(eng.fp.g(n, buf=gbuf) for n in eng.fp.params)
        return (None, None) + grads


class Encoder(nn.Module):
    def __init__(self, encoded_image_size=7, variant="base", compute_dtype=torch.bfloat16, frozen_fp8=False):
        super().__init__()
        self.enc_image_size = encoded_image_size
        self.variant = variant
        # frozen_fp8: the frozen CNBlocks that run as two GEMMs (C >= 384) use block-scaled fp8
        # (MX-FP8: LayerNorm -> fp8 rows, W1/W2 packed once, GELU output re-quantized in the
        # first GEMM's epilogue) -- config C5's "frozen stages in fp8" 
        self.frozen_fp8 = frozen_fp8
        self.encoder_dim = VARIANTS[variant][0][3]
        self.compute_dtype = compute_dtype
        self.convnext = build_features(variant)
        self.adaptive_pool = nn.AdaptiveAvgPool2d((encoded_image_size, encoded_image_size))
        self.sd_seed = 0
        self._packed = None
        self._packed_key = None
        # superseded packs stay referenced: a captured HIP graph holds raw pointers into them
        # (train_step drops them when it re-captures)
        self._retired_packs = []
        self._engine = None
        # bumped by weights_updated() after every fine-tuned optimizer step: the engine's Adam
        # writes the trainable children through raw pointers, which bumps no tensor version
        self._weights_epoch = 0
        self._packed_epoch = 0
        self.fine_tune()

    def fine_tune(self, fine_tune=True, startingLayer=7):
        """encoder.py:29-34: freeze everything, then set requires_grad on children[startingLayer:]."""
        for p in self.convnext.parameters():
            p.requires_grad = False
        for c in list(self.convnext.children())[startingLayer:]:
            for p in c.parameters():
                p.requires_grad = fine_tune

    # -- weight packing into kernel layouts ----------------------------------------------------
    def _pack_key(self):
        ps = list(self.convnext.parameters())
        return (self.compute_dtype, self.frozen_fp8, ps[0].device, tuple(p._version for p in ps),
                tuple(p.data_ptr() for p in ps))

    def _pack(self):
        key = self._pack_key()
        if self._packed is not None and self._packed_key == key:
            return self._packed
        if self._packed is not None:
            self._retired_packs.append(self._packed)
        ct = self.compute_dtype
        f = self.convnext
        with torch.no_grad():
            stem_conv, stem_ln = f[0][0], f[0][1]
            pk = {"stem": (stem_conv.weight.reshape(stem_conv.out_channels, 48).float().contiguous(),
                           stem_conv.bias.float().contiguous(), stem_ln.weight.float().contiguous(),
                           stem_ln.bias.float().contiguous())}
            stages = []
            for st in range(4):
                blocks = [self._pack_block(blk) for blk in f[1 + 2 * st]]
                down = self._pack_down(f[2 + 2 * st]) if st < 3 else None
                stages.append((blocks, down))
            pk["stages"] = stages
        self._packed, self._packed_key = pk, key
        self._packed_epoch = self._weights_epoch
        return pk

    def _pack_block(self, blk):
        ct = self.compute_dtype
        dw, ln, l1, l2 = blk.block[0], blk.block[2], blk.block[3], blk.block[5]
        C = dw.out_channels
        d = dict(w49=dw.weight.reshape(C, 49).t().float().contiguous(), dwb=dw.bias.float().contiguous(),
                 lnw=ln.weight.float().contiguous(), lnb=ln.bias.float().contiguous(),
                 w1=l1.weight.to(ct).contiguous(), b1=l1.bias.float().contiguous(),
                 w2=l2.weight.to(ct).contiguous(), b2=l2.bias.float().contiguous(),
                 gamma=blk.layer_scale.reshape(C).float().contiguous(), sd=blk.sd_prob)
        if self._mx_stage(C):  # fp8 copies of the frozen Linear weights (rows = outputs)
            d.update(w1mx=K.mx_quant_rows(l1.weight.float().contiguous()),
                     w2mx=K.mx_quant_rows(l2.weight.float().contiguous()))
        return d

    def _pack_down(self, seq):
        ln, cv = seq[0], seq[1]
        return dict(lnw=ln.weight.float().contiguous(), lnb=ln.bias.float().contiguous(),
                    w=cv.weight.permute(0, 2, 3, 1).reshape(cv.out_channels, -1).to(self.compute_dtype).contiguous(),
                    b=cv.bias.float().contiguous())

    def weights_updated(self):
        """The fine-tuned children's weights changed behind torch's back (EncoderEngine's Adam
        writes its flat buffer through raw pointers): the packed copies the frozen fast path reads
        for those children are refreshed before their next use (_run_frozen over them, e.g.
        validation under no_grad)."""
        self._weights_epoch += 1

    def _refresh_trainable(self, pk, upto):
        """Re-derive, in place, the packed entries of trainable children below ``upto`` (captured
        graphs keep their pointers; the frozen prefix is untouched)."""
        f = self.convnext
        with torch.no_grad():
            for st, (blocks, down) in enumerate(pk["stages"]):
                ci = 1 + 2 * st
                if ci < upto and any(p.requires_grad for p in f[ci].parameters()):
                    for d, blk in zip(blocks, f[ci]):
                        for k, v in self._pack_block(blk).items():
                            if torch.is_tensor(v):
                                d[k].copy_(v)
                            elif isinstance(v, tuple):
                                for a, b in zip(d[k], v):
                                    a.copy_(b)
                if down is not None and ci + 1 < upto and any(p.requires_grad for p in f[ci + 1].parameters()):
                    for k, v in self._pack_down(f[ci + 1]).items():
                        down[k].copy_(v)
        self._packed_epoch = self._weights_epoch

    def _mx_stage(self, C):
        return (self.frozen_fp8 and self.compute_dtype == torch.bfloat16 and C not in K.CNBLOCK_MLP_CHANNELS
                and C % 128 == 0)

    def _sd_scales(self, B, device):
        """StochasticDepth(p, "row") per-sample scales keep/(1-p) for every block (train mode),
        drawn on the device by the counter RNG (no host sync; graph-capturable)."""
        pk = self._pack()
        if "sd_probs" not in pk:
            probs = [blk.sd_prob for s in range(4) for blk in self.convnext[1 + 2 * s]]
            pk["sd_probs"] = torch.tensor(probs, device=device, dtype=torch.float32)
        probs = pk["sd_probs"]
        out = torch.empty(probs.numel(), B, device=device, dtype=torch.float32)
        K.stochastic_depth_scales(probs, B, self.sd_seed, SD_STREAM, out)
        self.sd_seed += 1
        return out

    def _run_frozen(self, images, upto=8, sd=None):
        """Stem + children [1, upto) of the trunk on the frozen fast path (no saved state).
        Returns (x NHWC in the compute dtype, index of the next CNBlock for the SD scales)."""
        pk = self._pack()
        if self._packed_epoch != self._weights_epoch:
            self._refresh_trainable(pk, upto)
        ct = self.compute_dtype
        B, _, H, W = images.shape
        dev = images.device
        C0 = pk["stem"][0].shape[0]
        x = torch.empty(B, H // 4, W // 4, C0, device=dev, dtype=ct)
        if images.dtype == torch.uint8 and "norm" not in pk:  # train.py:152 ImageNet normalisation
            pk["norm"] = (torch.tensor(IMAGENET_MEAN, device=dev), torch.tensor(IMAGENET_STD, device=dev))
        K.convnext_stem(images, *pk["stem"], x, norm=pk.get("norm"))
        bid = 0
        for st, (blocks, down) in enumerate(pk["stages"]):
            if 1 + 2 * st >= upto:
                break
            _, h, w, C = x.shape
            M = B * h * w
            z = torch.empty_like(x)
            hid = zn = None
            fused = ct == torch.bfloat16 and C in K.CNBLOCK_MLP_CHANNELS
            mx = self._mx_stage(C) and "w1mx" in blocks[0]
            if mx:
                u8 = dict(device=dev, dtype=torch.uint8)
                znq = (torch.empty(M, C, **u8), torch.empty(M, C // 32, **u8))
                hidq = (torch.empty(M, 4 * C, **u8), torch.empty(M, 4 * C // 32, **u8))
            elif not fused:
                hid = torch.empty(M, 4 * C, device=dev, dtype=ct)
                zn = torch.empty(M, C, device=dev, dtype=ct)
            x2 = x.view(M, C)
            # MX stages: the depthwise writes bf16 rows, the quantiser applies the LayerNorm and
            # writes the fp8 rows + block scales (a depthwise + LayerNorm + MX quantisation kernel
            # measured slower at C5 in round 4 and was removed)
            for blk in blocks:
                rs = sd[bid] if (sd is not None and blk["sd"] > 0) else None
                if w <= 64 and (mx or fused or not K.dw_ln_fused(w, C, ct)):
                    # channel-tiled depthwise; LayerNorm applied by the consumer
                    K.dwconv7(x, blk["w49"], blk["dwb"], z)
                    ln = (blk["lnw"], blk["lnb"])
                else:  # the LayerNorm fused: late stages (channel-pair kernel) / wide images (rows)
                    K.dwconv7_ln(x, blk["w49"], blk["dwb"], blk["lnw"], blk["lnb"], z)
                    ln = (None, None)
                if mx:  # LN -> fp8 rows; fp8 Linear + GELU -> fp8 hidden; fp8 Linear + scale + residual
                    if ln[0] is not None:
                        K.mx_quant_rows(z.view(M, C), ln[0], ln[1], 1e-6, out=znq)
                    else:
                        K.mx_quant_rows(z.view(M, C), out=znq)
                    K.gemm_mx(znq, blk["w1mx"], bias=blk["b1"], act=K.ACT_GELU, out_dtype="mx", out=hidq)
                    K.gemm_mx(hidq, blk["w2mx"], bias=blk["b2"], colscale=blk["gamma"], rowscale=rs,
                              rows_per_scale=h * w, res=x2, out=x2)
                elif fused:  # LN -> Linear -> GELU -> Linear -> layer_scale -> drop path -> residual, on chip
                    K.cnblock_mlp(z.view(M, C), blk["w1"], blk["b1"], blk["w2"], blk["b2"], blk["gamma"], x2,
                                  sd=rs, rows_per_sample=h * w, ln_w=ln[0], ln_b=ln[1])
                else:
                    zn2 = z.view(M, C)
                    if ln[0] is not None:
                        K.add_layernorm(zn2, None, ln[0], ln[1], 1e-6, y=zn)
                        zn2 = zn
                    K.gemm(zn2, blk["w1"], trans_b=True, bias=blk["b1"], act=K.ACT_GELU, out=hid)
                    K.gemm(hid, blk["w2"], trans_b=True, bias=blk["b2"], colscale=blk["gamma"], rowscale=rs,
                           rows_per_scale=h * w, res=x2, out=x2)
                bid += 1
            if down is not None and 2 + 2 * st < upto:
                patches = torch.empty(B * (h // 2) * (w // 2), 4 * C, device=dev, dtype=ct)
                K.ln_patchify2(x, down["lnw"], down["lnb"], patches)
                C2 = down["w"].shape[0]
                x = torch.empty(B, h // 2, w // 2, C2, device=dev, dtype=ct)
                K.gemm(patches, down["w"], trans_b=True, bias=down["b"], out=x.view(-1, C2))
        return x, bid

    def release_retired(self):
        """Drop the superseded weight packs (no captured graph refers to them any more)."""
        self._retired_packs = []

    def trainable(self):
        return any(p.requires_grad for p in self.convnext.parameters())

    def engine(self):
        """HIP engine of the trainable children (rebuilt when fine_tune changes the set)."""
        from ..encoder_engine import EncoderEngine
        key = tuple(n for n, p in self.named_parameters() if p.requires_grad)
        dev = next(self.convnext.parameters()).device
        if self._engine is None or self._engine.key != key or not self._engine.fp.check_bound():
            self._engine = EncoderEngine(self, dev)
        return self._engine

    def forward(self, images):
        """encoder.py:23-27.  images [B,3,H,W] on the GPU (normalised f32, or raw uint8 pixels that the
        stem normalises) -> [B, s, s, E] NHWC, compute dtype.
        With trainable children (fine_tune) and grad enabled the output is differentiable:
        backward runs the HIP encoder backward into the parameters' .grad."""
        if not images.is_cuda:
            raise RuntimeError("Encoder.forward runs on the HIP kernels only; move images to the GPU")
        if self.trainable() and torch.is_grad_enabled():
            eng = self.engine()
            return _EncoderTrain.apply(eng, images, *eng.fp.params.values())
        images = as_input(images)
        B = images.shape[0]
        sd = self._sd_scales(B, images.device) if self.training else None
        x, _ = self._run_frozen(images, 8, sd)
        s = self.enc_image_size
        if x.shape[1] == s and x.shape[2] == s:
            return x
        out = torch.empty(B, s, s, x.shape[3], device=images.device, dtype=self.compute_dtype)
        return K.adaptive_pool(x, s, s, out)

    def macs_per_image(self, hw=224, start=0):
        """Multiply-accumulates per image of convnext.children()[start:] (all of them by default)."""
        chans, depths, _ = VARIANTS[self.variant]
        h = hw // 4
        m = h * h * chans[0] * 48 if start <= 0 else 0
        for st in range(4):
            C = chans[st]
            if 1 + 2 * st >= start:
                m += depths[st] * (h * h * C * 49 + 2 * h * h * C * 4 * C)
            if st < 3:
                h //= 2
                if 2 + 2 * st >= start:
                    m += h * h * chans[st + 1] * 4 * C
        return m

"""ConvNeXt-{tiny,base,large} ``features`` trunk + adaptive pool, restated on torch CPU.

Follows models/encoder.py:14-34 (``convnext_base(...).features`` -> AdaptiveAvgPool2d(7) ->
permute(0,2,3,1)) and torchvision's published ConvNeXt definition for the trunk (third-party,
un-vendored; see oracle/__init__.py for how this is pinned):

  features[0]      Conv2d(3, C0, k=4, s=4, bias) -> LayerNorm2d(C0, eps=1e-6)
  features[1,3,5,7] stages of CNBlocks:
      y = x + SD_p( layer_scale * Linear2(GELU_erf(Linear1(LN_eps1e-6(dwconv7x7(x))))) )
      SD = StochasticDepth(p, "row"), p_i = p_max * i / (N_blocks - 1)
  features[2,4,6]  LayerNorm2d(C) -> Conv2d(C, 2C, k=2, s=2)
State-dict keys are ``convnext.{i}...`` exactly as the reference's ``Encoder`` holds them.
"""
import math

import torch
import torch.nn.functional as F

VARIANTS = {
    # channels, depths, stochastic-depth p_max (torchvision convnext_{tiny,base,large})
    "tiny": ((96, 192, 384, 768), (3, 3, 9, 3), 0.1),
    "small": ((96, 192, 384, 768), (3, 3, 27, 3), 0.4),
    "base": ((128, 256, 512, 1024), (3, 3, 27, 3), 0.5),
    "large": ((192, 384, 768, 1536), (3, 3, 27, 3), 0.5),
}


def param_shapes(variant):
    """{state-dict key: shape} of Encoder.convnext for a variant (encoder.py:19)."""
    chans, depths, _ = VARIANTS[variant]
    s = {"convnext.0.0.weight": (chans[0], 3, 4, 4), "convnext.0.0.bias": (chans[0],),
         "convnext.0.1.weight": (chans[0],), "convnext.0.1.bias": (chans[0],)}
    for st in range(4):
        C = chans[st]
        idx = 1 + 2 * st
        for j in range(depths[st]):
            p = f"convnext.{idx}.{j}."
            s[p + "block.0.weight"] = (C, 1, 7, 7)
            s[p + "block.0.bias"] = (C,)
            s[p + "block.2.weight"] = (C,)
            s[p + "block.2.bias"] = (C,)
            s[p + "block.3.weight"] = (4 * C, C)
            s[p + "block.3.bias"] = (4 * C,)
            s[p + "block.5.weight"] = (C, 4 * C)
            s[p + "block.5.bias"] = (C,)
            s[p + "layer_scale"] = (C, 1, 1)
        if st < 3:
            d = 2 + 2 * st
            s[f"convnext.{d}.0.weight"] = (C,)
            s[f"convnext.{d}.0.bias"] = (C,)
            s[f"convnext.{d}.1.weight"] = (chans[st + 1], C, 2, 2)
            s[f"convnext.{d}.1.bias"] = (chans[st + 1],)
    return s


def classifier_params(variant):
    """torchvision's classifier head (LayerNorm2d + Linear(C,1000)), only for the param-count check."""
    C = VARIANTS[variant][0][3]
    return 2 * C + C * 1000 + 1000


def macs_per_image(variant, hw=224):
    """Multiply-accumulates of features (+ classifier linear, as torchvision's GFLOPS count)."""
    chans, depths, _ = VARIANTS[variant]
    h = hw // 4
    m = h * h * chans[0] * 48
    for st in range(4):
        C = chans[st]
        m += depths[st] * (h * h * C * 49 + 2 * h * h * C * 4 * C)
        if st < 3:
            h //= 2
            m += h * h * chans[st + 1] * 4 * C
    return m + chans[3] * 1000


def sd_probs(variant):
    """Linearly ramped stochastic-depth probability per block (torchvision ConvNeXt)."""
    _, depths, pmax = VARIANTS[variant]
    n = sum(depths)
    return [pmax * i / (n - 1.0) for i in range(n)]


def _ln2d(x, w, b):  # LayerNorm2d on NCHW: normalise over C at each pixel, eps 1e-6
    return F.layer_norm(x.permute(0, 2, 3, 1), (x.shape[1],), w, b, 1e-6).permute(0, 3, 1, 2)


def _rb(t):  # round to bf16 and back (the HIP path stores activations / MFMA operands in bf16)
    return t.bfloat16().float()


def _id(t):
    return t


def features_forward(sd, variant, images, sd_keep=None, numerics="fp32", mx_children=()):
    """Encoder.convnext(images) (encoder.py:24).  ``images`` NCHW float; returns NCHW.

    ``sd_keep``: optional list (one per CNBlock) of per-sample scale vectors [B] applied to
    the residual branch (StochasticDepth "row" mode: keep/(1-p)); None = eval (identity).

    ``numerics`` (the build's arithmetic, for tighter parity gates than fp32-vs-bf16):
      "fp32": torchvision's fp32 semantics (the reference).
      "bf16": the HIP bf16 path's rounding points -- stem output, depthwise output, LayerNorm
              output (a GEMM operand), GELU hidden, block output, downsample LayerNorm output and
              result rounded to bf16; Linear / downsample weights bf16; stem and depthwise
              weights, biases, LayerNorm parameters, layer scale fp32; fp32 accumulation.
      "mx":   "bf16", and the CNBlocks of ``mx_children`` (feature indices 1/3/5/7) whose
              width qualifies (C % 128 == 0 and not a fused-MLP width 96/128/192) run the
              MX-FP8 path: LayerNorm output, both Linear weights and the GELU hidden are
              quantised per 32 along K (oracle/mx.py) instead of rounded to bf16.
    """
    from . import mx as mxq
    r = _id if numerics == "fp32" else _rb
    chans, depths, _ = VARIANTS[variant]
    x = F.conv2d(images, sd["convnext.0.0.weight"], sd["convnext.0.0.bias"], stride=4)
    x = r(_ln2d(x, sd["convnext.0.1.weight"], sd["convnext.0.1.bias"]))
    blk = 0
    for st in range(4):
        C = chans[st]
        idx = 1 + 2 * st
        use_mx = numerics == "mx" and idx in mx_children and C % 128 == 0 and C not in (96, 128, 192)
        q = mxq.qdq if use_mx else r
        for j in range(depths[st]):
            p = f"convnext.{idx}.{j}."
            y = r(F.conv2d(x, sd[p + "block.0.weight"], sd[p + "block.0.bias"], padding=3, groups=C))
            y = y.permute(0, 2, 3, 1)
            y = q(F.layer_norm(y, (C,), sd[p + "block.2.weight"], sd[p + "block.2.bias"], 1e-6))
            y = F.linear(y, q(sd[p + "block.3.weight"]), sd[p + "block.3.bias"])
            y = q(F.gelu(y))
            y = F.linear(y, q(sd[p + "block.5.weight"]), sd[p + "block.5.bias"])
            y = y.permute(0, 3, 1, 2)
            y = sd[p + "layer_scale"] * y
            if sd_keep is not None:
                y = y * sd_keep[blk].view(-1, 1, 1, 1).to(y.dtype)
            x = r(x + y)
            blk += 1
        if st < 3:
            d = 2 + 2 * st
            x = r(_ln2d(x, sd[f"convnext.{d}.0.weight"], sd[f"convnext.{d}.0.bias"]))
            x = r(F.conv2d(x, r(sd[f"convnext.{d}.1.weight"]), sd[f"convnext.{d}.1.bias"], stride=2))
    return x


def encoder_forward(sd, variant, images, encoded_image_size=7, sd_keep=None, numerics="fp32", mx_children=()):
    """Encoder.forward (encoder.py:23-27): features -> AdaptiveAvgPool2d(7) -> NHWC."""
    x = features_forward(sd, variant, images, sd_keep, numerics, mx_children)
    if x.shape[2] != encoded_image_size or x.shape[3] != encoded_image_size:
        x = F.adaptive_avg_pool2d(x, (encoded_image_size, encoded_image_size))
        if numerics != "fp32":
            x = _rb(x)
    return x.permute(0, 2, 3, 1)


def init_params(variant, generator=None):
    """torchvision-style init: trunc_normal(std .02) conv/linear weights, zero biases,
    LN weight 1 / bias 0, layer_scale 1e-6 (used by the product for random-init weights)."""
    out = {}
    for k, shp in param_shapes(variant).items():
        if k.endswith("layer_scale"):
            out[k] = torch.full(shp, 1e-6)
        elif len(shp) >= 2:
            t = torch.empty(shp)
            torch.nn.init.trunc_normal_(t, std=0.02, generator=generator)
            out[k] = t
        elif k.endswith("weight"):
            out[k] = torch.ones(shp)
        else:
            out[k] = torch.zeros(shp)
    return out


def param_count(variant):
    return sum(math.prod(s) for s in param_shapes(variant).values())

"""Deterministic parameter/input recipes shared by tools/gen_golden.py (which runs the
reference in this container) and the tests (which run here and on the GPU box).

The recipes use only torch's CPU generator, so the same torch build reproduces them
bit-for-bit on both machines (the GPU box runs the same image).  Test infrastructure only.
"""
import math
import os

import torch

GOLDEN_DIR = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def make_params(named_shapes, seed):
    """Fill ``{name: shape}`` deterministically (names visited in sorted order).

    2-D/4-D weights ~ U(-1/sqrt(fan_in), 1/sqrt(fan_in)); norm weights ~ 1 + U(-.1,.1);
    every other 1-D tensor (biases, layer-scale) ~ U(-.1, .1).  Layer scale is randomised
    on purpose so the ConvNeXt block branch is exercised (SURVEY.md §7 hard part vi).
    """
    g = torch.Generator().manual_seed(seed)
    out = {}
    for name in sorted(named_shapes):
        shape = tuple(named_shapes[name])
        u = torch.rand(shape, generator=g, dtype=torch.float64) * 2 - 1
        if len(shape) >= 2 and not name.endswith("layer_scale"):
            fan_in = int(math.prod(shape[1:]))
            t = u / math.sqrt(fan_in)
        elif ("norm" in name or name.endswith(".2.weight") or "convnext.0.1" in name) and name.endswith("weight") and len(shape) == 1:
            t = 1.0 + 0.1 * u
        else:
            t = 0.1 * u
        out[name] = t.to(torch.float32).contiguous()
    return out


def make_captions(B, L, caplens, V, seed):
    """Captions as the reference's COCO files hold them (utils.py:138-144):
    ``<start>`` w_1..w_{n-2} ``<end>`` ``<pad>``...; ids: <pad>=0, <unk>=V-3, <start>=V-2,
    <end>=V-1 (SURVEY.md §8 notation)."""
    g = torch.Generator().manual_seed(seed)
    caps = torch.randint(1, V - 3, (B, L), generator=g, dtype=torch.int64)
    for b, n in enumerate(caplens):
        caps[b, 0] = V - 2
        caps[b, n - 1] = V - 1
        caps[b, n:] = 0
    return caps, torch.tensor(caplens, dtype=torch.int64).view(B, 1)


def make_features(shape, seed):
    g = torch.Generator().manual_seed(seed)
    return torch.randn(shape, generator=g, dtype=torch.float32)


def word_map(V):
    wm = {f"w{i}": i for i in range(1, V - 3)}
    wm.update({"<pad>": 0, "<unk>": V - 3, "<start>": V - 2, "<end>": V - 1})
    return wm

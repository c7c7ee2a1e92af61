"""Flat parameter storage: one contiguous fp32 master buffer per optimizer, laid out for HBM.

The trainable parameters of a module become views into ``flat``; their ``.grad`` become views
into ``grad``; Adam's moments live in ``m``/``v`` and the bf16 copy the kernels read lives in
``shadow``.  Consequences:
  * clip_gradient + Adam.step (utils.py:183-192, train.py:289-291) is ONE kernel launch over
    the whole buffer (imgcap_clamp_adam), which also refreshes the bf16 shadow;
  * the DDP gradient all-reduce (trainMultiGPU.py:233,384) is ONE collective on ``grad``;
  * parameters that the kernels consume as one operand (e.g. the LSTM's
    [decoder_att.weight; f_beta.weight; weight_hh] rows) are placed back to back inside a
    "group", so the concatenated operand is a zero-copy view of the shadow / grad buffers.
State-dict keys and nn.Parameter identities are unchanged (only ``.data`` is re-pointed).
"""
import math

import numpy as np
import torch

from . import kernels as K

ALIGN = 64  # elements between groups (256 B)


class FlatParams:
    def __init__(self, groups, device, compute_dtype):
        """groups: list of lists of (name, nn.Parameter); members of a group are contiguous."""
        self.device = torch.device(device)
        self.compute_dtype = compute_dtype
        self.offsets = {}
        self.params = {}
        off = 0
        for grp in groups:
            off = (off + ALIGN - 1) // ALIGN * ALIGN
            for name, p in grp:
                self.offsets[name] = (off, tuple(p.shape))
                self.params[name] = p
                off += p.numel()
        self.numel = (off + ALIGN - 1) // ALIGN * ALIGN
        f32 = dict(device=self.device, dtype=torch.float32)
        self.flat = torch.zeros(self.numel, **f32)
        self.grad = torch.zeros(self.numel, **f32)
        self.m = torch.zeros(self.numel, **f32)
        self.v = torch.zeros(self.numel, **f32)
        self.shadow = (torch.zeros(self.numel, device=self.device, dtype=torch.bfloat16)
                       if compute_dtype == torch.bfloat16 else None)
        with torch.no_grad():
            for name, p in self.params.items():
                o, shp = self.offsets[name]
                n = math.prod(shp)
                self.flat[o:o + n].copy_(p.data.reshape(-1).to(self.flat))
                p.data = self.flat[o:o + n].view(shp)
                p.grad = self.grad[o:o + n].view(shp)
        self.step_count = 0
        self._shadow_version = None
        self.refresh_shadow()

    # -- views -------------------------------------------------------------------------------
    def _span(self, name, count=None):
        o, shp = self.offsets[name]
        return o, math.prod(shp) if count is None else count

    def span(self, names):
        """[lo, hi) of the flat buffers covering ``names`` (must be contiguous up to alignment)."""
        lo = min(self.offsets[n][0] for n in names)
        hi = max(self.offsets[n][0] + math.prod(self.offsets[n][1]) for n in names)
        hi = min(self.numel, (hi + ALIGN - 1) // ALIGN * ALIGN)
        covered = sum(math.prod(self.offsets[n][1]) for n in names)
        inside = [n for n in self.params if lo <= self.offsets[n][0] < hi]
        if sorted(inside) != sorted(names) or covered > hi - lo:
            raise ValueError(f"parameters {names} are not contiguous in the flat buffer")
        return lo, hi

    def master(self, name):
        o, shp = self.offsets[name]
        return self.flat[o:o + math.prod(shp)].view(shp)

    def g(self, name, shape=None, count=None, buf=None):
        """View of ``name`` (or of ``count`` elements from its start) in the grad buffer."""
        o, n = self._span(name, count)
        return (self.grad if buf is None else buf)[o:o + n].view(shape or self.offsets[name][1])

    def w(self, name, shape=None, count=None):
        """Compute-dtype view (bf16 shadow or the fp32 master itself)."""
        self.sync_shadow()
        src = self.shadow if self.shadow is not None else self.flat
        o, n = self._span(name, count)
        return src[o:o + n].view(shape or self.offsets[name][1])

    def f32(self, name, shape=None, count=None):
        o, n = self._span(name, count)
        return self.flat[o:o + n].view(shape or self.offsets[name][1])

    # -- maintenance -------------------------------------------------------------------------
    def check_bound(self):
        """True while every nn.Parameter still views the flat buffer (module not re-.to()'d)."""
        for name, p in self.params.items():
            o, shp = self.offsets[name]
            if p.data.data_ptr() != self.flat.data_ptr() + 4 * o:
                return False
        return True

    def refresh_shadow(self):
        if self.shadow is not None:
            K.cast(self.flat, self.shadow)
        self._shadow_version = self.flat._version

    def sync_shadow(self):
        # in-place writes through the parameter views (load_state_dict, user code) bump the
        # shared version counter; the Adam kernel refreshes the shadow itself
        if self._shadow_version != self.flat._version:
            self.refresh_shadow()

    def zero_grad(self):
        self.grad.zero_()

    def adam_step(self, lr, clip, grad_div=1.0, betas=(0.9, 0.999), eps=1e-8, skip=None):
        """clip_gradient (clamp +-clip) then Adam, fused; refreshes the bf16 shadow.  ``skip``: a
        device fp32 word (the step's hand-off error count); nonzero at run time leaves the
        parameters, moments and shadow unchanged, but the host-side step count still advances
        (the skip word is only read on the device): a caller that catches the hand-off error from
        drain_metrics and keeps training runs Adam's bias correction one step ahead of the
        updates applied -- unlike torch.optim.Adam, which never takes a skipped step."""
        self.sync_shadow()
        self.step_count += 1
        K.clamp_adam(self.flat, self.grad, self.m, self.v, self.shadow, lr, self.step_count, clip,
                     grad_div=grad_div, betas=betas, eps=eps, skip=skip)
        self._shadow_version = self.flat._version  # kernel wrote flat + shadow through raw pointers

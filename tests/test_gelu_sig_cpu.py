"""The fused MLP's GELU (common.h ``gelu_sig``: x * sigmoid(x p(min(x^2, 25)))) restated in
numpy fp32 with the coefficients parsed from the header, against the exact erf form torch's
nn.GELU computes (the reference's torchvision CNBlock): the documented |error| <= 5.5e-5 over R,
saturation to x / -0 in the tails, NaN propagation."""
import math
import os
import re

import numpy as np

HDR = os.path.join(os.path.dirname(__file__), "..", "imagecaptioningconvnext_amd", "csrc", "common.h")


def _coeffs():
    src = open(HDR).read()
    body = src[src.index("DEV float gelu_sig(float x)"):]
    body = body[:body.index("}")]
    clamp = float(re.search(r"fminf\(x \* x, ([0-9.eE+-]+)f\)", body).group(1))
    k2, k1, k0 = (float(v) for v in re.search(
        r"fmaf\(fmaf\(s, ([0-9.eE+-]+)f, ([0-9.eE+-]+)f\), s, ([0-9.eE+-]+)f\)", body).groups())
    return clamp, k2, k1, k0


def gelu_sig(x):
    clamp, k2, k1, k0 = (np.float32(v) for v in _coeffs())
    x = x.astype(np.float32)
    s = np.minimum(x * x, clamp)
    p = (s * k2 + k1).astype(np.float32)
    p = (p * s + k0).astype(np.float32)
    with np.errstate(over="ignore"):
        e = np.exp2((x * p).astype(np.float32)).astype(np.float32)
    return (x * (np.float32(1) / (np.float32(1) + e))).astype(np.float32)


def gelu_erf(x):
    erf = np.vectorize(math.erf)
    x = x.astype(np.float64)
    return 0.5 * x * (1.0 + erf(x / math.sqrt(2.0)))


def test_gelu_sig_error_bound():
    x = np.linspace(-30, 30, 200001, dtype=np.float32)
    err = np.abs(gelu_sig(x).astype(np.float64) - gelu_erf(x))
    assert err.max() <= 5.5e-5, err.max()


def test_gelu_sig_tails_and_nan():
    x = np.array([-1e30, -80.0, 80.0, 1e30, np.nan], dtype=np.float32)
    y = gelu_sig(x)
    assert y[0] == 0 and y[1] == 0 and np.signbit(y[1])
    assert y[2] == np.float32(80.0) and y[3] == np.float32(1e30)
    assert np.isnan(y[4])

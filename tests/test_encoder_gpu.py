"""ConvNeXt encoder on the HIP path vs the CPU oracle (torchvision ConvNeXt definition)."""
import pytest
import torch

from golden_util import make_params
from oracle import convnext

pytestmark = pytest.mark.gpu


def _rel(a, b):
    a, b = a.detach().float().cpu(), b.detach().float().cpu()
    return ((a - b).norm() / (b.norm() + 1e-12)).item()


@pytest.mark.parametrize("dtype,tol", [(torch.float32, 1e-4), (torch.bfloat16, 3e-2)])
@pytest.mark.parametrize("hw", [224, 256])
def test_encoder_tiny_vs_oracle(hip_device, dtype, tol, hw):
    from imagecaptioningconvnext_amd.models.encoder import Encoder
    sd = make_params(convnext.param_shapes("tiny"), 5)
    enc = Encoder(variant="tiny", compute_dtype=dtype)
    enc.load_state_dict(sd)
    enc = enc.to(hip_device).eval()
    g = torch.Generator().manual_seed(6)
    img = torch.randn(2, 3, hw, hw, generator=g)
    with torch.no_grad():
        out = enc(img.to(hip_device))
        ref = convnext.encoder_forward(sd, "tiny", img)
    assert out.shape == ref.shape == (2, 7, 7, 768)
    assert _rel(out, ref) < tol


def test_encoder_stochastic_depth_train_mode(hip_device):
    """train(): per-sample row drop of residual branches; deterministic per seed; eval unaffected."""
    from imagecaptioningconvnext_amd.models.encoder import Encoder
    sd = make_params(convnext.param_shapes("tiny"), 7)
    enc = Encoder(variant="tiny", compute_dtype=torch.float32)
    enc.load_state_dict(sd)
    enc = enc.to(hip_device)
    img = torch.randn(4, 3, 224, 224).to(hip_device)
    with torch.no_grad():
        enc.eval()
        e0 = enc(img)
        enc.train()
        enc.sd_seed = 3
        a = enc(img)
        enc.sd_seed = 3
        b = enc(img)
    assert torch.equal(a, b)
    assert not torch.equal(a, e0)
    # reference oracle with the same keep masks reproduces the train-mode output
    scales = None
    enc.sd_seed = 3
    scales = enc._sd_scales(4, hip_device).cpu()
    with torch.no_grad():
        ref = convnext.encoder_forward(sd, "tiny", img.cpu(), sd_keep=list(scales))
    assert _rel(a, ref) < 1e-4

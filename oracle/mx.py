"""CPU ORACLE (test infrastructure) -- MX-FP8 block quantisation as the C5 frozen-encoder path
uses it (OCP MX: FP8 e4m3fn elements, one E8M0 power-of-two scale per 32 consecutive elements of
a row).  Restates the documented encoding of ``imgcap_mx_quant_rows`` (include/imgcap_abi.h):

  scale exponent sb = clamp(exponent(amax of the block) - 8, >= 1)   (8 = e4m3's max exponent)
                      127 for an all-zero block
  q = e4m3fn(clamp(v * 2^(127 - sb), -448, 448))                    (round to nearest even)
  value = q * 2^(sb - 127)

Used by the fp8-emulating encoder oracle (oracle/convnext.py, numerics="mx") and by
tests/test_mx_gpu.py (bit-exact against the kernel)."""
import torch


def quant(v):
    """fp32 rows [R, K] (K % 32 == 0) -> (q uint8 [R, K] e4m3fn bytes, sb uint8 [R, K/32])."""
    R, Kc = v.shape
    blk = v.float().reshape(R, Kc // 32, 32)
    amax = blk.abs().amax(-1)
    ex = (amax.view(torch.int32) >> 23) & 0xFF
    sb = torch.where(ex == 0, torch.full_like(ex, 127), (ex - 8).clamp(min=1))
    inv = torch.exp2((127 - sb).float()).unsqueeze(-1)
    q = (blk * inv).clamp(-448, 448).to(torch.float8_e4m3fn).view(torch.uint8).reshape(R, Kc)
    return q, sb.to(torch.uint8)


def dequant(q, sb):
    v = q.view(torch.float8_e4m3fn).float()
    e = (sb.to(torch.int32) - 127).float()
    return (v.reshape(q.shape[0], -1, 32) * torch.exp2(e).unsqueeze(-1)).reshape(q.shape)


def qdq(v):
    """Quantise-dequantise along the last dimension (any leading shape)."""
    shp = v.shape
    q, s = quant(v.reshape(-1, shp[-1]))
    return dequant(q, s).reshape(shp)

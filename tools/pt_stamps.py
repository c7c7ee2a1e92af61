"""In-kernel s_memtime stamps of the stream-tile GEMM's k-loop (diagnostic build, GPU box):
    make -C imagecaptioningconvnext_amd/csrc diag && python tools/pt_stamps.py [cfg]
Per iteration of wave 0 (first 64 iterations of every block): wait, barrier, DMA issue, MFMAs,
epilogue / rest; prints median cycles per phase over blocks and iterations, the iteration total,
and the same for the first iteration of each tile."""
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
os.environ["IMGCAP_LIB"] = os.path.join(ROOT, "build", "libimgcap_hip_diag.so")
sys.path.insert(0, ROOT)
import torch  # noqa: E402

from imagecaptioningconvnext_amd import _abi  # noqa: E402
from imagecaptioningconvnext_amd import kernels as K  # noqa: E402

L = _abi.lib()
L.imgcap_debug_stamps.argtypes = [ctypes.c_void_p]
dev = torch.device("cuda:0")
bf = torch.bfloat16
cfg = int(sys.argv[1]) if len(sys.argv) > 1 else 4


def run(M, N, Kd):
    a = torch.randn(M, Kd, device=dev).to(bf)
    b = torch.randn(N, Kd, device=dev).to(bf)
    out = torch.empty(M, N, device=dev, dtype=bf)
    prev = K.gemm_get_pt()
    K.gemm_set_pt(cfg)
    st = torch.zeros(1024 * 64 * 8, device=dev, dtype=torch.int64)  # [block][iteration][phase]
    for _ in range(3):
        K.gemm(a, b, trans_b=True, out=out)
    torch.cuda.synchronize()
    L.imgcap_debug_stamps(st.data_ptr())
    K.gemm(a, b, trans_b=True, out=out)
    torch.cuda.synchronize()
    L.imgcap_debug_stamps(None)
    K.gemm_set_pt(prev)
    s = st.view(1024, 64, 8).cpu().double()
    used = s[:, :, 0] > 0
    names = ["mfma0+reads", "wait", "barrier", "issue/eload", "reads+mfma1", "epi"]
    res = []
    for k in range(6):
        d = (s[:, :, k + 1] - s[:, :, k])[used]
        res.append(d.median().item())
    nxt = (s[:, 1:, 0] - s[:, :-1, 0])[used[:, 1:]]
    print(f"cfg {cfg} M={M} N={N} K={Kd}: " + "  ".join(f"{n} {v:.0f}" for n, v in zip(names, res)) +
          f"  | iteration {nxt.median().item():.0f} cyc (p10 {nxt.quantile(0.1).item():.0f} p90 {nxt.quantile(0.9).item():.0f})",
          flush=True)


shapes = ((12544, 1536, 384), (12544, 384, 1536), (3136, 768, 3072), (4096, 4096, 4096), (3328, 512, 512))
if os.environ.get("IMGCAP_PT_DBG"):
    print(f"IMGCAP_PT_DBG={os.environ['IMGCAP_PT_DBG']} (1: DMA of k-step 0 only, 2: no MFMA, 4: no DMA)")
    shapes = shapes[1:2] + shapes[3:4]
for shape in shapes:
    run(*shape)

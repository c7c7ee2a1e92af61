"""In-kernel s_memtime stamps of the 256x256 GEMM (diagnostic build, GPU box):
    make -C imagecaptioningconvnext_amd/csrc diag && python tools/gemm_stamps.py
Per block: t0 start, t1 first k-step landed, t2 main loop done, t3 first epilogue pass,
t4 epilogue issued, t5 stores drained.  Prints medians (cycles) and the implied clock."""
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


def run(M, N, Kd, pol=1, act=0):
    a = torch.randn(M, Kd, device=dev).to(bf)
    b = torch.randn(N, Kd, device=dev).to(bf)
    out = torch.empty(M, N, device=dev, dtype=bf)
    K.gemm_set_policy(pol)
    nblk = ((M + 255) // 256) * ((N + 255) // 256)
    st = torch.zeros(nblk * 8, device=dev, dtype=torch.int64)
    for _ in range(3):
        K.gemm(a, b, trans_b=True, out=out, act=act)
    torch.cuda.synchronize()
    L.imgcap_debug_stamps(st.data_ptr())
    K.gemm(a, b, trans_b=True, out=out, act=act)
    torch.cuda.synchronize()
    L.imgcap_debug_stamps(None)
    K.gemm_set_policy(-1)
    s = st.view(nblk, 8).cpu().double()
    t0 = s[:, 0]
    d = lambda i, j: (s[:, j] - s[:, i]).median().item()  # noqa: E731
    span = (s[:, 5].max() - t0.min()).item()
    print(f"M={M} N={N} K={Kd} blocks={nblk}: first-tile {d(0, 1):.0f}  loop {d(1, 2):.0f} "
          f"({d(1, 2) / max(1, (Kd + 31) // 32):.0f}/32k)  epi-pass0 {d(2, 3):.0f}  epi {d(2, 4):.0f}  "
          f"drain {d(4, 5):.0f}  block {d(0, 5):.0f}  launch span {span:.0f} cyc;  start skew "
          f"{(t0.max() - t0.min()).item():.0f}")


for shape in ((1568, 1536, 384), (6272, 1536, 384), (6272, 1536, 1536), (4096, 4096, 4096)):
    for pol in (1, 2):
        print(f"policy {pol}: ", end="")
        run(*shape, pol=pol)

"""Stream-tile GEMM ablations by launch time (diagnostic library, GPU box):
    make -C imagecaptioningconvnext_amd/csrc diag && python tools/pt_ablate.py
IMGCAP_PT_DBG bits (gemm_pt.h): 1 every DMA reads k-step 0 (L2-resident operands), 2 no MFMAs,
4 no DMA after the prologue.  Prints us per launch and ns per k-step of the busiest block for each
switch set, config and shape (the numbers are not results: the outputs are wrong by design)."""
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if len(sys.argv) == 1:  # driver: one process per switch set (the library reads them once)
    for d in os.environ.get("DBGS", "0 1 2 4 6").split():
        env = dict(os.environ, IMGCAP_PT_DBG=str(d))
        subprocess.run([sys.executable, "-u", __file__, "child"], env=env, check=True)
    sys.exit(0)
os.environ["IMGCAP_LIB"] = os.path.join(ROOT, "build", "libimgcap_hip_diag.so")
sys.path.insert(0, ROOT)
import torch  # noqa: E402

from imagecaptioningconvnext_amd import kernels as K  # noqa: E402
from tools.microbench import time_launch  # noqa: E402

dev = torch.device("cuda:0")
bf = torch.bfloat16
cfgs = {2: (256, 128), 4: (128, 128), 6: (128, 128)}
row = []
for (M, N, Kd) in ((12544, 384, 1536), (12544, 1536, 384), (4096, 4096, 4096), (3328, 512, 512)):
    a = torch.randn(M, Kd, device=dev).to(bf)
    b = torch.randn(N, Kd, device=dev).to(bf)
    out = torch.empty(M, N, device=dev, dtype=bf)
    for c, (bm, bn) in cfgs.items():
        with K.gemm_pt_mode(c):
            t = time_launch(lambda: K.gemm(a, b, trans_b=True, out=out), reps=20)
        tiles = ((M + bm - 1) // bm) * ((N + bn - 1) // bn)
        steps = -(-tiles // (512 if c == 6 else 256)) * ((Kd + 63) // 64)
        row.append(f"{M}x{N}x{Kd} {bm}x{bn}: {t * 1e6:7.1f} us {t * 1e9 / steps:6.0f} ns/step")
print(f"IMGCAP_PT_DBG={os.environ.get('IMGCAP_PT_DBG')}: " + " | ".join(row), flush=True)

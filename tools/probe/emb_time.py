import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch
from imagecaptioningconvnext_amd import kernels as K
for n, V in ((1632, 9490), (3328, 9490)):
    ids = torch.randint(0, V, (n,), device="cuda")
    d = torch.randn(n, 512, device="cuda").bfloat16()
    t = torch.zeros(V, 512, device="cuda")
    for _ in range(5):
        K.embedding_bwd(ids, d, t)
    torch.cuda.synchronize()

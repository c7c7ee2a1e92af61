"""Which hipBLASLt kernels torch.matmul picks for the train step's GEMM shapes (run under
rocprofv3 --kernel-trace --stats; the kernel names encode the macro tile / wave tiling)."""
import torch

dev = torch.device("cuda:0")
shapes = [(12544, 1536, 384), (12544, 384, 1536), (3136, 3072, 768), (3136, 768, 3072), (3328, 1536, 512),
          (3328, 512, 512), (4096, 4096, 4096)]
for M, N, K in shapes:
    a = torch.randn(M, K, device=dev, dtype=torch.bfloat16)
    b = torch.randn(N, K, device=dev, dtype=torch.bfloat16)
    for _ in range(3):
        c = torch.matmul(a, b.t())
    torch.cuda.synchronize()
    print(M, N, K, flush=True)

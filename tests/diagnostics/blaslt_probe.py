"""Diagnostic (GPU box): run torch.mm (hipBLASLt) once per c4 GEMM shape so that a rocprofv3 kernel
trace shows which library kernel (macro tile, split) it picks for each shape."""
import torch

dev = torch.device("cuda:0")
for name, M, N, K in [("v.qkv", 6368, 2304, 768), ("v.proj", 6368, 768, 3072), ("v.dqkv", 6368, 768, 2304),
                      ("v.fc", 6368, 3072, 768), ("v.out", 6368, 768, 768)]:
    A = torch.randn(M, K, device=dev).half()
    B = torch.randn(N, K, device=dev).half()
    C = torch.empty(M, N, device=dev, dtype=torch.float16)
    for _ in range(3):
        torch.mm(A, B.t(), out=C)
    torch.cuda.synchronize()
    print(name, flush=True)

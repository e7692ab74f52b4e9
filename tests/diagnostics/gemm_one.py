"""Diagnostic (GPU box): a few launches of one GEMM tile on one shape, for rocprofv3 --pmc passes:
    python gemm_one.py M N K tile [reps] [epi]
tile -2 runs torch.mm (hipBLASLt) on the same operands instead, for a counter-by-counter comparison."""
import sys
from pathlib import Path

import torch

sys.path.insert(0, str(Path(__file__).resolve().parents[2]))
from federated_multi_modal_amd import ops  # noqa: E402

M, N, K, tile = (int(x) for x in sys.argv[1:5])
reps = int(sys.argv[5]) if len(sys.argv) > 5 else 5
epi = int(sys.argv[6]) if len(sys.argv) > 6 else ops.EPI_NONE
dev = torch.device("cuda:0")
torch.manual_seed(0)
A = torch.randn(M, K, device=dev).half()
B = (torch.randn(N, K, device=dev) * K ** -0.5).half()
C = torch.empty(M, N, device=dev, dtype=torch.float16)
bias = (torch.randn(N, device=dev) * 0.1).half() if epi == ops.EPI_BIAS else None
for _ in range(reps):
    if tile == -2:
        torch.mm(A, B.t(), out=C)
    else:
        ops.gemm_nt(A, B, C=C, bias=bias, epilogue=epi, tile=tile)
torch.cuda.synchronize()
print("ok", M, N, K, tile)

"""Diagnostic (GPU box): run ONE mf_gemm_nt configuration `reps` times (for rocprofv3 PMC passes).
    python gemm_one.py M N K epilogue tile [reps]"""
import sys
from pathlib import Path

import torch

sys.path.insert(0, str(Path(__file__).resolve().parents[2]))
from federated_multi_modal_amd import ops  # noqa: E402


def main():
    M, N, K, epi, tile = (int(x) for x in sys.argv[1:6])
    reps = int(sys.argv[6]) if len(sys.argv) > 6 else 20
    dev = torch.device("cuda:0")
    torch.manual_seed(0)
    A = torch.randn(M, K, device=dev).half()
    B = (torch.randn(N, K, device=dev) * K ** -0.5).half()
    kw = dict(C=torch.empty(M, N, device=dev, dtype=torch.float16), epilogue=epi, tile=tile)
    if epi in (ops.EPI_BIAS, ops.EPI_BIAS_RESID, ops.EPI_BIAS_GELU):
        kw["bias"] = torch.randn(N, device=dev).half() * 0.1
    if epi in (ops.EPI_BIAS_RESID, ops.EPI_DGELU):
        kw["aux_in"] = torch.randn(M, N, device=dev).half()
    if epi == ops.EPI_BIAS_GELU:
        kw["aux_out"] = torch.empty(M, N, device=dev, dtype=torch.float16)
    for _ in range(reps):
        ops.gemm_nt(A, B, **kw)
    torch.cuda.synchronize()
    print("done", M, N, K, epi, tile)


if __name__ == "__main__":
    main()

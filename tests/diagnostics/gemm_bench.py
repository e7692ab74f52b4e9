"""Diagnostic (GPU box): time every mf_gemm_nt tile configuration on the MaPLe step's GEMM shapes,
check each against a torch fp32 matmul, print TFLOP/s.  Usage: python gemm_bench.py [tiles]"""
import sys
from pathlib import Path

import torch

sys.path.insert(0, str(Path(__file__).resolve().parents[2]))
from federated_multi_modal_amd import ops  # noqa: E402

SHAPES = [  # (name, M, N, K, epilogue)
    ("v.qkv", 6368, 2304, 768, ops.EPI_BIAS), ("v.out", 6368, 768, 768, ops.EPI_BIAS_RESID),
    ("v.fc", 6368, 3072, 768, ops.EPI_BIAS_GELU), ("v.proj", 6368, 768, 3072, ops.EPI_BIAS_RESID),
    ("v.dfc", 6368, 3072, 768, ops.EPI_DGELU), ("v.dh", 6368, 768, 3072, ops.EPI_NONE),
    ("v.dqkv", 6368, 768, 2304, ops.EPI_NONE),
    ("t.qkv", 2926, 1536, 512, ops.EPI_BIAS), ("t.fc", 2926, 2048, 512, ops.EPI_BIAS_GELU),
    ("t.proj", 2926, 512, 2048, ops.EPI_BIAS_RESID), ("t.dh", 2926, 512, 2048, ops.EPI_NONE),
    ("v.dW_fc", 3072, 768, 6400, ops.EPI_NONE),
]


def main():
    tiles = [int(t) for t in sys.argv[1].split(",")] if len(sys.argv) > 1 else list(range(1, 10))
    dev = torch.device("cuda:0")
    torch.manual_seed(0)
    print(f"{'shape':10s} " + " ".join(f"{'t' + str(t):>8s}" for t in tiles), flush=True)
    for name, M, N, K, epi in SHAPES:
        A = torch.randn(M, K, device=dev).half()
        B = (torch.randn(N, K, device=dev) * K ** -0.5).half()
        bias = torch.randn(N, device=dev).half() * 0.1
        aux = torch.randn(M, N, device=dev).half()
        auxo = torch.empty(M, N, device=dev, dtype=torch.float16)
        C = torch.empty(M, N, device=dev, dtype=torch.float16)
        ref = (A.float() @ B.float().t())
        res = []
        for t in tiles:
            kw = dict(C=C, epilogue=epi, tile=t)
            if epi in (ops.EPI_BIAS, ops.EPI_BIAS_RESID, ops.EPI_BIAS_GELU):
                kw["bias"] = bias
            if epi in (ops.EPI_BIAS_RESID, ops.EPI_DGELU):
                kw["aux_in"] = aux
            if epi == ops.EPI_BIAS_GELU:
                kw["aux_out"] = auxo
            try:
                ops.gemm_nt(A, B, **kw)
            except Exception as e:  # noqa: BLE001
                res.append("   err")
                continue
            # correctness of the raw product through EPI_NONE
            C0 = ops.gemm_nt(A, B, epilogue=ops.EPI_NONE, tile=t)
            err = (C0.float() - ref).abs().max().item()
            ok = err < 2e-2 * ref.abs().max().item()
            torch.cuda.synchronize()
            s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            for _ in range(3):
                ops.gemm_nt(A, B, **kw)
            s.record()
            for _ in range(20):
                ops.gemm_nt(A, B, **kw)
            e.record()
            torch.cuda.synchronize()
            us = s.elapsed_time(e) / 20 * 1e3
            tf = 2 * M * N * K / us / 1e6
            res.append(f"{tf:7.0f}{'' if ok else '!'}")
        print(f"{name:10s} " + " ".join(f"{r:>8s}" for r in res), flush=True)


if __name__ == "__main__":
    main()

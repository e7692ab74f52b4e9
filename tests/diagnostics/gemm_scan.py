"""Diagnostic (GPU box): TFLOP/s of mf_gemm_nt tiles on calibration shapes (square 4k/8k, and the
vision QKV shape scaled in M and K) on random operands, vs hipBLASLt (torch.mm).
    python gemm_scan.py tiles"""
import sys
from pathlib import Path

import torch

sys.path.insert(0, str(Path(__file__).resolve().parents[2]))
from federated_multi_modal_amd import ops  # noqa: E402
from gemm_bench import timeit  # noqa: E402

SHAPES = [(4096, 4096, 4096), (8192, 8192, 8192), (6368, 2304, 768), (12736, 2304, 768), (3184, 2304, 768),
          (6368, 2304, 3072), (6368, 2304, 192), (6368, 768, 768), (6368, 768, 3072)]


def main():
    tiles = [int(t) for t in sys.argv[1].split(",")]
    dev = torch.device("cuda:0")
    print(f"{'M,N,K':18s} {'blasLt':>7s} " + " ".join(f"{'t' + str(t):>7s}" for t in tiles), flush=True)
    for M, N, K in SHAPES:
        A = torch.rand(M, K, device=dev).sub(0.5).half()
        B = torch.rand(N, K, device=dev).sub(0.5).half()
        C = torch.empty(M, N, device=dev, dtype=torch.float16)
        fl = 2 * M * N * K
        ub = timeit(lambda: torch.mm(A, B.t(), out=C), 10)
        res = [f"{fl / timeit(lambda: ops.gemm_nt(A, B, C=C, tile=t), 10) / 1e6:7.0f}" for t in tiles]
        print(f"{str((M, N, K)):18s} {fl / ub / 1e6:7.0f} " + " ".join(res), flush=True)


if __name__ == "__main__":
    main()

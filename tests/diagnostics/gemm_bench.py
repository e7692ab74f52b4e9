"""Diagnostic (GPU box): time mf_gemm_nt on the MaPLe step's GEMM shapes (c4: vision M = 32*199,
text M = 38*77), against hipBLASLt (torch.mm, plain product, no epilogue) as a yardstick, and check
each tile configuration against a torch fp32 matmul.  Prints TFLOP/s.

    python gemm_bench.py [tiles] [big]  tiles: comma list of mf_gemm_nt tile ids (0 = heuristic);
                                        big: square 4096^3 / 8192^3 products instead of the step's shapes
                                        (the guide's long-K yardstick for the main loop alone);
                                        c5: the K = 1000 text tower's products (77 000 rows)
                                        c3: the B = 4 / K = 10 client's products (796 / 770 rows)
                                        eval: a 100-image test batch's forward products (19 900 rows)
                                        eval4: the eval engine's launches at EVAL_GROUP 4 (400 images, 79 600
                                        rows); in both eval sets c_fc stores no pre-activation (forward-only engine)

GEMM_BENCH_REPS (default 20) sets the launches per timed hipGraph (300 holds each kernel ~10-30 ms,
long enough for the clock to settle to the sustained-load level the engine sees).

A "!" marks a tile whose plain product misses the fp32 reference, "~" one whose output (with the
shape's epilogue) is not bit-identical to the first listed tile's.
"""
import os
import sys
from pathlib import Path

import torch

sys.path.insert(0, str(Path(__file__).resolve().parents[2]))
from federated_multi_modal_amd import ops  # noqa: E402

SHAPES = [  # (name, M, N, K, epilogue, calls per c4 step)
    ("v.qkv", 6368, 2304, 768, ops.EPI_BIAS, 12), ("v.out", 6368, 768, 768, ops.EPI_BIAS_RESID, 12),
    ("v.fc", 6368, 3072, 768, ops.EPI_BIAS_GELU, 12), ("v.proj", 6368, 768, 3072, ops.EPI_BIAS_RESID, 12),
    ("v.dfc", 6368, 3072, 768, ops.EPI_DGELU, 12), ("v.dh", 6368, 768, 3072, ops.EPI_NONE, 12),
    ("v.do", 6368, 768, 768, ops.EPI_NONE, 12), ("v.dqkv", 6368, 768, 2304, ops.EPI_NONE, 12),
    ("t.qkv", 2926, 1536, 512, ops.EPI_BIAS, 12), ("t.out", 2926, 512, 512, ops.EPI_BIAS_RESID, 12),
    ("t.fc", 2926, 2048, 512, ops.EPI_BIAS_GELU, 12), ("t.proj", 2926, 512, 2048, ops.EPI_BIAS_RESID, 12),
    ("t.dfc", 2926, 2048, 512, ops.EPI_DGELU, 12), ("t.dh", 2926, 512, 2048, ops.EPI_NONE, 12),
    ("t.do", 2926, 512, 512, ops.EPI_NONE, 12), ("t.dqkv", 2926, 512, 1536, ops.EPI_NONE, 12),
    ("v.dW_fc", 3072, 768, 6400, ops.EPI_NONE, 1), ("v.dW_qkv", 2304, 768, 6400, ops.EPI_NONE, 1),
]


ROUNDS = 3


def timeit(fn, reps=int(os.environ.get("GEMM_BENCH_REPS", "20"))):
    """Kernel time per call: `reps` calls captured in one hipGraph and replayed (no host overhead)."""
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        for _ in range(reps):
            fn()
    g.replay()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(3):
        g.replay()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / (3 * reps) * 1e3  # us


def main():
    tiles = [int(t) for t in sys.argv[1].split(",")] if len(sys.argv) > 1 else [0]
    dev = torch.device("cuda:0")
    torch.manual_seed(0)
    print(f"{'shape':10s} {'blasLt':>8s} " + " ".join(f"{'t' + str(t):>8s}" for t in tiles) + "   (TFLOP/s; "
          "last col: us/step at heuristic tile)", flush=True)
    tot_us, tot_blas = 0.0, 0.0
    shapes = SHAPES
    if len(sys.argv) > 2 and sys.argv[2] == "c5":  # the K = 1000 text tower (77 000 rows)
        shapes = [("c5.qkv", 77000, 1536, 512, ops.EPI_BIAS, 12), ("c5.out", 77000, 512, 512, ops.EPI_BIAS_RESID, 12),
                  ("c5.fc", 77000, 2048, 512, ops.EPI_BIAS_GELU, 12),
                  ("c5.proj", 77000, 512, 2048, ops.EPI_BIAS_RESID, 12),
                  ("c5.dfc", 77000, 2048, 512, ops.EPI_DGELU, 12), ("c5.dh", 77000, 512, 2048, ops.EPI_NONE, 12),
                  ("c5.do", 77000, 512, 512, ops.EPI_NONE, 12), ("c5.dqkv", 77000, 512, 1536, ops.EPI_NONE, 12)]
    if len(sys.argv) > 2 and sys.argv[2] == "c3":  # C3 / C2 clients: B = 4 images (4 x 199 rows), K = 10 classes
        shapes = [("c3v.qkv", 796, 2304, 768, ops.EPI_BIAS, 12), ("c3v.out", 796, 768, 768, ops.EPI_BIAS_RESID, 12),
                  ("c3v.fc", 796, 3072, 768, ops.EPI_BIAS_GELU, 12), ("c3v.proj", 796, 768, 3072, ops.EPI_BIAS_RESID, 12),
                  ("c3v.dfc", 796, 3072, 768, ops.EPI_DGELU, 12), ("c3v.dh", 796, 768, 3072, ops.EPI_NONE, 12),
                  ("c3v.do", 796, 768, 768, ops.EPI_NONE, 12), ("c3v.dqkv", 796, 768, 2304, ops.EPI_NONE, 12),
                  ("c3t.qkv", 770, 1536, 512, ops.EPI_BIAS, 12), ("c3t.out", 770, 512, 512, ops.EPI_BIAS_RESID, 12),
                  ("c3t.fc", 770, 2048, 512, ops.EPI_BIAS_GELU, 12), ("c3t.proj", 770, 512, 2048, ops.EPI_BIAS_RESID, 12),
                  ("c3t.dfc", 770, 2048, 512, ops.EPI_DGELU, 12), ("c3t.dh", 770, 512, 2048, ops.EPI_NONE, 12),
                  ("c3t.do", 770, 512, 512, ops.EPI_NONE, 12), ("c3t.dqkv", 770, 512, 1536, ops.EPI_NONE, 12)]
    evalm = {"eval": 19900, "eval4": 79600}.get(sys.argv[2] if len(sys.argv) > 2 else "")
    if evalm:  # test() batches: 100 (or 4 x 100) images, forward only
        shapes = [("ev.qkv", evalm, 2304, 768, ops.EPI_BIAS, 12), ("ev.out", evalm, 768, 768, ops.EPI_BIAS_RESID, 12),
                  ("ev.fc", evalm, 3072, 768, ops.EPI_BIAS_GELU, 12), ("ev.proj", evalm, 768, 3072, ops.EPI_BIAS_RESID, 12)]
    if len(sys.argv) > 2 and sys.argv[2] == "big":
        shapes = [("4096^3", 4096, 4096, 4096, ops.EPI_NONE, 1), ("8192^3", 8192, 8192, 8192, ops.EPI_NONE, 1),
                  ("v.fc K4k", 6368, 3072, 4096, ops.EPI_NONE, 1), ("v.qkv K3k", 6368, 2304, 3072, ops.EPI_NONE, 1)]
    for name, M, N, K, epi, calls in shapes:
        A = torch.randn(M, K, device=dev).half()
        B = (torch.randn(N, K, device=dev) * K ** -0.5).half()
        bias = torch.randn(N, device=dev).half() * 0.1
        aux = torch.randn(M, N, device=dev).half()
        auxo = torch.empty(M, N, device=dev, dtype=torch.float16)
        C = torch.empty(M, N, device=dev, dtype=torch.float16)
        ref = (A.float() @ B.float().t())
        fl = 2 * M * N * K
        ub = ub0 = timeit(lambda: torch.mm(A, B.t(), out=C))
        tot_blas += ub * calls
        first = None
        marks, fns = {}, {}
        for t in tiles:
            kw = dict(C=C, epilogue=epi, tile=t)
            if epi in (ops.EPI_BIAS, ops.EPI_BIAS_RESID, ops.EPI_BIAS_GELU):
                kw["bias"] = bias
            if epi in (ops.EPI_BIAS_RESID, ops.EPI_DGELU):
                kw["aux_in"] = aux
            if epi == ops.EPI_BIAS_GELU and not evalm:
                kw["aux_out"] = auxo
            try:
                ops.gemm_nt(A, B, **kw)
                C0 = ops.gemm_nt(A, B, epilogue=ops.EPI_NONE, tile=t)
            except Exception:  # noqa: BLE001
                marks[t] = None
                continue
            err = (C0.float() - ref).abs().max().item()
            ok = err < 2e-2 * ref.abs().max().item()
            Ce = ops.gemm_nt(A, B, **{**kw, "C": torch.empty_like(C)})
            if first is None:
                first = Ce
            same = torch.equal(Ce, first)  # bit-identical to the first tile's output (same epilogue)
            marks[t] = ('' if ok else '!') + ('' if same else '~')
            fns[t] = (lambda kw=kw: ops.gemm_nt(A, B, **kw))
        # every tile (and the library) timed ROUNDS times round-robin, best time kept: the first-measured column
        # no longer pays the clock / cache warm-up of the shape (r03 note in DESIGN.md §6)
        best = {t: float("inf") for t in fns}
        for _ in range(ROUNDS):
            ub = min(ub, timeit(lambda: torch.mm(A, B.t(), out=C)))
            for t, fn in fns.items():
                best[t] = min(best[t], timeit(fn))
        res = []
        for t in tiles:
            if marks.get(t) is None:
                res.append("   err")
                continue
            if t == tiles[0]:
                tot_us += best[t] * calls
            res.append(f"{fl / best[t] / 1e6:7.0f}{marks[t]}")
        tot_blas += ub * calls - ub0 * calls
        print(f"{name:10s} {fl / ub / 1e6:8.0f} " + " ".join(f"{r:>8s}" for r in res), flush=True)
    print(f"sum over a c4 step: ours (tile {tiles[0]}) {tot_us / 1e3:.2f} ms, hipBLASLt plain {tot_blas / 1e3:.2f} ms")
    if shapes is not SHAPES:
        return  # the sum line above is then over the listed shapes at the listed call counts
    # K-major operand forms (dX = dY . W with W read as [out][in]; dW = dY^T X read in place)
    print("K-major forms (TFLOP/s): NN = B K-major, TN = both K-major", flush=True)
    for name, M, N, K, epi, ak, bk in [("v.dfc NN", 6368, 3072, 768, ops.EPI_DGELU, False, True),
                                       ("v.dh NN", 6368, 768, 3072, ops.EPI_NONE, False, True),
                                       ("v.dqkv NN", 6368, 768, 2304, ops.EPI_NONE, False, True),
                                       ("t.dh NN", 2926, 512, 2048, ops.EPI_NONE, False, True),
                                       ("v.dW_fc TN", 3072, 768, 6368, ops.EPI_NONE, True, True),
                                       ("v.dW_pr TN", 768, 3072, 6368, ops.EPI_NONE, True, True)]:
        A = (torch.randn(K, M, device=dev) if ak else torch.randn(M, K, device=dev)).half()
        B = ((torch.randn(K, N, device=dev) if bk else torch.randn(N, K, device=dev)) * K ** -0.5).half()
        aux = torch.randn(M, N, device=dev).half()
        C = torch.empty(M, N, device=dev, dtype=torch.float16)
        kw = dict(C=C, epilogue=epi, a_kmajor=ak, b_kmajor=bk)
        if epi == ops.EPI_DGELU:
            kw["aux_in"] = aux
        fl = 2 * M * N * K
        res = []
        for t in (1, 2, 3):
            us = timeit(lambda: ops.gemm(A, B, tile=t, **kw))
            res.append(f"t{t} {fl / us / 1e6:6.0f}")
        us0 = timeit(lambda: ops.gemm(A, B, tile=0, **kw))
        print(f"{name:12s} " + "  ".join(res) + f"  auto {fl / us0 / 1e6:6.0f}", flush=True)


if __name__ == "__main__":
    main()

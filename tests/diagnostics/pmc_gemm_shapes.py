"""Per-kernel / per-grid GEMM traffic from the PMC passes of scripts/gpu_pmc.sh (no GPU needed).

    python pmc_gemm_shapes.py FETCH_CSV WRITE_CSV [OUT.txt]

FETCH_SIZE is doubled (gfx950 correction, MI355X_MICROARCH.md HBM section), WRITE_SIZE taken as is; both are
memory-side L2 counters (reads served by the Infinity Cache count).  The c4 shape of each launch is named
from its tile and grid (the dispatch table of gemm.hip at c4), with its algorithmic read bytes: A and B once,
plus the epilogue's aux operand (residual or QuickGELU pre-activation) where it reads one."""
import csv
import re
import sys
from collections import defaultdict

# (kernel, workgroups) -> (product, M, N, K, aux_read) at c4 (vision M = 6368, text M = 2926)
C4 = {
    ("gemm8s_kernel<1>", 225): ("vision in_proj fwd", 6368, 2304, 768, False),
    ("gemm_nt_kernel<160,128,2,2,2,3,false,false>", 960): ("vision c_fc fwd (+QuickGELU, pre-activation out)", 6368, 3072, 768, False),
    ("gemm_nt_kernel<96,128,2,2,2,2,false,false>", 402): ("vision c_proj fwd / c_fc dX (+residual)", 6368, 768, 3072, True),
    ("gemm_nt_kernel<160,64,2,2,2,2,false,false>", 480): ("vision out_proj fwd (+residual)", 6368, 768, 768, True),
    ("gemm_nt_kernel<96,128,2,2,2,0,false,false>", 402): ("vision in_proj dX", 6368, 768, 2304, False),
    ("gemm_nt_kernel<160,128,2,2,2,4,false,false>", 960): ("vision c_proj dX (x QuickGELU')", 6368, 3072, 768, True),
    ("gemm_nt_kernel<160,64,2,2,2,0,false,false>", 480): ("vision out_proj dX", 6368, 768, 768, False),
}


def load(path, counter):
    acc, ids = defaultdict(float), defaultdict(set)
    with open(path) as f:
        for row in csv.DictReader(f):
            if row["Counter_Name"] != counter or "gemm" not in row["Kernel_Name"]:
                continue
            m = re.search(r"(gemm\w*kernel)<([^>]*)>", row["Kernel_Name"])
            name = m.group(1) + "<" + m.group(2).replace(" ", "") + ">" if m else row["Kernel_Name"][:60]
            wgs = int(row["Grid_Size"]) // max(int(row["Workgroup_Size"]), 1)
            acc[(name, wgs)] += float(row["Counter_Value"])
            ids[(name, wgs)].add(row["Dispatch_Id"])
    return {k: (acc[k] / len(ids[k]), len(ids[k])) for k in acc}


def main():
    f = load(sys.argv[1], "FETCH_SIZE")
    w = load(sys.argv[2], "WRITE_SIZE")
    lines = [f"{'kernel':46s} {'wgs':>5s} {'n':>4s} {'read MB':>8s} {'write MB':>8s}  c4 product: algorithmic read MB, read / algorithmic"]
    for k, (v, n) in sorted(f.items(), key=lambda kv: -kv[1][0] * kv[1][1]):
        rd, wr = 2 * v * 1024 / 1e6, w.get(k, (0.0, 0))[0] * 1024 / 1e6
        line = f"{k[0][:46]:46s} {k[1]:5d} {n:4d} {rd:8.1f} {wr:8.1f}"
        if k in C4:
            what, M, N, K, aux = C4[k]
            alg = (2 * M * K + 2 * N * K + (2 * M * N if aux else 0)) / 1e6
            line += f"  {what}: {alg:.1f}, {rd / alg:.2f}x"
        lines.append(line)
    text = "\n".join(lines[:30])
    print(text)
    if len(sys.argv) > 3:
        open(sys.argv[3], "w").write(text + "\n")


if __name__ == "__main__":
    main()

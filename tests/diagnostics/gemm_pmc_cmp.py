"""Counter-by-counter comparison of GEMM launches from scripts/gemm_pmc_probe.sh (no GPU needed).

    python tests/diagnostics/gemm_pmc_cmp.py gpurun_out/gpmc [OUT.txt]

For every config directory pair <tag>_p1/_p2/_p3 it sums each counter over the GEMM dispatches (hand-written
gemm* kernels or hipBLASLt's Cijk_*) and prints per-dispatch values plus the derived fractions: MFMA busy per SIMD
over GRBM_GUI_ACTIVE (SQ_VALU_MFMA_BUSY_CYCLES is summed over the 1 024 SIMDs, GRBM_GUI_ACTIVE over the 8 XCDs),
waves' wait / issue-stall / LDS-issue-stall shares of their cycles, LDS bank conflicts per LDS-active cycle."""
import csv
import sys
from collections import defaultdict
from pathlib import Path


def load(d):
    vals, disp = defaultdict(float), set()
    for f in Path(d).glob("*counter_collection.csv"):
        with open(f) as fh:
            for row in csv.DictReader(fh):
                name = row.get("Kernel_Name", "")
                if "gemm" not in name and "Cijk_" not in name:
                    continue
                vals[row["Counter_Name"]] += float(row["Counter_Value"])
                disp.add(row.get("Dispatch_Id"))
    return vals, len(disp)


def main():
    root = Path(sys.argv[1])
    tags = sorted({p.name.rsplit("_p", 1)[0] for p in root.iterdir() if p.is_dir() and "_p" in p.name})
    lines = []
    for tag in tags:
        tot, n = {}, 0
        for p in (1, 2, 3):
            v, k = load(root / f"{tag}_p{p}")
            tot.update(v)
            n = max(n, k)
        if not n:
            continue
        per = {c: x / n for c, x in tot.items()}
        lines.append(f"== {tag}: {n} dispatches")
        for c in sorted(per):
            lines.append(f"   {c:28s} {per[c]:16.0f}")
        g = per.get("GRBM_GUI_ACTIVE", 0.0)
        if g:
            lines.append(f"   mfma_busy_per_simd        {per.get('SQ_VALU_MFMA_BUSY_CYCLES', 0) / 1024 / (g / 8):.3f}")
        w = per.get("SQ_WAVE_CYCLES", 0.0)
        if w:
            for c in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_WAIT_INST_LDS", "SQ_ACTIVE_INST_ANY", "SQ_ACTIVE_INST_LDS",
                      "SQ_ACTIVE_INST_VMEM", "SQ_ACTIVE_INST_VALU", "SQ_ACTIVE_INST_SCA", "SQ_INST_CYCLES_VMEM"):
                if c in per:
                    lines.append(f"   {c + ' / wave cycles':40s} {per[c] / w:.3f}")
        if per.get("SQ_LDS_IDX_ACTIVE"):
            lines.append(f"   lds bank conflict / lds active  {per.get('SQ_LDS_BANK_CONFLICT', 0) / per['SQ_LDS_IDX_ACTIVE']:.3f}")
    text = "\n".join(lines)
    print(text)
    if len(sys.argv) > 2:
        Path(sys.argv[2]).write_text(text + "\n")


if __name__ == "__main__":
    main()

"""Summarise the attention PMC passes of scripts/attn_pmc.sh per kernel and launch shape (no GPU needed).

    python attn_pmc_summary.py OUT.json DIR1 DIR2 ...   (each DIR holds one pass's *counter_collection.csv)

Per (kernel, grid size): the per-launch average of every counter collected, and derived figures:
  read_bytes / write_bytes   FETCH_SIZE x 2 (the gfx950 correction, MI355X_MICROARCH.md HBM section) and
                             WRITE_SIZE, in bytes; memory-side L2 counters, so Infinity Cache hits count
  algorithmic_bytes          Q, K, V (+ O, dO) read and O (dQ, dK, dV) written once, LSE 4 B per row-head
  mfma_busy_frac             SQ_VALU_MFMA_BUSY_CYCLES / (1024 SIMDs x GRBM_GUI_ACTIVE / 8 XCDs)
  valu_active_frac / lds_active_frac   SQ_ACTIVE_INST_VALU / SQ_ACTIVE_INST_LDS over SQ_WAVE_CYCLES
  lds_bank_conflict_frac     SQ_LDS_BANK_CONFLICT over SQ_LDS_IDX_ACTIVE
"""
import csv
import glob
import json
import re
import sys
from collections import defaultdict

SHAPES = {  # launches of tests/diagnostics/attn_pmc_run.py: rows x heads -> (N, L, H)
    "vision": (32, 199, 12), "text": (38, 77, 8)}


def short(name: str) -> str:
    d = re.search(r"((?:qkv_)?attn_\w+?_kernel)<([^>]*)>", name)  # demangled
    if d:
        return d.group(1) + "<" + d.group(2).replace(" ", "") + ">"
    m = re.search(r"((?:qkv_)?attn_\w+?_kernel)I(.*?)EEEv", name)  # mangled
    if not m:
        return name[:60]
    args = re.findall(r"Li(\d+)|Lb(\d)", m.group(2))
    return m.group(1) + "<" + ",".join(a or ("true" if b == "1" else "false") for a, b in args) + ">"


def main():
    out = sys.argv[1]
    acc = defaultdict(lambda: defaultdict(float))  # (kernel, grid) -> counter -> sum
    disp = defaultdict(lambda: defaultdict(set))   # (kernel, grid) -> counter -> dispatch ids
    for d in sys.argv[2:]:
        for path in glob.glob(f"{d}/**/*counter_collection.csv", recursive=True):
            with open(path) as f:
                for row in csv.DictReader(f):
                    name = row.get("Kernel_Name", "")
                    if "attn_" not in name:
                        continue
                    key = (short(name), row.get("Grid_Size", "?"))
                    c = row["Counter_Name"]
                    acc[key][c] += float(row["Counter_Value"])
                    disp[key][c].add(row.get("Dispatch_Id") or row.get("Correlation_Id"))
    res = {}
    for (k, grid), cs in sorted(acc.items()):
        per = {c: v / max(len(disp[(k, grid)][c]), 1) for c, v in cs.items()}
        r = {"grid_threads": grid, "launches": max(len(s) for s in disp[(k, grid)].values()), "counters": per}
        if "FETCH_SIZE" in per:
            r["read_bytes"] = 2 * per["FETCH_SIZE"] * 1024
        if "WRITE_SIZE" in per:
            r["write_bytes"] = per["WRITE_SIZE"] * 1024
        if per.get("GRBM_GUI_ACTIVE") and "SQ_VALU_MFMA_BUSY_CYCLES" in per:
            r["mfma_busy_frac"] = per["SQ_VALU_MFMA_BUSY_CYCLES"] / 1024 / (per["GRBM_GUI_ACTIVE"] / 8)
        if per.get("SQ_WAVE_CYCLES"):
            for c, n in (("SQ_ACTIVE_INST_VALU", "valu_active_frac"), ("SQ_ACTIVE_INST_LDS", "lds_active_frac"),
                         ("SQ_WAIT_INST_LDS", "lds_wait_frac"), ("SQ_WAIT_ANY", "wait_any_frac")):
                if c in per:
                    r[n] = per[c] / per["SQ_WAVE_CYCLES"]
        if per.get("SQ_LDS_IDX_ACTIVE") and "SQ_LDS_BANK_CONFLICT" in per:
            r["lds_bank_conflict_frac"] = per["SQ_LDS_BANK_CONFLICT"] / per["SQ_LDS_IDX_ACTIVE"]
        tower = "vision" if ("208" in k or "224" in k) else ("text" if ("80" in k or "96" in k) else None)
        if tower:
            N, L, H = SHAPES[tower]
            per_row = (2 * 8 * 64 + 4) if "bwd" in k else (2 * 4 * 64 + 4)
            r["tower"] = tower
            r["algorithmic_bytes"] = N * H * L * per_row
            if k.startswith("qkv_attn"):  # x and W read once, qkv + O written (fp16), LSE (fp32)
                D = 64 * H
                r["algorithmic_bytes"] = 2 * N * L * D + 2 * 3 * D * D + 2 * N * L * 4 * D + 4 * N * H * L
            if "read_bytes" in r and "write_bytes" in r:
                r["traffic_over_algorithmic"] = (r["read_bytes"] + r["write_bytes"]) / r["algorithmic_bytes"]
        res[f"{k} grid={grid}"] = r
    json.dump(res, open(out, "w"), indent=1)
    for k, r in res.items():
        print(k, {x: (round(v, 4) if isinstance(v, float) else v) for x, v in r.items() if x != "counters"})


if __name__ == "__main__":
    main()

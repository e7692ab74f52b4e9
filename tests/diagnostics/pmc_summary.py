"""Summarise rocprofv3 --pmc counter CSVs per kernel family (GPU-box diagnostics, no GPU needed).

    python pmc_summary.py OUT.json fetch=DIR/..._counter_collection.csv write=DIR/..._counter_collection.csv \
        [mfma=DIR/..._counter_collection.csv]

HBM bytes follow MI355X_MICROARCH.md §HBM: FETCH_SIZE (KiB) counts exactly half of a wide coalesced
streaming read's bytes on gfx950 -> doubled; WRITE_SIZE (KiB) is exact for 16-B stores.  Both are
memory-side (TCC EA) counters: reads served by the Infinity Cache are counted, L2 hits are not."""
import csv
import json
import sys
from collections import defaultdict

FAMILIES = [("gemm", "gemm"), ("attention", "attn_"), ("layernorm", "ln_"), ("transpose", "transpose"),
            ("optim", "sgd")]


def family(name):
    for f, key in FAMILIES:
        if key in name:
            return f
    return "other"


def load(path, counter):
    per = defaultdict(lambda: [0.0, 0])  # family -> [sum, dispatches]
    seen = set()
    with open(path) as f:
        for row in csv.DictReader(f):
            if row.get("Counter_Name") != counter:
                continue
            d = row.get("Dispatch_Id") or row.get("Correlation_Id")
            fam = family(row.get("Kernel_Name", ""))
            per[fam][0] += float(row["Counter_Value"])
            if (d, counter) not in seen:
                seen.add((d, counter))
                per[fam][1] += 1
    return per


def main():
    out = sys.argv[1]
    args = dict(a.split("=", 1) for a in sys.argv[2:])
    res = {}
    if "fetch" in args:
        for fam, (v, n) in load(args["fetch"], "FETCH_SIZE").items():
            res.setdefault(fam, {})["read_bytes_per_launch"] = 2 * v * 1024 / max(n, 1)
            res[fam]["launches"] = n
    if "write" in args:
        for fam, (v, n) in load(args["write"], "WRITE_SIZE").items():
            res.setdefault(fam, {})["write_bytes_per_launch"] = v * 1024 / max(n, 1)
    if "mfma" in args:
        busy = load(args["mfma"], "SQ_VALU_MFMA_BUSY_CYCLES")
        gui = load(args["mfma"], "GRBM_GUI_ACTIVE")
        for fam in busy:
            # MFMA busy cycles are summed over all SIMDs (1024 on MI355X); GRBM_GUI_ACTIVE over 8 XCDs
            b, _ = busy[fam]
            g, _ = gui.get(fam, (0.0, 0))
            if g:
                res.setdefault(fam, {})["mfma_busy_frac"] = b / 1024 / (g / 8)
    for fam, r in res.items():
        if "read_bytes_per_launch" in r and "write_bytes_per_launch" in r:
            r["hbm_bytes_per_launch"] = r["read_bytes_per_launch"] + r["write_bytes_per_launch"]
    json.dump(res, open(out, "w"), indent=1)
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()

"""GEMM-family HBM traffic against algorithmic bytes, over exactly the launches bench.py's roofline probes.

    # on the GPU box, one rocprofv3 --pmc pass per counter over the same command (scripts/gpu.sh pmc_gemm):
    python tests/diagnostics/gemm_traffic.py run PROBE.json [c4]
    # no GPU needed:
    python tests/diagnostics/gemm_traffic.py summarize PROBE.json FETCH_CSV WRITE_CSV OUT.json

`run` builds the bench's engine, takes one warm eager step, then runs bench.py's probe (two eager training
steps, towers serialised on one stream, HIP events around every GEMM launch) and writes every probed launch
in launch order: (M, N, K, epilogue), duration, FLOPs and algorithmic bytes (ops._gemm_bytes: A and B once,
C once at its element size, the epilogue's aux operand once).  The probed GEMMs are the last GEMM-family
dispatches of the process, so `summarize` pairs the last n GEMM dispatches of the PMC CSVs (Dispatch_Id
order; a split-K launch's reduce pass is charged to it) with the n probed launches one to one.  Traffic per
launch = FETCH_SIZE x 2 (the gfx950 correction, MI355X_MICROARCH.md §HBM) + WRITE_SIZE, in bytes; both are
memory-side L2 counters, so reads served by the Infinity Cache count too (an upper bound on HBM bytes).
OUT.json holds the totals bench.py's `roofline.traffic` reads and the per-shape table."""
import csv
import json
import sys
from collections import defaultdict
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[2]))

GEMM_KEYS = ("gemm", "Cijk_")   # hand-written GEMM kernels; hipBLASLt's (when its A/B route is on)
REDUCE_KEY = "splitk_reduce"    # the split-K combine pass: charged to the GEMM launch before it


def run(out, config="c4"):
    import torch
    import bench
    from federated_multi_modal_amd import ops
    from federated_multi_modal_amd import synthetic as syn
    from federated_multi_modal_amd.engine import EngineConfig, MapleEngine
    J, K, B, _ = bench.CONFIGS[config]
    dev = torch.device("cuda:0")
    e = MapleEngine(EngineConfig(batch=B, classnames=syn.synthetic_classnames(K, 0), prompt_depth=J, seed=0),
                    device=dev)
    e.set_lr(0.0026)
    cb = syn.client_batch(0, 0, 0, B, K)
    e.img_in.copy_(torch.from_numpy(cb.images))
    e.label_in.copy_(torch.from_numpy(cb.labels))
    e.train_step()
    torch.cuda.synchronize()
    probe = ops.KernelProbe("gemm")
    e.overlap_towers = False
    ops.set_probe(probe)
    for _ in range(2):
        e.train_step()
    ops.set_probe(None)
    torch.cuda.synchronize()
    recs = probe.launches()
    Path(out).write_text(json.dumps({"config": config, "launches": recs}))
    print(f"{len(recs)} probed GEMM launches -> {out}")


def _dispatches(path, counter):
    """GEMM-family dispatches of a counter CSV in Dispatch_Id order: [(name, grid, value)], reduce passes
    folded into the dispatch before them."""
    rows = {}
    with open(path) as f:
        for row in csv.DictReader(f):
            if row.get("Counter_Name") != counter:
                continue
            name = row.get("Kernel_Name", "")
            gemm, red = any(k in name for k in GEMM_KEYS), REDUCE_KEY in name
            if not (gemm or red):
                continue
            d = int(row.get("Dispatch_Id") or row.get("Correlation_Id"))
            ent = rows.setdefault(d, [name, int(row.get("Grid_Size", 0) or 0), 0.0, red])
            ent[2] += float(row["Counter_Value"])
    out = []
    for d in sorted(rows):
        name, grid, v, red = rows[d]
        if red:
            if out:
                out[-1][2] += v
            continue
        out.append([name, grid, v])
    return out


def summarize(probe_json, fetch_csv, write_csv, out):
    pr = json.loads(Path(probe_json).read_text())
    recs = pr["launches"]
    n = len(recs)
    fe, wr = _dispatches(fetch_csv, "FETCH_SIZE"), _dispatches(write_csv, "WRITE_SIZE")
    if len(fe) < n or len(wr) < n:
        raise SystemExit(f"fewer GEMM dispatches in the PMC CSVs ({len(fe)}, {len(wr)}) than probed launches ({n})")
    fe, wr = fe[-n:], wr[-n:]
    shapes = defaultdict(lambda: {"n": 0, "read": 0.0, "write": 0.0, "alg": 0.0, "us": 0.0, "flops": 0.0,
                                  "kernel": ""})
    tot_traffic = tot_alg = 0.0
    for r, f, w in zip(recs, fe, wr):
        rd, wt = 2.0 * f[2] * 1024, w[2] * 1024
        tot_traffic += rd + wt
        tot_alg += r["bytes"]
        m = r["meta"] or ["?"] * 4
        key = f"{r['key'].split('/')[-1]:6s} M={m[0]} N={m[1]} K={m[2]} epi={m[3]}"
        s = shapes[key]
        s["n"] += 1
        s["read"] += rd
        s["write"] += wt
        s["alg"] += r["bytes"]
        s["us"] += r["us"]
        s["flops"] += r["flops"]
        s["kernel"] = f[0][:90]
    table = []
    for key, s in sorted(shapes.items(), key=lambda kv: -kv[1]["us"]):
        table.append({"shape": key, "launches": s["n"], "kernel": s["kernel"],
                      "read_mb": s["read"] / s["n"] / 1e6, "write_mb": s["write"] / s["n"] / 1e6,
                      "algorithmic_mb": s["alg"] / s["n"] / 1e6,
                      "traffic_over_algorithmic": (s["read"] + s["write"]) / max(s["alg"], 1.0),
                      "avg_us": s["us"] / s["n"], "tflops": s["flops"] / (s["us"] * 1e-6) / 1e12})
    res = {"config": pr["config"], "launches": n,
           "traffic_bytes_per_launch": tot_traffic / n, "algorithmic_bytes_per_launch": tot_alg / n,
           "traffic_over_algorithmic": tot_traffic / tot_alg,
           "avg_launch_us": sum(r["us"] for r in recs) / n,
           "tflops": sum(r["flops"] for r in recs) / (sum(r["us"] for r in recs) * 1e-6) / 1e12,
           "source": "rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes over tests/diagnostics/gemm_traffic.py run "
                     "(bench.py's GEMM probe: two eager c4 steps, towers serialised); FETCH_SIZE x 2 + WRITE_SIZE",
           "by_shape": table}
    Path(out).write_text(json.dumps(res, indent=1))
    print(f"{n} launches: traffic {res['traffic_bytes_per_launch'] / 1e6:.1f} MB / algorithmic "
          f"{res['algorithmic_bytes_per_launch'] / 1e6:.1f} MB per launch = {res['traffic_over_algorithmic']:.2f}x")
    for t in table:
        print(f"  {t['shape']:44s} x{t['launches']:3d} {t['avg_us']:7.1f} us {t['tflops']:6.0f} TF  read "
              f"{t['read_mb']:7.1f} write {t['write_mb']:6.1f} alg {t['algorithmic_mb']:6.1f} MB "
              f"({t['traffic_over_algorithmic']:.2f}x)  {t['kernel'][:48]}")


if __name__ == "__main__":
    if sys.argv[1] == "run":
        run(sys.argv[2], *(sys.argv[3:4]))
    else:
        summarize(*sys.argv[2:6])

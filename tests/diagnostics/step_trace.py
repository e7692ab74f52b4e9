"""Diagnostic (GPU box): the c4 (or, with `c5`, the K = 1000-class) client step, no captions,
hipGraph-replayed, for a rocprofv3 kernel trace whose timeline shows the step's idle gaps and stream
overlap (rocprofv3's tracing serialises the two streams, so the per-kernel times are isolated ones):
    rocprofv3 --kernel-trace -d gpurun_out/trace -o run -- python3 tests/diagnostics/step_trace.py 5 [c5]
then `python tests/diagnostics/step_trace.py --analyze gpurun_out/trace/run_results.db` (CPU)."""
import sys
import time
from pathlib import Path


def analyze(path):
    """path: rocprofv3's results database (run_results.db) or a kernel_trace.csv."""
    if path.endswith(".db"):
        import sqlite3
        ks = sorted(sqlite3.connect(path).execute("select start, end, name, queue_id from kernels").fetchall())
    else:
        import csv
        ks = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"], r.get("Queue_Id", "?"))
                    for r in csv.DictReader(open(path)))
    # the replays: split where the gap exceeds 200 us (host sync between replays is not in a graph)
    steps, cur = [], [ks[0]]
    for k in ks[1:]:
        if k[0] - max(c[1] for c in cur) > 200_000:
            steps.append(cur)
            cur = []
        cur.append(k)
    steps.append(cur)
    for s in steps[-3:]:
        t0, t1 = s[0][0], max(k[1] for k in s)
        busy, end = 0, t0
        for a, b, _, _ in s:  # union of kernel intervals
            if b > end:
                busy += b - max(a, end)
                end = b
        ksum = sum(b - a for a, b, _, _ in s)
        queues = {}
        for a, b, n, qid in s:
            queues.setdefault(qid, []).append(b - a)
        print(f"step: wall {(t1 - t0) / 1e3:.1f} us, {len(s)} kernels, GPU busy (any kernel) {busy / 1e3:.1f} us "
              f"({busy / (t1 - t0):.1%}), kernel sum {ksum / 1e3:.1f} us; per queue: " +
              ", ".join(f"{q}: {len(v)} kernels {sum(v) / 1e3:.0f} us" for q, v in queues.items()))


if __name__ == "__main__":
    if len(sys.argv) > 2 and sys.argv[1] == "--analyze":
        analyze(sys.argv[2])
        sys.exit(0)
    import torch
    sys.path.insert(0, str(Path(__file__).resolve().parents[2]))
    from federated_multi_modal_amd import synthetic as syn  # noqa: E402
    from federated_multi_modal_amd.engine import EngineConfig, MapleEngine  # noqa: E402

    J, B, seed, steps = 9, 32, 0, int(sys.argv[1]) if len(sys.argv) > 1 else 5
    K = 1000 if len(sys.argv) > 2 and sys.argv[2] == "c5" else 38
    dev = torch.device("cuda:0")
    e = MapleEngine(EngineConfig(batch=B, classnames=syn.synthetic_classnames(K, seed), prompt_depth=J, seed=seed),
                    device=dev)
    e.set_lr(0.0026)
    b = syn.client_batch(seed, 0, 0, B, K)
    e.load_batch(torch.from_numpy(b.images), torch.from_numpy(b.labels))
    e.train_step()
    g = e.capture_train_step()
    g.replay()
    torch.cuda.synchronize()
    for _ in range(steps):  # one replay at a time, a host sync between: the trace splits on the gaps
        a = time.perf_counter()
        g.replay()
        torch.cuda.synchronize()
        time.sleep(0.002)
    print(f"K={K} step: last {1e3 * (time.perf_counter() - a):.2f} ms, loss {e.loss():.4f}")

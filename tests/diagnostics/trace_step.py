"""Diagnostic: critical-path view of one graph-replayed step from a rocprofv3 kernel trace CSV.
Finds the timed steps (the sgd_kernel launches end each step), takes step `idx`, and prints per
queue: busy time, the union of busy time over all queues, idle gaps, and per-family totals.
    python trace_step.py run_kernel_trace.csv [step_index]"""
import collections
import csv
import re
import sys


def fam(n):
    m = re.search(r"(gemm8?_\w*kernel|attn_\w+?_kernel|ln_\w+?_kernel|transpose|col_reduce|copyBuffer|inject\w*"
                  r"|small_linear\w*|sgd|sumsq|[A-Za-z_]+kernel)", n)
    return m.group(1) if m else n[:40]


def main():
    rows = list(csv.DictReader(open(sys.argv[1])))
    idx = int(sys.argv[2]) if len(sys.argv) > 2 else -3
    ks = sorted(((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Queue_Id"], r["Kernel_Name"]) for r in rows))
    ends = [i for i, k in enumerate(ks) if re.search(r"sgd8?_kernel", k[3])]
    # a step = kernels after the previous step's sgd (exclusive) .. this step's last sgd (inclusive)
    groups, prev = [], -1
    for i in ends:
        if i - prev > 50:
            groups.append((prev + 1, i))
        prev = i
    a, b = groups[idx]
    step = ks[a:b + 1]
    t0, t1 = step[0][0], max(k[1] for k in step)
    print(f"{len(groups)} steps found; step {idx}: {len(step)} kernels, wall {(t1 - t0) / 1e3:.1f} us")
    q = collections.defaultdict(float)
    for s, e, qu, n in step:
        q[qu] += e - s
    for qu, v in q.items():
        print(f"  queue {qu}: busy {v / 1e3:.1f} us")
    # union of busy intervals
    iv = sorted((s, e) for s, e, _, _ in step)
    busy, cs, ce, gaps = 0, iv[0][0], iv[0][1], []
    for s, e in iv[1:]:
        if s > ce:
            busy += ce - cs
            gaps.append(s - ce)
            cs, ce = s, e
        else:
            ce = max(ce, e)
    busy += ce - cs
    print(f"  union busy {busy / 1e3:.1f} us, idle {(t1 - t0 - busy) / 1e3:.1f} us in {len(gaps)} gaps "
          f"(mean {sum(gaps) / max(len(gaps), 1) / 1e3:.2f} us)")
    f = collections.defaultdict(lambda: [0.0, 0])
    for s, e, qu, n in step:
        f[(qu, fam(n))][0] += e - s
        f[(qu, fam(n))][1] += 1
    for (qu, n), (v, c) in sorted(f.items(), key=lambda x: -x[1][0])[:30]:
        print(f"  q{qu} {n:36s} {v / 1e3:8.1f} us  {c:4d} launches")


if __name__ == "__main__":
    main()

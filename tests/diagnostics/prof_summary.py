"""Summarise a rocprofv3 kernel trace (rocpd sqlite .db or kernel_stats.csv) per kernel name."""
import csv
import sqlite3
import sys


def from_db(path):
    c = sqlite3.connect(path)
    rows = c.execute("select name, count(*), sum(end-start), avg(end-start), min(end-start), max(end-start) "
                     "from kernels group by name order by sum(end-start) desc").fetchall()
    return [(r[0], r[1], r[2] / 1e3, r[3] / 1e3, r[4] / 1e3, r[5] / 1e3) for r in rows]


def main():
    path, out = sys.argv[1], sys.argv[2] if len(sys.argv) > 2 else None
    rows = from_db(path)
    tot = sum(r[2] for r in rows)
    lines = [f"# kernel time summary of {path}: total {tot / 1e3:.2f} ms over all dispatches"]
    lines.append("pct,total_us,calls,avg_us,min_us,max_us,name")
    for r in rows:
        lines.append(f"{100 * r[2] / tot:.2f},{r[2]:.1f},{r[1]},{r[3]:.2f},{r[4]:.2f},{r[5]:.2f},\"{r[0]}\"")
    text = "\n".join(lines) + "\n"
    if out:
        open(out, "w").write(text)
    print(text[:4000])


if __name__ == "__main__":
    main()

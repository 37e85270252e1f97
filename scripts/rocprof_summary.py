"""Summarise a rocprofv3 --kernel-trace --stats output (SQLite .db or *_kernel_stats.csv) as a table.

Columns: calls, total and average duration, share of kernel time, and "busy ms/call": the union of the
kernel's dispatch intervals divided by its calls. With launches alternating over two HIP streams two
dispatches of one kernel overlap; the union counts that overlap once, so busy ms/call is the kernel's share
of the wall clock per launch (bench.py's live dominant_ms is the same quantity from HIP events). Needs the
.db form (per-dispatch start/end); the CSV form prints the average there.
"""
import csv
import glob
import os
import sqlite3
import sys


def union_ms(iv):
    iv = sorted(iv)
    acc, lo, hi = 0, None, None
    for a, b in iv:
        if hi is None or a > hi:
            if hi is not None:
                acc += hi - lo
            lo, hi = a, b
        elif b > hi:
            hi = b
    if hi is not None:
        acc += hi - lo
    return acc / 1e6  # ns -> ms


def main(path: str) -> None:
    dbs = glob.glob(os.path.join(path, "**", "*.db"), recursive=True)
    rows = []
    if dbs:
        c = sqlite3.connect(dbs[0])
        spans = {}
        for name, a, b in c.execute("select name, start, end from kernels"):
            spans.setdefault(name, []).append((a, b))
        busy = {name: union_ms(iv) / len(iv) for name, iv in spans.items()}
        # the rocpd top_kernels view reports microseconds
        rows = [(n, k, t * 1e3, a * 1e3, p, busy.get(n, a * 1e-3)) for n, k, t, a, p in
                c.execute("select name, total_calls, total_duration, average, percentage from top_kernels")]
    else:
        for f in glob.glob(os.path.join(path, "**", "*kernel_stats.csv"), recursive=True):
            with open(f) as fh:
                for r in csv.DictReader(fh):
                    rows.append((r["Name"], int(r["Calls"]), float(r["TotalDurationNs"]), float(r["AverageNs"]),
                                 float(r["Percentage"]), float(r["AverageNs"]) / 1e6))
    print("| kernel | calls | total ms | avg ms | % | busy ms/call |")
    print("|---|---|---|---|---|---|")
    for name, calls, tot, avg, pct, bz in rows:
        short = name.split("(")[0][:90]
        print(f"| `{short}` | {calls} | {tot / 1e6:.3f} | {avg / 1e6:.4f} | {pct:.2f} | {bz:.4f} |")


def calls(path: str, substr: str) -> None:
    """Per-dispatch durations (us) of the kernels whose name contains substr, in dispatch order."""
    db = glob.glob(os.path.join(path, "**", "*.db"), recursive=True)[0]
    c = sqlite3.connect(db)
    rows = [(n, a, b) for n, a, b in c.execute("select name, start, end from kernels order by start") if substr in n]
    for i, (n, a, b) in enumerate(rows):
        print(f"{i} {(b - a) / 1e3:.1f} {n.split('(')[0][:60]}")


if __name__ == "__main__":
    if len(sys.argv) > 3 and sys.argv[2] == "--calls":
        calls(sys.argv[1], sys.argv[3])
    else:
        main(sys.argv[1])

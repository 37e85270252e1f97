"""Summarise a rocprofv3 --kernel-trace --stats output (SQLite .db or *_kernel_stats.csv) as a table."""
import csv
import glob
import os
import sqlite3
import sys


def main(path: str) -> None:
    dbs = glob.glob(os.path.join(path, "**", "*.db"), recursive=True)
    rows = []
    if dbs:
        c = sqlite3.connect(dbs[0])
        # the rocpd top_kernels view reports microseconds
        rows = [(n, k, t * 1e3, a * 1e3, p) for n, k, t, a, p in
                c.execute("select name, total_calls, total_duration, average, percentage from top_kernels")]
    else:
        for f in glob.glob(os.path.join(path, "**", "*kernel_stats.csv"), recursive=True):
            with open(f) as fh:
                for r in csv.DictReader(fh):
                    rows.append((r["Name"], int(r["Calls"]), float(r["TotalDurationNs"]), float(r["AverageNs"]),
                                 float(r["Percentage"])))
    print("| kernel | calls | total ms | avg ms | % |")
    print("|---|---|---|---|---|")
    for name, calls, tot, avg, pct in rows:
        short = name.split("(")[0][:90]
        print(f"| `{short}` | {calls} | {tot / 1e6:.3f} | {avg / 1e6:.4f} | {pct:.2f} |")


if __name__ == "__main__":
    main(sys.argv[1])

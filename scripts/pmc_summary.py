"""Sum rocprofv3 --pmc counters per kernel from the SQLite output (counters_collection view)."""
import glob
import os
import sqlite3
import sys
from collections import defaultdict


def collect(path: str):
    out = defaultdict(lambda: defaultdict(float))
    calls = defaultdict(set)
    for db in glob.glob(os.path.join(path, "**", "*.db"), recursive=True):
        c = sqlite3.connect(db)
        for name, ctr, val, disp in c.execute(
                "select kernel_name, counter_name, value, dispatch_id from counters_collection"):
            short = name.split("(")[0]
            out[short][ctr] += val
            calls[short].add(disp)
    return out, calls


if __name__ == "__main__":
    agg = defaultdict(lambda: defaultdict(float))
    ncall = {}
    for p in sys.argv[1:]:
        o, c = collect(p)
        for k, v in o.items():
            agg[k].update(v)
            ncall[k] = len(c[k])
    for k, v in agg.items():
        print(f"{k}  (dispatches: {ncall[k]})")
        for ctr in sorted(v):
            print(f"    {ctr:24s} {v[ctr]:.6g}")

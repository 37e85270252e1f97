"""Sum rocprofv3 --pmc counter CSVs per kernel (one value per counter per dispatch summed over the
dispatch's instances), with each kernel's mean dispatch duration. Usage: pmc_csv.py DIR... [--kernel SUBSTR]"""
import csv
import glob
import os
import sys
from collections import defaultdict


def collect(paths, want=None):
    vals = defaultdict(lambda: defaultdict(float))
    disp = defaultdict(dict)
    for p in paths:
        for f in glob.glob(os.path.join(p, "**", "*counter_collection.csv"), recursive=True):
            for row in csv.DictReader(open(f)):
                k = row["Kernel_Name"].split("(")[0]
                if want and want not in k:
                    continue
                vals[k][row["Counter_Name"]] += float(row["Counter_Value"])
                disp[k][(f, row["Dispatch_Id"])] = int(row["End_Timestamp"]) - int(row["Start_Timestamp"])
    return vals, disp


if __name__ == "__main__":
    args = [a for a in sys.argv[1:] if not a.startswith("--")]
    want = None
    if "--kernel" in sys.argv:
        want = sys.argv[sys.argv.index("--kernel") + 1]
        args = [a for a in args if a != want]
    vals, disp = collect(args, want)
    for k, v in vals.items():
        d = disp[k]
        print(f"{k}  dispatches={len(d)}  mean_ms={sum(d.values()) / max(len(d), 1) / 1e6:.4f}")
        for c in sorted(v):
            print(f"    {c:26s} {v[c]:.6g}")

"""Per-kernel rocprofv3 --pmc counters from one or more pass directories, PER DISPATCH: each counter's value is
its mean over the dispatches of the pass(es) that collected it (a counter in two passes averages over both), so
every figure is one launch's value. The header of each kernel carries its mean dispatch duration and its code
object's resources as rocprofv3 records them (VGPRs, SGPRs, scratch bytes per lane, LDS bytes per workgroup,
grid and workgroup size). Usage: pmc_csv.py DIR... [--kernel SUBSTR]"""
import csv
import glob
import os
import sys
from collections import defaultdict


def collect(paths, want=None):
    vals = defaultdict(lambda: defaultdict(list))  # kernel -> counter -> [per-dispatch values]
    disp = defaultdict(dict)                        # kernel -> (file, dispatch) -> ns
    res = {}
    for p in paths:
        for f in glob.glob(os.path.join(p, "**", "*counter_collection.csv"), recursive=True):
            per = defaultdict(float)  # (kernel, dispatch, counter) -> value summed over the row's instances
            for row in csv.DictReader(open(f)):
                k = row["Kernel_Name"].split("(")[0]
                if want and want not in k:
                    continue
                per[(k, row["Dispatch_Id"], row["Counter_Name"])] += float(row["Counter_Value"])
                disp[k][(f, row["Dispatch_Id"])] = int(row["End_Timestamp"]) - int(row["Start_Timestamp"])
                res[k] = {"vgpr": row.get("VGPR_Count"), "agpr": row.get("Accum_VGPR_Count"), "sgpr": row.get("SGPR_Count"),
                          "scratch": row.get("Scratch_Size"), "lds": row.get("LDS_Block_Size"),
                          "grid": row.get("Grid_Size"), "wg": row.get("Workgroup_Size")}
            for (k, _, c), v in per.items():
                vals[k][c].append(v)
    return vals, disp, res


if __name__ == "__main__":
    args = [a for a in sys.argv[1:] if not a.startswith("--")]
    want = None
    if "--kernel" in sys.argv:
        want = sys.argv[sys.argv.index("--kernel") + 1]
        args = [a for a in args if a != want]
    vals, disp, res = collect(args, want)
    print("# per-dispatch values (mean over the dispatches of the passes that collected each counter)")
    for k, v in vals.items():
        d = disp[k]
        r = res.get(k, {})
        extra = " ".join(f"{x}={r[x]}" for x in ("vgpr", "agpr", "sgpr", "scratch", "lds", "grid", "wg") if r.get(x))
        print(f"{k}  dispatches={len(d)}  mean_ms={sum(d.values()) / max(len(d), 1) / 1e6:.4f}  {extra}")
        for c in sorted(v):
            print(f"    {c:26s} {sum(v[c]) / len(v[c]):.6g}")

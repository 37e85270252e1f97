#!/bin/bash
# Register / scratch / LDS use of every kernel in a HIP object (the gfx950 code object's metadata notes).
# usage: scripts/kernel_regs.sh miningsimulation_amd/csrc/obj/msim_sel_kernels_m9.o [name-regex]
set -e
t=$(mktemp -d)
cp "$1" "$t/k.o"
(cd "$t" && /opt/rocm/lib/llvm/bin/llvm-objdump --offloading k.o > /dev/null)
/opt/rocm/lib/llvm/bin/llvm-readelf --notes "$t"/k.o.*gfx950* > "$t/notes.txt"
python3 - "$t/notes.txt" "${2:-}" <<'PY'
import re, sys
flt = re.compile(sys.argv[2])
keys = ["vgpr_count", "agpr_count", "vgpr_spill_count", "sgpr_spill_count", "private_segment_fixed_size",
        "group_segment_fixed_size"]
short = {"vgpr_count": "vgpr", "agpr_count": "agpr", "vgpr_spill_count": "vspill", "sgpr_spill_count": "sspill",
         "private_segment_fixed_size": "scratch", "group_segment_fixed_size": "lds"}
cur = {}
for line in open(sys.argv[1]):
    m = re.match(r"\s+\.(\w+):\s+(\S+)", line)
    if not m:
        continue
    k, v = m.groups()
    if k == "name" and v.startswith("_Z"):
        cur = {"name": v}
    elif k in keys and "name" in cur:
        cur[k] = v
    if k == "wavefront_size" and "name" in cur:
        if flt.search(cur["name"]):
            print(cur["name"][:80], " ".join("%s=%s" % (short[x], cur.get(x)) for x in keys))
        cur = {}
PY
rm -rf "$t"

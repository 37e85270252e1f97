#!/bin/bash
# E1 pool diagnostics: per-wave POOLPROF counters (SEL_PROF variant) on configs[2], and the kernel trace
# (LDS / VGPR / scratch per kernel as the runtime saw them).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/${TAG:-poolprof}; mkdir -p $O
MSIM_LIB=$PWD/miningsimulation_amd/variants/libmsim_prof.so timeout -k 10 120 python -u scripts/stage_c3.py ${N:-131072} > $O/prof_c3.txt 2>&1 || { tail -20 $O/prof_c3.txt; exit 1; }
grep -c POOLPROF $O/prof_c3.txt; grep POOLPROF $O/prof_c3.txt | head -16; grep "^c3" $O/prof_c3.txt
timeout -k 10 120 rocprofv3 --kernel-trace --output-format csv -d $O/kt -o kt -- python3 scripts/stage_c3.py 32768 > $O/kt.log 2>&1 || { tail -20 $O/kt.log; exit 1; }
python3 - <<'PY'
import csv,glob
f=glob.glob('gpurun_out/'+__import__('os').environ.get('TAG','poolprof')+'/kt/**/*kernel_trace.csv',recursive=True)[0]
rows=list(csv.DictReader(open(f)))
print(list(rows[0].keys()))
seen=set()
for r in rows:
    n=r['Kernel_Name'][:70]
    if n in seen: continue
    seen.add(n)
    print(n, {k:r[k] for k in r if any(s in k for s in ('LDS','Scratch','VGPR','SGPR','Workgroup','Grid'))}, int(r['End_Timestamp'])-int(r['Start_Timestamp']))
PY

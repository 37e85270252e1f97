#!/bin/bash
# sweep per-kernel timing: default capacity classes vs SMALL everywhere
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r2i}; mkdir -p $O
timeout -k 10 300 python -u scripts/stage_sweep.py 2048 > $O/sweep_default.txt 2>&1 || { cat $O/sweep_default.txt; exit 1; }
grep sweep $O/sweep_default.txt
MSIM_SEL_CAPS=0 timeout -k 10 300 python -u scripts/stage_sweep.py 2048 > $O/sweep_small.txt 2>&1 || { cat $O/sweep_small.txt; exit 1; }
grep sweep $O/sweep_small.txt
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_sweep -o sweep -- python3 scripts/stage_sweep.py 2048 > $O/prof_sweep.log 2>&1 || { tail -20 $O/prof_sweep.log; exit 1; }
find $O/prof_sweep -name "*kernel_stats.csv" -exec cat {} \; | cut -c1-200

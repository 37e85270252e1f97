#!/bin/bash
# Three-tier engine-phase threshold (16 / 32 / 48 for delays <= 2 s / <= 10 s / above): sweep and c3.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r2x}; mkdir -p $O
timeout -k 10 200 python -u scripts/stage_sweep.py 8192 > $O/sweep.txt 2>&1 || { cat $O/sweep.txt; exit 1; }
grep sweep $O/sweep.txt
timeout -k 10 120 python -u scripts/stage_c3.py > $O/c3.txt 2>&1 || { cat $O/c3.txt; exit 1; }
grep '^c3' $O/c3.txt | cut -c1-140

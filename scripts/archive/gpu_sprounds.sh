#!/bin/bash
# Selfish pipeline S2 rounds (MSIM_SELPIPE=1, configs[2], one serial step under rocprofv3): per-dispatch durations
# of the table-path and engine kernels, round by round.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp MSIM_SELPIPE=1
O=gpurun_out/${TAG:-r05/sprounds}; mkdir -p $O
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o prof -- python3 bench.py --config c3 --steps 1 --warmup 0 --streams 1 --no-cpu-baseline > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
python3 scripts/rocprof_summary.py $O/prof > $O/rocprof.md && head -8 $O/rocprof.md
python3 scripts/rocprof_summary.py $O/prof --calls msim_sp_ > $O/calls.txt && rm -rf $O/prof
awk 'NR % 20 == 1' $O/calls.txt | head -60

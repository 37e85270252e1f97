#!/bin/bash
# Quick E1 pool check: POOLPROF counters (SEL_PROF variant) and the c3 bench line of the default library.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/${TAG:-poolq}; mkdir -p $O
MSIM_LIB=$PWD/miningsimulation_amd/variants/libmsim_prof.so timeout -k 10 120 python -u scripts/stage_c3.py ${N:-131072} > $O/prof_c3.txt 2>&1 || { tail -20 $O/prof_c3.txt; exit 1; }
grep POOLPROF $O/prof_c3.txt | head -8; grep "^c3" $O/prof_c3.txt | cut -c1-150
timeout -k 10 300 python -u bench.py --config c3 --streams 1 --no-cpu-baseline > $O/bench_c3_s1.json 2> $O/bench_c3_s1.err || { tail -30 $O/bench_c3_s1.err; exit 1; }
python3 -c "import json;d=json.load(open('$O/bench_c3_s1.json'));print('c3 s1',d['value'],d['ms_per_step'])"
if [ -n "$SWEEP" ]; then timeout -k 10 300 python -u scripts/stage_sweep.py 8192 > $O/sweep.txt 2>&1 || { cat $O/sweep.txt; exit 1; }; grep sweep $O/sweep.txt; fi

#!/bin/bash
# c2 tails A/B (round 5): serial rocprof of the c2 bench line for each K2 grid cap in CAPS (MSIM_K2_GRID, 0 = the
# list capacity's grid).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r05/k2grid}; mkdir -p $O
for c in ${CAPS}; do
  E=""; [ $c != 0 ] && E="MSIM_K2_GRID=$c"
  env $E timeout -k 10 300 python3 bench.py --config c2 --streams 1 --no-cpu-baseline > $O/bench_$c.json 2> $O/bench_$c.err || { tail -5 $O/bench_$c.err; exit 1; }
  python3 -c "import json;d=json.load(open('$O/bench_$c.json'));print('cap $c',d['value'],d['ms_per_step'])"
done

#!/bin/bash
# configs[3] sweep A/B (round 5): the sweep bench at 8 192 runs per point with the points dispatched costliest
# first (msim_sweep_create) against the caller's grid order (MSIM_SWEEP_LISTED_ORDER=1), each twice.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r05/sweeplpt}; mkdir -p $O
for r in ${REPS:-1 2}; do
  for v in ${VARS:-lpt listed}; do
    E=""; [ $v = listed ] && E="MSIM_SWEEP_LISTED_ORDER=1"
    env $E timeout -k 10 300 python3 scripts/bench_sweep.py --runs-per-point 8192 > $O/sweep_${v}_$r.json 2> $O/sweep_${v}_$r.err || { tail -5 $O/sweep_${v}_$r.err; exit 1; }
    python3 -c "import json;d=json.load(open('$O/sweep_${v}_$r.json'));print('$v $r',d['value'],d['ms_per_step'])"
  done
done

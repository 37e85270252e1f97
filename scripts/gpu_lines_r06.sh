#!/bin/bash
# The bench lines without a profiler, after the rocprof summaries and PMC files they read are in place under
# profiles/r06/final (so every file-backed field of a line refers to the committed files): the default line
# with the CPU baseline, then c1/c2/c3/c5 with two streams (_s0) and --streams 1 (_s1). Output gpurun_out/$TAG.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/${TAG:-lines06}; mkdir -p $O
timeout -k 10 400 python -u bench.py > $O/bench_default.json 2> $O/bench_default.err || { tail -20 $O/bench_default.err; exit 1; }
for c in ${CFGS:-c1 c2 c3 c5}; do
  for s in 0 1; do
    B=""; [ $s = 1 ] && B="--streams 1"
    timeout -k 10 300 python3 bench.py --config $c $B --no-cpu-baseline > $O/bench_${c}_s$s.json 2> $O/bench_${c}_s$s.err || { tail -20 $O/bench_${c}_s$s.err; exit 1; }
    python3 -c "import json;d=json.load(open('$O/bench_${c}_s$s.json'));r=d['roofline'];print('$c s$s',d['value'],d['ms_per_step'],r.get('frac'),r.get('frac_cycles'),r.get('frac_cycles_serial'))"
  done
done

#!/bin/bash
# The bench lines as the driver runs them (no profiler): the default line (c2, with the CPU baseline), then
# c3 and c5 with the default two streams, then c2, c3 and c5 serial (--streams 1). Each reads its roofline
# constants from profiles/r05/final. With INSTALL=DIR the rocprof summaries in DIR (a gpu_r05.sh output of the same
# call) are first copied into profiles/r05/final on the box, so the lines read the summaries made beside them.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r05/lines}; mkdir -p $O
[ -n "$INSTALL" ] && cp $INSTALL/rocprof_*.md profiles/r05/final/
timeout -k 10 400 python -u bench.py > $O/bench_default.json 2> $O/bench_default.err || { tail -30 $O/bench_default.err; exit 1; }
for c in ${CFGS-c3 c5}; do
  timeout -k 10 300 python -u bench.py --config $c --no-cpu-baseline > $O/bench_line_$c.json 2> $O/bench_line_$c.err || { tail -30 $O/bench_line_$c.err; exit 1; }
done
for c in ${SERIAL-c2 c3 c5}; do
  timeout -k 10 300 python -u bench.py --config $c --streams 1 --no-cpu-baseline > $O/bench_line_${c}_s1.json 2> $O/bench_line_${c}_s1.err || { tail -30 $O/bench_line_${c}_s1.err; exit 1; }
done
for f in $O/bench_*.json; do
  python3 -c "import json;d=json.load(open('$f'));r=d['roofline'];print('$f',d['value'],d['ms_per_step'],r.get('frac'),r.get('dominant_ms_file'),r.get('traffic'))"
done

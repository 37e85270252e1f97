#!/bin/bash
# Bench line with the dominant-kernel roofline (default args), and serial (--streams 1) kernel stats of c2 and
# c3 for clean per-kernel durations.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r2u}; mkdir -p $O
timeout -k 10 300 python -u bench.py --no-cpu-baseline > $O/bench_c2.json 2> $O/bench_c2.err || { tail -30 $O/bench_c2.err; exit 1; }
cat $O/bench_c2.json
timeout -k 10 300 python -u bench.py --config c3 --no-cpu-baseline > $O/bench_c3.json 2> $O/bench_c3.err || { tail -30 $O/bench_c3.err; exit 1; }
python3 -c "import json;d=json.load(open('$O/bench_c3.json'));print('c3',d['value'],d['roofline'])"
for c in c2 c3; do
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_${c}_s1 -o $c -- python3 bench.py --config $c --streams 1 --no-cpu-baseline > $O/prof_${c}_s1.log 2>&1 || { tail -20 $O/prof_${c}_s1.log; exit 1; }
done
find $O -name "*kernel_stats.csv" -exec cut -c1-120 {} \;

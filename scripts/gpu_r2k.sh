#!/bin/bash
# Round-2 re-entry rehearsal: full GPU suite, smoke, c2/c3 bench lines, kernel stats of c2 and c3.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r2k}; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -3 $O/pytest.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -30 $O/smoke.log; exit 1; }
cat $O/smoke.log
timeout -k 10 300 python -u bench.py --config c2 > $O/bench_c2.json 2> $O/bench_c2.err || { tail -30 $O/bench_c2.err; exit 1; }
cat $O/bench_c2.json
timeout -k 10 300 python -u bench.py --config c3 --no-cpu-baseline > $O/bench_c3.json 2> $O/bench_c3.err || { tail -30 $O/bench_c3.err; exit 1; }
cat $O/bench_c3.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_c2 -o c2 -- python3 bench.py --config c2 --no-cpu-baseline > $O/prof_c2.log 2>&1 || { tail -20 $O/prof_c2.log; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_c3 -o c3 -- python3 bench.py --config c3 --no-cpu-baseline > $O/prof_c3.log 2>&1 || { tail -20 $O/prof_c3.log; exit 1; }
find $O -name "*kernel_stats.csv" -exec cut -c1-160 {} \;

#!/bin/bash
# Rehearsal of the committed code: full GPU suite, smoke, default bench (with CPU baseline),
# c3 / c5 bench lines, the configs[3] sweep at 8192 runs/point.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/${TAG:-rehearsal}; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -30 $O/smoke.log; exit 1; }
tail -3 $O/smoke.log
timeout -k 10 400 python -u bench.py > $O/bench_default.json 2> $O/bench_default.err || { tail -30 $O/bench_default.err; exit 1; }
python3 -c "import json;d=json.load(open('$O/bench_default.json'));print('c2',d['value'],d['ms_per_step'],d['roofline']['frac'],d['roofline']['valu_issue_frac_pmc'],d['cpu_baseline']['value'])"
for c in c3 c5; do
  timeout -k 10 300 python -u bench.py --config $c --no-cpu-baseline > $O/bench_$c.json 2> $O/bench_$c.err || { tail -30 $O/bench_$c.err; exit 1; }
  python3 -c "import json;d=json.load(open('$O/bench_$c.json'));print('$c',d['value'],d['ms_per_step'],d['roofline']['frac'],d['roofline'].get('valu_issue_frac_pmc'))"
done
timeout -k 10 200 python -u scripts/stage_sweep.py 8192 > $O/sweep.txt 2>&1 || { cat $O/sweep.txt; exit 1; }
grep sweep $O/sweep.txt
if [ -n "$PROF" ]; then
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_c2s1 -o prof -- python3 bench.py --config c2 --streams 1 --steps 10 --warmup 2 --no-cpu-baseline > $O/prof_c2s1.log 2>&1 || { tail -20 $O/prof_c2s1.log; exit 1; }
  python3 scripts/rocprof_summary.py $O/prof_c2s1 | head -8
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_c3 -o prof -- python3 bench.py --config c3 --steps 3 --warmup 1 --no-cpu-baseline > $O/prof_c3.log 2>&1 || { tail -20 $O/prof_c3.log; exit 1; }
  python3 scripts/rocprof_summary.py $O/prof_c3 | head -8
fi

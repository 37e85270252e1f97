#!/bin/bash
# Round-4 measurement of the shipped code: GPU suite, default bench line, and rocprofv3 kernel-trace
# summaries of the EXACT bench commands (default two streams, 40 steps) beside the serial ones, so every
# roofline field of the bench line can be recomputed from a file under profiles/r04/.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r04base}; mkdir -p $O
if [ -z "$NOTEST" ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
  tail -1 $O/pytest.log
fi
timeout -k 10 400 python -u bench.py > $O/bench_default.json 2> $O/bench_default.err || { tail -30 $O/bench_default.err; exit 1; }
python3 -c "import json;d=json.load(open('$O/bench_default.json'));print('c2',d['value'],d['ms_per_step'],d['roofline']['frac'],d['roofline']['dominant_ms'],d['cpu_baseline']['value'])"
for c in ${CFGS:-c2 c3 c5}; do
  for s in 0 1; do
    B=""; [ $s = 1 ] && B="--streams 1"
    timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_${c}_s$s -o prof -- python3 bench.py --config $c $B --no-cpu-baseline > $O/bench_${c}_s$s.json 2> $O/prof_${c}_s$s.err || { tail -20 $O/prof_${c}_s$s.err; exit 1; }
    python3 -c "import json;d=json.load(open('$O/bench_${c}_s$s.json'));r=d['roofline'];print('$c s$s',d['value'],d['ms_per_step'],r['frac'],r['dominant_ms'])"
    python3 scripts/rocprof_summary.py $O/prof_${c}_s$s > $O/rocprof_${c}_s$s.md
    head -6 $O/rocprof_${c}_s$s.md
  done
done

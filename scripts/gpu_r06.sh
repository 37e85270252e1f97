#!/bin/bash
# Round-6 measurement of the shipped code through gpurun (one call):
#   pytest -m gpu (unless NOTEST=1), smoke (SMOKE=1), the default bench line with the CPU baseline (unless
#   NOBENCH=1), and for every config in CFGS (default c2 c3 c5) rocprofv3 --kernel-trace --stats summaries of
#   the exact bench commands, default two streams (_s0) and --streams 1 (_s1), then (PMC=1) the counter passes
#   behind the bench line's PMC constants (scripts/gpu_pmc_r06.sh). Output under gpurun_out/$TAG.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r06}; mkdir -p $O
if [ -z "$NOTEST" ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread ${PYTEST_K:+-k "$PYTEST_K"} > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
  tail -1 $O/pytest.log
fi
if [ -n "$SMOKE" ]; then
  timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -30 $O/smoke.log; exit 1; }
  tail -3 $O/smoke.log
fi
if [ -z "$NOBENCH" ]; then
  timeout -k 10 400 python -u bench.py > $O/bench_default.json 2> $O/bench_default.err || { tail -30 $O/bench_default.err; exit 1; }
  python3 -c "import json;d=json.load(open('$O/bench_default.json'));r=d['roofline'];print('c2',d['value'],d['ms_per_step'],r.get('frac'),r['dominant_ms'],d['cpu_baseline']['value'])"
fi
for c in ${CFGS-c2 c3 c5}; do
  for s in ${STREAMS:-0 1}; do
    B=""; [ $s = 1 ] && B="--streams 1"
    timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_${c}_s$s -o prof -- python3 bench.py --config $c $B --no-cpu-baseline > $O/bench_${c}_s$s.json 2> $O/prof_${c}_s$s.err || { tail -20 $O/prof_${c}_s$s.err; exit 1; }
    python3 -c "import json;d=json.load(open('$O/bench_${c}_s$s.json'));r=d['roofline'];print('$c s$s',d['value'],d['ms_per_step'],r.get('frac'),r['dominant_ms'],r['kernels_busy_ms'])"
    python3 scripts/rocprof_summary.py $O/prof_${c}_s$s > $O/rocprof_${c}_s$s.md
    head -6 $O/rocprof_${c}_s$s.md
    rm -rf $O/prof_${c}_s$s
  done
done
if [ -n "$PMC" ]; then
  TAG=${TAG:-r06}/pmc bash scripts/gpu_pmc_r06.sh > $O/pmc.log 2>&1 || { tail -20 $O/pmc.log; exit 1; }
  echo pmc done
fi

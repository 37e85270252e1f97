#!/bin/bash
# Segment-parallel selfish path (msim_selseg.h): its GPU tests, the selfish GPU tests, then c3 bench lines (default
# and serial, MSIM_SELSEG=1) with rocprof summaries, and E1 (the default) on the same box for comparison.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/${TAG:-seg}; mkdir -p $O
if [ -z "$NOTEST" ]; then
  timeout -k 10 600 python -u -m pytest ${PYTEST_FILES:-tests/test_gpu_selseg.py} -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
  tail -1 $O/pytest.log
fi
for s in ${STREAMS:-1 0}; do
  B=""; [ $s = 1 ] && B="--streams 1"
  MSIM_SELSEG=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_c3_s$s -o prof -- python3 bench.py --config c3 $B --steps ${STEPS:-10} --warmup 2 --no-cpu-baseline > $O/bench_c3_s$s.json 2> $O/prof_c3_s$s.err || { tail -20 $O/prof_c3_s$s.err; exit 1; }
  python3 -c "import json;d=json.load(open('$O/bench_c3_s$s.json'));print('seg c3 s$s',d['value'],d['ms_per_step'])"
  python3 scripts/rocprof_summary.py $O/prof_c3_s$s > $O/rocprof_c3_s$s.md
  head -8 $O/rocprof_c3_s$s.md
  rm -rf $O/prof_c3_s$s
done
if [ -n "$E1" ]; then
  timeout -k 10 300 python3 bench.py --config c3 --streams 1 --steps 10 --warmup 2 --no-cpu-baseline > $O/bench_c3_e1_s1.json 2> $O/e1.err || { tail -20 $O/e1.err; exit 1; }
  python3 -c "import json;d=json.load(open('$O/bench_c3_e1_s1.json'));print('E1 c3 s1',d['value'],d['ms_per_step'])"
fi

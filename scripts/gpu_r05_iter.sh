#!/bin/bash
# Round-5 iteration on one GPU: the GPU tests named by PYTEST_FILES (default: the selfish / parity / pipeline
# ones), then one bench line per config in CFGS (default two streams and --streams 1) and, with PROF=1, a
# rocprofv3 --kernel-trace --stats summary of each. Output under gpurun_out/$TAG.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r05iter}; mkdir -p $O
if [ -z "$NOTEST" ]; then
  timeout -k 10 900 python -u -m pytest ${PYTEST_FILES:-tests/test_gpu_selfish.py tests/test_gpu_parity.py} -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
  tail -1 $O/pytest.log
fi
for c in ${CFGS-c3 c2 c1}; do
  for st in ${STREAMS:-0 1}; do
    B=""; [ $st = 1 ] && B="--streams 1"
    if [ -n "$PROF" ]; then
      timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_${c}_s$st -o prof -- python3 bench.py --config $c $B --no-cpu-baseline ${BENCH_ARGS} > $O/bench_${c}_s$st.json 2> $O/bench_${c}_s$st.err || { tail -20 $O/bench_${c}_s$st.err; exit 1; }
      python3 scripts/rocprof_summary.py $O/prof_${c}_s$st > $O/rocprof_${c}_s$st.md && rm -rf $O/prof_${c}_s$st
      head -8 $O/rocprof_${c}_s$st.md
    else
      timeout -k 10 300 python3 bench.py --config $c $B --no-cpu-baseline ${BENCH_ARGS} > $O/bench_${c}_s$st.json 2> $O/bench_${c}_s$st.err || { tail -20 $O/bench_${c}_s$st.err; exit 1; }
    fi
    python3 -c "import json;d=json.load(open('$O/bench_${c}_s$st.json'));r=d['roofline'];print('$c s$st',d['value'],d['ms_per_step'],r.get('frac'),r['dominant_ms'],r['kernels_busy_ms'])"
  done
done

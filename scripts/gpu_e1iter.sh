#!/bin/bash
# E1 iteration (round 5): the selfish / parity GPU tests, the c3 bench line (serial and default), the configs[3]
# sweep at 8 192 runs per point, and a rocprof summary of the serial c3 line.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r05/e1}; mkdir -p $O
timeout -k 10 600 python -u -m pytest ${PYTEST_FILES:-tests/test_gpu_selfish.py tests/test_gpu_parity.py tests/test_selkat.py} -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for st in 1 2; do
  timeout -k 10 300 python3 bench.py --config c3 --streams $st --no-cpu-baseline > $O/bench_c3_s$st.json 2> $O/bench_c3_s$st.err || { tail -5 $O/bench_c3_s$st.err; exit 1; }
  python3 -c "import json;d=json.load(open('$O/bench_c3_s$st.json'));print('c3 streams $st',d['value'],d['ms_per_step'])"
done
timeout -k 10 300 python3 scripts/bench_sweep.py --runs-per-point 8192 > $O/sweep.json 2> $O/sweep.err || { tail -5 $O/sweep.err; exit 1; }
cat $O/sweep.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o prof -- python3 bench.py --config c3 --streams 1 --no-cpu-baseline > $O/prof_c3.json 2> $O/prof_c3.err || { tail -5 $O/prof_c3.err; exit 1; }
python3 scripts/rocprof_summary.py $O/prof > $O/rocprof_c3_s1.md && rm -rf $O/prof && head -5 $O/rocprof_c3_s1.md

#!/bin/bash
# E1 workgroup pool: selfish / general / parity GPU tests, then c3 bench lines and the configs[3] sweep.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/${TAG:-pool}; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_selfish.py tests/test_gpu_general.py -x -v --timeout 240 --timeout-method thread > $O/pytest_sel.log 2>&1 || { tail -40 $O/pytest_sel.log; exit 1; }
tail -2 $O/pytest_sel.log
for s in 1 2; do
  timeout -k 10 300 python -u bench.py --config c3 --streams $s --no-cpu-baseline > $O/bench_c3_s$s.json 2> $O/bench_c3_s$s.err || { tail -30 $O/bench_c3_s$s.err; exit 1; }
  python3 -c "import json;d=json.load(open('$O/bench_c3_s$s.json'));print('c3 s$s',d['value'],d['ms_per_step'],d['roofline']['kernel_ms'])"
done
timeout -k 10 300 python -u scripts/stage_sweep.py 8192 > $O/sweep.txt 2>&1 || { cat $O/sweep.txt; exit 1; }
grep sweep $O/sweep.txt
if [ -n "$FULL" ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_all.log 2>&1 || { tail -40 $O/pytest_all.log; exit 1; }
  tail -1 $O/pytest_all.log
fi

#!/bin/bash
# Settled-state (macro) form for one-selfish networks: selfish GPU parity, c3 and sweep timing (macro vs
# MSIM_SEL_NO_MACRO), kernel stats of c3.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r2m}; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_selfish.py tests/test_gpu_parity.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -3 $O/pytest.log
timeout -k 10 300 python -u bench.py --config c3 --no-cpu-baseline > $O/bench_c3.json 2> $O/bench_c3.err || { tail -30 $O/bench_c3.err; exit 1; }
cat $O/bench_c3.json
MSIM_SEL_NO_MACRO=1 timeout -k 10 300 python -u scripts/stage_c3.py > $O/c3_nomacro.txt 2>&1 || { cat $O/c3_nomacro.txt; exit 1; }
cat $O/c3_nomacro.txt
timeout -k 10 300 python -u scripts/stage_sweep.py 2048 > $O/sweep.txt 2>&1 || { cat $O/sweep.txt; exit 1; }
cat $O/sweep.txt
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_c3 -o c3 -- python3 bench.py --config c3 --no-cpu-baseline > $O/prof_c3.log 2>&1 || { tail -20 $O/prof_c3.log; exit 1; }
find $O -name "*kernel_stats.csv" -exec cut -c1-160 {} \;

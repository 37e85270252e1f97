#!/bin/bash
# Pipeline without the per-block word stream: GPU parity (honest + selfish), c2 bench + kernel stats,
# then the mixed-selfish A/B variants and SQ counters (gpu_r2n.sh).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r2o}; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_selfish.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
timeout -k 10 300 python -u bench.py --config c2 --no-cpu-baseline > $O/bench_c2.json 2> $O/bench_c2.err || { tail -30 $O/bench_c2.err; exit 1; }
cut -c1-600 $O/bench_c2.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_c2 -o c2 -- python3 bench.py --config c2 --no-cpu-baseline > $O/prof_c2.log 2>&1 || { tail -20 $O/prof_c2.log; exit 1; }
find $O/prof_c2 -name "*kernel_stats.csv" -exec cut -c1-150 {} \;
TAG=r2o_ab bash scripts/gpu_r2n.sh

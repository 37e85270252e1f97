#!/bin/bash
# Per-point engine-phase threshold (16 for delays <= 2 s, 32 above): selfish GPU tests, overlap test, c3, sweep,
# and the sweep with every point at 48.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r2w}; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_selfish.py tests/test_gpu_parity.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
timeout -k 10 120 python -u scripts/stage_c3.py > $O/c3.txt 2>&1 || { cat $O/c3.txt; exit 1; }
grep '^c3' $O/c3.txt | cut -c1-140
timeout -k 10 200 python -u scripts/stage_sweep.py 8192 > $O/sweep.txt 2>&1 || { cat $O/sweep.txt; exit 1; }
grep sweep $O/sweep.txt
MSIM_SEL_XTH=48 timeout -k 10 200 python -u scripts/stage_sweep.py 8192 > $O/sweep48.txt 2>&1 || { cat $O/sweep48.txt; exit 1; }
grep sweep $O/sweep48.txt

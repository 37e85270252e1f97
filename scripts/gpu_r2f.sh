#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${TAG:-r2f}; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_selfish.py -q --timeout 300 --timeout-method thread -m gpu -k "not readme and not full_sweep" > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
timeout -k 10 300 python -u scripts/stage_c3.py 131072 > $O/stage.txt 2>&1 || { cat $O/stage.txt; exit 1; }
grep c3 $O/stage.txt
timeout -k 10 300 python -u scripts/stage_sweep.py 2048 > $O/sweep.txt 2>&1 || { cat $O/sweep.txt; exit 1; }
grep sweep $O/sweep.txt

#!/bin/bash
# multi-device entry points + wide sharding exactness
set -o pipefail
make -s -C host >/dev/null 2>&1 || true
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r2j}; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_multi.py tests/test_gpu_wide.py tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread -m gpu > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -3 $O/pytest.log


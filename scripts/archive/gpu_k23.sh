#!/bin/bash
# K2/K3 changes: the pipeline parity tests, then the c2 tails (rocprof, serial) and K3 phase timing.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/${TAG:-k23}; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_samplers.py -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
TAG=${TAG:-k23}/tails bash scripts/gpu_tails.sh
grep K3PROF gpurun_out/${TAG:-k23}/tails/k3.json | head -4

#!/bin/bash
# Large-network pipeline changes: its GPU parity tests, then the c5 tail profile (scripts/archive/gpu_w3prof.sh).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${TAG:-wide}; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread -k "wide or c5 or large" > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
TAG=${TAG:-wide} bash scripts/archive/gpu_w3prof.sh

#!/bin/bash
# K3 restructured (fewer dependent memory rounds, one-wave workgroups): the GPU parity tests of the honest
# pipeline, then the c2 tails A/B (scripts/gpu_tails.sh) against the previous K3 (variant old256).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${TAG:-k3v2}; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread -k "parity or preset or shard or pipeline or retry or golden" > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
TAG=${TAG:-k3v2} VARIANTS="${VARIANTS:-old256 n256}" bash scripts/gpu_tails.sh

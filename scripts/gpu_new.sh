#!/bin/bash
# New GPU tests (samplers, model cross-check, wide path) + a c3 bench.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${1:-n1}
mkdir -p "$OUT"
export TMPDIR=/tmp
stop() { echo "STOP after $1 rc=$2" | tee -a "$OUT/status.txt"; exit "$2"; }
timeout -k 10 400 python -u -m pytest tests/test_gpu_samplers.py tests/test_gpu_wide.py tests/test_abi.py -x -v --timeout 200 --timeout-method thread -p no:cacheprovider > "$OUT/pytest.log" 2>&1
rc=$?; echo "pytest rc=$rc" >> "$OUT/status.txt"; [ $rc -eq 0 ] || stop pytest $rc
echo done >> "$OUT/status.txt"

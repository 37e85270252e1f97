#!/bin/bash
# GPU tests + sweep bench (configs[3]) + selfish bench at configs[2]'s per-GPU share (2^20 / 8 runs).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${1:-sw}
mkdir -p "$OUT"
export TMPDIR=/tmp
stop() { echo "STOP after $1 rc=$2" | tee -a "$OUT/status.txt"; exit "$2"; }
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 180 --timeout-method thread -p no:cacheprovider > "$OUT/pytest_gpu.log" 2>&1
rc=$?; echo "pytest rc=$rc" >> "$OUT/status.txt"; [ $rc -eq 0 ] || stop pytest $rc
timeout -k 10 300 python scripts/bench_sweep.py --runs-per-point 2048 --steps 2 --warmup 1 > "$OUT/bench_sweep.json" 2> "$OUT/bench_sweep.err"
rc=$?; echo "sweep rc=$rc" >> "$OUT/status.txt"; [ $rc -eq 0 ] || stop sweep $rc
timeout -k 10 300 python bench.py --config c3 --runs 131072 --steps 2 --warmup 1 --no-cpu-baseline > "$OUT/bench_c3_131072.json" 2> "$OUT/bench_c3.err"
rc=$?; echo "c3 rc=$rc" >> "$OUT/status.txt"; [ $rc -eq 0 ] || stop c3 $rc
echo done >> "$OUT/status.txt"

#!/bin/bash
# Selfish network (configs[2]) bench at the configs' per-GPU size and at SIM_RUNS, plus the selfish parity tests.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${1:-c3}
mkdir -p "$OUT"
export TMPDIR=/tmp
stop() { echo "STOP after $1 rc=$2" | tee -a "$OUT/status.txt"; exit "$2"; }
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -v --timeout 200 --timeout-method thread -p no:cacheprovider -k "golden or presets or random or sweep or retry or sharding" > "$OUT/pytest.log" 2>&1
rc=$?; echo "pytest rc=$rc" >> "$OUT/status.txt"; [ $rc -eq 0 ] || stop pytest $rc
timeout -k 10 300 python bench.py --config c3 --steps 2 --warmup 1 --no-cpu-baseline > "$OUT/bench_c3.json" 2> "$OUT/bench_c3.err"
rc=$?; echo "bench c3 rc=$rc" >> "$OUT/status.txt"; [ $rc -eq 0 ] || stop bench_c3 $rc
timeout -k 10 300 python bench.py --config c3 --runs 32768 --steps 3 --warmup 1 --no-cpu-baseline > "$OUT/bench_c3_32k.json" 2> "$OUT/bench_c3_32k.err"
rc=$?; echo "bench c3 32k rc=$rc" >> "$OUT/status.txt"; [ $rc -eq 0 ] || stop bench_c3_32k $rc
echo done >> "$OUT/status.txt"

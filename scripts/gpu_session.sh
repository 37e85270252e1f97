#!/bin/bash
# One GPU session: parity tests, bench, rocprofv3 kernel trace. Stops at the first crash/timeout.
#   bash scripts/gpu_session.sh NAME [quick]
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${1:-s1}
mkdir -p "$OUT"
export TMPDIR=/tmp
stop() { echo "STOP after $1 rc=$2" | tee -a "$OUT/status.txt"; exit "$2"; }

timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 180 --timeout-method thread -p no:cacheprovider > "$OUT/pytest_gpu.log" 2>&1
rc=$?; echo "pytest rc=$rc" >> "$OUT/status.txt"; [ $rc -eq 0 ] || [ $rc -eq 1 ] || stop pytest $rc
[ $rc -eq 0 ] || stop pytest-failed $rc

timeout -k 10 300 python bench.py --steps 10 --warmup 2 > "$OUT/bench.json" 2> "$OUT/bench.err"
rc=$?; echo "bench rc=$rc" >> "$OUT/status.txt"; [ $rc -eq 0 ] || stop bench $rc

timeout -k 10 300 python bench.py --config c3 --steps 3 --warmup 1 > "$OUT/bench_c3.json" 2> "$OUT/bench_c3.err"
rc=$?; echo "bench c3 rc=$rc" >> "$OUT/status.txt"; [ $rc -eq 0 ] || stop bench_c3 $rc

timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof" -o run -- python3 bench.py --steps 5 --warmup 1 --no-cpu-baseline > "$OUT/rocprof.log" 2>&1
rc=$?; echo "rocprof rc=$rc" >> "$OUT/status.txt"; [ $rc -eq 0 ] || stop rocprof $rc
echo done >> "$OUT/status.txt"

#!/bin/bash
# Large-network pipeline (configs[4]) on the GPU: parity tests, c5 bench, rocprofv3 kernel trace.
#   bash scripts/gpu_wide.sh NAME
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${1:-w1}
mkdir -p "$OUT"
export TMPDIR=/tmp
stop() { echo "STOP after $1 rc=$2" | tee -a "$OUT/status.txt"; exit "$2"; }
timeout -k 10 400 python -u -m pytest tests/test_gpu_wide.py -x -v --timeout 200 --timeout-method thread -p no:cacheprovider > "$OUT/pytest_wide.log" 2>&1
rc=$?; echo "pytest rc=$rc" >> "$OUT/status.txt"; [ $rc -eq 0 ] || stop pytest $rc
timeout -k 10 300 python bench.py --config c5 --steps 5 --warmup 1 > "$OUT/bench_c5.json" 2> "$OUT/bench_c5.err"
rc=$?; echo "bench c5 rc=$rc" >> "$OUT/status.txt"; [ $rc -eq 0 ] || stop bench_c5 $rc
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof" -o run -- python3 bench.py --config c5 --steps 3 --warmup 1 --no-cpu-baseline > "$OUT/rocprof.log" 2>&1
rc=$?; echo "rocprof rc=$rc" >> "$OUT/status.txt"; [ $rc -eq 0 ] || stop rocprof $rc
echo done >> "$OUT/status.txt"

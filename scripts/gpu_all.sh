#!/bin/bash
# Full GPU session: every GPU parity test, c2 + c5 benches, rocprofv3 kernel traces of both.
#   bash scripts/gpu_all.sh NAME
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${1:-a1}
mkdir -p "$OUT"
export TMPDIR=/tmp
stop() { echo "STOP after $1 rc=$2" | tee -a "$OUT/status.txt"; exit "$2"; }
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread -p no:cacheprovider > "$OUT/pytest_gpu.log" 2>&1
rc=$?; echo "pytest rc=$rc" >> "$OUT/status.txt"; [ $rc -eq 0 ] || stop pytest $rc
timeout -k 10 300 python bench.py --config c5 --steps 5 --warmup 1 > "$OUT/bench_c5.json" 2> "$OUT/bench_c5.err"
rc=$?; echo "bench c5 rc=$rc" >> "$OUT/status.txt"; [ $rc -eq 0 ] || stop bench_c5 $rc
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof_c5" -o run -- python3 bench.py --config c5 --steps 3 --warmup 1 --no-cpu-baseline > "$OUT/rocprof_c5.log" 2>&1
rc=$?; echo "rocprof c5 rc=$rc" >> "$OUT/status.txt"; [ $rc -eq 0 ] || stop rocprof_c5 $rc
timeout -k 10 300 python bench.py --steps 10 --warmup 2 > "$OUT/bench_c2.json" 2> "$OUT/bench_c2.err"
rc=$?; echo "bench c2 rc=$rc" >> "$OUT/status.txt"; [ $rc -eq 0 ] || stop bench_c2 $rc
echo done >> "$OUT/status.txt"

#!/bin/bash
# One GPU session: parity tests, bench, rocprofv3 kernel trace. Stops at the first crash/timeout.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${1:-s1}
mkdir -p "$OUT"
export TMPDIR=/tmp
stop() { echo "STOP after $1 rc=$2" | tee -a "$OUT/status.txt"; exit "$2"; }
ok_or_testfail() { [ "$1" -eq 0 ] || [ "$1" -eq 1 ]; }

timeout -k 10 900 python -m pytest tests -m gpu -x -q -p no:cacheprovider > "$OUT/pytest_gpu.log" 2>&1
rc=$?; echo "pytest rc=$rc" >> "$OUT/status.txt"; ok_or_testfail $rc || stop pytest $rc

timeout -k 10 600 python bench.py --steps 5 --warmup 1 > "$OUT/bench.json" 2> "$OUT/bench.err"
rc=$?; echo "bench rc=$rc" >> "$OUT/status.txt"; [ $rc -eq 0 ] || stop bench $rc

for R in 131072 262144; do
  timeout -k 10 300 python bench.py --steps 3 --warmup 1 --runs $R --no-cpu-baseline > "$OUT/bench_runs$R.json" 2>> "$OUT/bench.err"
  rc=$?; echo "bench runs=$R rc=$rc" >> "$OUT/status.txt"; [ $rc -eq 0 ] || stop bench$R $rc
done

timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof" -o run -- python bench.py --steps 3 --warmup 1 --no-cpu-baseline > "$OUT/rocprof.log" 2>&1
rc=$?; echo "rocprof rc=$rc" >> "$OUT/status.txt"; [ $rc -eq 0 ] || stop rocprof $rc
echo done >> "$OUT/status.txt"

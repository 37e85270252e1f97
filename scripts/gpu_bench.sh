#!/bin/bash
# Bench + rocprofv3 kernel trace (+ optional PMC pass) of the current tree.   bash scripts/gpu_bench.sh NAME
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${1:-b1}
mkdir -p "$OUT"
export TMPDIR=/tmp
stop() { echo "STOP after $1 rc=$2" | tee -a "$OUT/status.txt"; exit "$2"; }
timeout -k 10 300 python bench.py --steps 10 --warmup 2 > "$OUT/bench.json" 2> "$OUT/bench.err"
rc=$?; echo "bench rc=$rc" >> "$OUT/status.txt"; [ $rc -eq 0 ] || stop bench $rc
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof" -o run -- python3 bench.py --steps 5 --warmup 1 --no-cpu-baseline > "$OUT/rocprof.log" 2>&1
rc=$?; echo "rocprof rc=$rc" >> "$OUT/status.txt"; [ $rc -eq 0 ] || stop rocprof $rc
if [ "${PMC:-1}" = 1 ]; then
  timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_LDS SQ_ACTIVE_INST_VALU SQ_INSTS_VMEM_WR --output-format csv -d "$OUT/pmc1" -o pmc -- python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline > "$OUT/pmc1.log" 2>&1
  rc=$?; echo "pmc1 rc=$rc" >> "$OUT/status.txt"; [ $rc -eq 0 ] || stop pmc1 $rc
  timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$OUT/pmc2" -o pmc -- python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline > "$OUT/pmc2.log" 2>&1
  rc=$?; echo "pmc2 rc=$rc" >> "$OUT/status.txt"; [ $rc -eq 0 ] || stop pmc2 $rc
  timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE GRBM_GUI_ACTIVE --output-format csv -d "$OUT/pmc3" -o pmc -- python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline > "$OUT/pmc3.log" 2>&1
  rc=$?; echo "pmc3 rc=$rc" >> "$OUT/status.txt"; [ $rc -eq 0 ] || stop pmc3 $rc
fi
echo done >> "$OUT/status.txt"

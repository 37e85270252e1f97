#!/bin/bash
# Throughput vs runs-per-launch, plus one PMC pass (instruction counts) of the default bench.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${1:-probe}
mkdir -p "$OUT"
export TMPDIR=/tmp
for R in ${RUNS:-32768 131072 524288}; do
  timeout -k 10 300 python bench.py --steps 2 --warmup 1 --runs $R --no-cpu-baseline > "$OUT/bench_runs$R.json" 2>> "$OUT/bench.err" || { echo "bench $R failed rc=$?" >> "$OUT/status.txt"; exit 1; }
  echo "bench $R ok" >> "$OUT/status.txt"
done
timeout -s KILL 240 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_ACTIVE_INST_VALU --output-format csv -d "$OUT/pmc1" -o pmc -- python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline > "$OUT/pmc1.log" 2>&1
echo "pmc1 rc=$?" >> "$OUT/status.txt"

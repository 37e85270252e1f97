#!/bin/bash
# Selfish-network (c3) probe: throughput vs runs per launch, one PMC pass of instruction counts.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${1:-probe_c3}
mkdir -p "$OUT"
export TMPDIR=/tmp
for R in ${RUNS:-32768 131072}; do
  timeout -k 10 300 python bench.py --config c3 --steps 2 --warmup 1 --runs $R --no-cpu-baseline > "$OUT/bench_runs$R.json" 2>> "$OUT/bench.err" || { echo "bench $R failed rc=$?" >> "$OUT/status.txt"; exit 1; }
  echo "bench $R ok" >> "$OUT/status.txt"
done
timeout -s KILL 240 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VMEM_RD SQ_INSTS_SMEM SQ_ACTIVE_INST_VALU --output-format csv -d "$OUT/pmc1" -o pmc -- python3 bench.py --config c3 --steps 1 --warmup 0 --no-cpu-baseline > "$OUT/pmc1.log" 2>&1
echo "pmc1 rc=$?" >> "$OUT/status.txt"
timeout -s KILL 240 rocprofv3 --pmc SQ_THREAD_CYCLES_VALU SQ_INSTS_VMEM_WR SQ_INSTS_SCRATCH_RD SQ_INSTS_SCRATCH_WR GRBM_GUI_ACTIVE --output-format csv -d "$OUT/pmc2" -o pmc -- python3 bench.py --config c3 --steps 1 --warmup 0 --no-cpu-baseline > "$OUT/pmc2.log" 2>&1
echo "pmc2 rc=$?" >> "$OUT/status.txt"

#!/bin/bash
# Round-end refresh: every GPU test, every BASELINE config bench (c2 default, c3, c4 sweep, c5), rocprofv3
# kernel traces (c2, c5) and PMC passes (HBM bytes, VALU counters) for c2 and c5.   bash scripts/gpu_final.sh NAME
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${1:-f1}
mkdir -p "$OUT"
export TMPDIR=/tmp
stop() { echo "STOP after $1 rc=$2" | tee -a "$OUT/status.txt"; exit "$2"; }
run() {  # name timeout cmd...
    local name=$1 t=$2; shift 2
    timeout -k 10 "$t" "$@" > "$OUT/$name.out" 2> "$OUT/$name.err"
    local rc=$?; echo "$name rc=$rc" >> "$OUT/status.txt"; [ $rc -eq 0 ] || stop "$name" $rc
}
run pytest 600 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread -p no:cacheprovider
run bench_c2 300 python bench.py --steps 10 --warmup 2
run bench_c3 300 python bench.py --config c3 --steps 2 --warmup 1
run bench_c5 300 python bench.py --config c5 --steps 5 --warmup 1
run bench_sweep 300 python scripts/bench_sweep.py --runs-per-point 2048 --steps 2 --warmup 1
run prof_c2 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof_c2" -o run -- python3 bench.py --steps 5 --warmup 1 --no-cpu-baseline
run prof_c5 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof_c5" -o run -- python3 bench.py --config c5 --steps 3 --warmup 1 --no-cpu-baseline
for cfg in c2 c5; do
    run pmc_fetch_$cfg 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$OUT/pmc_fetch_$cfg" -o pmc -- python3 bench.py --config $cfg --steps 1 --warmup 0 --no-cpu-baseline
    run pmc_write_$cfg 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$OUT/pmc_write_$cfg" -o pmc -- python3 bench.py --config $cfg --steps 1 --warmup 0 --no-cpu-baseline
    run pmc_sq_$cfg 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_LDS SQ_ACTIVE_INST_VALU SQ_INSTS_VMEM_WR --output-format csv -d "$OUT/pmc_sq_$cfg" -o pmc -- python3 bench.py --config $cfg --steps 1 --warmup 0 --no-cpu-baseline
done
echo done >> "$OUT/status.txt"

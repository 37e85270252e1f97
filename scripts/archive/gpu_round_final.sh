#!/bin/bash
# Round-end evidence in one call: the rehearsal (every GPU test, smoke, bench lines, sweep, rocprof of c2
# serial and c3), then the PMC passes behind the bench line's recorded constants (c2 K1 FETCH_SIZE /
# WRITE_SIZE / instruction mix) and the c3 E1 stall split.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
TAG=${TAG:-final} PROF=1 bash scripts/archive/gpu_rehearsal.sh || exit 1
export TMPDIR=/tmp
O=gpurun_out/${TAG:-final}/pmc; mkdir -p $O
P="python3 bench.py --config c2 --steps 1 --warmup 0 --streams 1 --no-cpu-baseline"
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/pmc_f -o f -- $P > $O/pmc_f.log 2>&1 || { tail -5 $O/pmc_f.log; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/pmc_w -o w -- $P > $O/pmc_w.log 2>&1 || { tail -5 $O/pmc_w.log; exit 1; }
TAG=${TAG:-final}/stalls CFGS="c2 c3" bash scripts/gpu_stalls.sh || exit 1

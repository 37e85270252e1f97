#!/bin/bash
# North-star counters per dominant kernel (VALUBusy, occupancy, VALU utilization / divergence):
# c2 K1, c3 E1 (+D1), c5 W1; one launch each, one pass per config.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/${TAG:-counters}; mkdir -p $O
C="SQ_THREAD_CYCLES_VALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_WAVES SQ_BUSY_CYCLES SQ_INSTS_VALU GRBM_GUI_ACTIVE GRBM_COUNT"
timeout -s KILL 120 rocprofv3 --pmc $C --output-format csv -d $O/c2 -o c2 -- python3 bench.py --config c2 --steps 1 --warmup 0 --streams 1 --no-cpu-baseline > $O/c2.log 2>&1 || { tail -5 $O/c2.log; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc $C --output-format csv -d $O/c3 -o c3 -- python3 scripts/stage_c3.py > $O/c3.log 2>&1 || { tail -5 $O/c3.log; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc $C --output-format csv -d $O/c5 -o c5 -- python3 bench.py --config c5 --steps 1 --warmup 0 --streams 1 --no-cpu-baseline > $O/c5.log 2>&1 || { tail -5 $O/c5.log; exit 1; }
find $O -name "*counter_collection.csv"

#!/bin/bash
# K1 LDS / issue counters (one rocprofv3 --pmc pass per set), c2 serial, one launch.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/${TAG:-k1lds}; mkdir -p $O
timeout -s KILL 60 rocprofv3 -L > $O/counters_list.txt 2>&1 || true
grep -iE "LDS|BANK" $O/counters_list.txt | head -40 > $O/lds_counters.txt || true
P="python3 bench.py --config c2 --steps 1 --warmup 0 --streams 1 --no-cpu-baseline"
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU GRBM_GUI_ACTIVE GRBM_COUNT --output-format csv -d $O/p1 -o p1 -- $P > $O/p1.log 2>&1 || { tail -5 $O/p1.log; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_LDS SQ_BUSY_CYCLES SQ_WAVES SQ_INSTS_SALU --output-format csv -d $O/p2 -o p2 -- $P > $O/p2.log 2>&1 || { tail -5 $O/p2.log; echo "p2 failed"; }
find $O -name "*counter_collection.csv"

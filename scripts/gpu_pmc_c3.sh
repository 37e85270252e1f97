#!/bin/bash
# PMC passes of configs[2] (131072 runs, one launch after a warm-up) for the entity engine.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/${TAG:-pmc}; mkdir -p $O
N=${N:-131072}
timeout -k 10 -s KILL 300 rocprofv3 --kernel-trace --stats -d $O/kt -o kt -- python3 scripts/stage_c3.py $N > $O/kt.log 2>&1 || { tail -20 $O/kt.log; exit 1; }
timeout -k 10 -s KILL 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SMEM SQ_INSTS_BRANCH -d $O/p1 -o p1 -- python3 scripts/stage_c3.py $N > $O/p1.log 2>&1 || { tail -20 $O/p1.log; exit 1; }
timeout -k 10 -s KILL 300 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_THREAD_CYCLES_VALU SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE GRBM_COUNT -d $O/p2 -o p2 -- python3 scripts/stage_c3.py $N > $O/p2.log 2>&1 || { tail -20 $O/p2.log; exit 1; }
timeout -k 10 -s KILL 300 rocprofv3 --pmc SQ_INSTS_VALU_INT32 SQ_INSTS_VALU_INT64 SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_TRANS_F64 SQ_ACTIVE_INST_SCA SQ_INST_CYCLES_VMEM -d $O/p3 -o p3 -- python3 scripts/stage_c3.py $N > $O/p3.log 2>&1 || { tail -20 $O/p3.log; echo "p3 failed (counter names?)"; }
echo done

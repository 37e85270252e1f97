#!/bin/bash
# Issue / stall split of the dominant kernels (c2 K1, c3 E1): instruction counts by type and the disjoint
# wave-cycle buckets (ACTIVE_INST_ANY + WAIT_INST_ANY + WAIT_ANY ~= WAVE_CYCLES, MI355X_MICROARCH.md), plus
# LDS issue stalls and bank conflicts. One rocprofv3 --pmc pass per counter set.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/${TAG:-stalls}; mkdir -p $O
A="SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU"
B="SQ_INSTS_SMEM SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA SQ_INSTS_BRANCH"
for cfg in ${CFGS:-c3 c2}; do
  if [ $cfg = c3 ]; then P="python3 scripts/stage_c3.py"; else P="python3 bench.py --config $cfg --steps 1 --warmup 0 --streams 1 --no-cpu-baseline"; fi
  for set in A B; do
    timeout -s KILL 120 rocprofv3 --pmc ${!set} --output-format csv -d $O/${cfg}_$set -o p -- $P > $O/${cfg}_$set.log 2>&1 || { tail -5 $O/${cfg}_$set.log; echo "pass $cfg $set failed"; [ $set = A ] && exit 1; }
  done
done
find $O -name "*counter_collection.csv"

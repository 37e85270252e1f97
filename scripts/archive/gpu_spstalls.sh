#!/bin/bash
# Issue / stall split of the selfish pipeline's S2 (MSIM_SELPIPE=1, configs[2], one serial step): instruction
# counts by type and the wave-cycle buckets, one rocprofv3 --pmc pass per counter set, then per-kernel sums.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r05/spstalls}; mkdir -p $O
A="SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU"
B="SQ_INSTS_SMEM SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA SQ_INSTS_BRANCH"
P="python3 bench.py --config c3 --steps 1 --warmup 0 --streams 1 --no-cpu-baseline"
for set in A B; do
  MSIM_SELPIPE=1 MSIM_LIB=${LIB:-miningsimulation_amd/libmsim.so} timeout -s KILL 120 rocprofv3 --pmc ${!set} --output-format csv -d $O/c3_$set -o p -- $P > $O/c3_$set.log 2>&1 || { tail -5 $O/c3_$set.log; echo "pass $set failed"; exit 1; }
done
python3 scripts/pmc_csv.py $O/c3_A $O/c3_B --kernel selpipe > $O/pmc_s2.txt 2>&1; cat $O/pmc_s2.txt
python3 scripts/pmc_csv.py $O/c3_A $O/c3_B --kernel draws > $O/pmc_k1.txt 2>&1; cat $O/pmc_k1.txt

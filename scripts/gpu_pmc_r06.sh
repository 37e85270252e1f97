#!/bin/bash
# PMC passes behind the bench line's recorded constants and north_star's counters, per BASELINE workload
# (serial bench, 2 steps = 2 launches; pmc_csv.py sums a pass's counters over its launches):
#   f  FETCH_SIZE                     HBM read bytes (doubled per the gfx950 rule in MI355X_MICROARCH.md)
#   w  WRITE_SIZE                     HBM write bytes
#   s  issue / stall split            SQ_INSTS_VALU/SALU/LDS, SQ_WAVE_CYCLES, SQ_WAIT_ANY, SQ_WAIT_INST_ANY, ...
#   x  VALU instruction mix           FP64 FMA/MUL/ADD/TRANS, INT64, INT32, CVT, all VALU
#   v  VALU busy / utilisation        SQ_ACTIVE_INST_VALU (quad-cycles the VALU works), SQ_THREAD_CYCLES_VALU
#                                     (active-lane cycles: divergence), SQ_BUSY_CYCLES, GRBM_GUI_ACTIVE
# c1 (configs[0]'s 10 s network) is profiled with the others: its dominant kernel is K2.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/${TAG:-pmc06}; mkdir -p $O
S="SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAVES"
X="SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_TRANS_F64 SQ_INSTS_VALU_INT64 SQ_INSTS_VALU_INT32 SQ_INSTS_VALU_CVT SQ_INSTS_VALU"
V="SQ_ACTIVE_INST_VALU SQ_THREAD_CYCLES_VALU SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAVES GRBM_GUI_ACTIVE"
for c in ${CFGS:-c2 c3 c5 c1}; do
  P="python3 bench.py --config $c --steps 2 --warmup 0 --streams 1 --no-cpu-baseline"
  for pass in f w s x v; do
    case $pass in f) C=FETCH_SIZE;; w) C=WRITE_SIZE;; s) C=$S;; x) C=$X;; v) C=$V;; esac
    timeout -s KILL 150 rocprofv3 --pmc $C --output-format csv -d $O/${c}_$pass -o $pass -- $P > $O/${c}_$pass.log 2>&1 || { tail -5 $O/${c}_$pass.log; exit 1; }
  done
  python3 scripts/pmc_csv.py $O/${c}_f $O/${c}_w $O/${c}_s $O/${c}_x $O/${c}_v > $O/pmc_$c.txt
  echo "== $c done"
done

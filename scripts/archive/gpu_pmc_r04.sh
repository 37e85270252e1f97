#!/bin/bash
# PMC passes behind the bench line's recorded constants, per BASELINE workload (serial bench, 2 steps):
# FETCH_SIZE and WRITE_SIZE (separate passes: HBM bytes per launch, FETCH doubled per the gfx950 rule in
# MI355X_MICROARCH.md), and the SQ instruction / wave-cycle set (VALU issue fraction, stall split).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/${TAG:-pmc04}; mkdir -p $O
A="SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAVES"
for c in ${CFGS:-c2 c3 c5}; do
  P="python3 bench.py --config $c --steps 2 --warmup 0 --streams 1 --no-cpu-baseline"
  timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/${c}_f -o f -- $P > $O/${c}_f.log 2>&1 || { tail -5 $O/${c}_f.log; exit 1; }
  timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/${c}_w -o w -- $P > $O/${c}_w.log 2>&1 || { tail -5 $O/${c}_w.log; exit 1; }
  timeout -s KILL 120 rocprofv3 --pmc $A --output-format csv -d $O/${c}_s -o s -- $P > $O/${c}_s.log 2>&1 || { tail -5 $O/${c}_s.log; exit 1; }
  python3 scripts/pmc_csv.py $O/${c}_f $O/${c}_w $O/${c}_s > $O/pmc_$c.txt
  head -30 $O/pmc_$c.txt
done

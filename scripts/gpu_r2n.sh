#!/bin/bash
# A/B of the mixed selfish kernel variants (c3 at 131072 runs, sweep at 2048 runs/point) + SQ counters of c3.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r2n}; mkdir -p $O
for v in default lds8 lds32 reg w1; do
  if [ $v = default ]; then L=miningsimulation_amd/libmsim.so; else L=miningsimulation_amd/variants/libmsim_$v.so; fi
  MSIM_LIB=$L timeout -k 10 120 python -u scripts/stage_c3.py > $O/c3_$v.txt 2>&1 || { cat $O/c3_$v.txt; exit 1; }
  echo "$v $(grep '^c3' $O/c3_$v.txt | cut -c1-200)"
  MSIM_LIB=$L timeout -k 10 120 python -u scripts/stage_sweep.py 2048 > $O/sweep_$v.txt 2>&1 || { cat $O/sweep_$v.txt; exit 1; }
  echo "$v $(grep sweep $O/sweep_$v.txt)"
done
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAVES --output-format csv -d $O/pmc1 -o pmc1 -- python3 scripts/stage_c3.py > $O/pmc1.log 2>&1 || { tail -5 $O/pmc1.log; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_INST_CYCLES_VMEM_RD SQ_WAIT_ANY --output-format csv -d $O/pmc2 -o pmc2 -- python3 scripts/stage_c3.py > $O/pmc2.log 2>&1 || { tail -5 $O/pmc2.log; exit 1; }
find $O -name "*counter_collection.csv" | head

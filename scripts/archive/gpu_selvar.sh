#!/bin/bash
# E1 A/B: the c3 bench line and the configs[3] sweep for each variant library (VARIANTS) and the default.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/${TAG:-selvar}; mkdir -p $O
for v in default $VARIANTS; do
  if [ $v = default ]; then unset MSIM_LIB; else export MSIM_LIB=$PWD/miningsimulation_amd/variants/libmsim_$v.so; fi
  timeout -k 10 200 python -u bench.py --config c3 --no-cpu-baseline > $O/$v.c3.json 2> $O/$v.c3.err || { tail -20 $O/$v.c3.err; exit 1; }
  timeout -k 10 200 python -u scripts/stage_sweep.py ${SWEEP_RPP:-8192} > $O/$v.sweep.txt 2>&1 || { cat $O/$v.sweep.txt; exit 1; }
  python3 -c "import json;d=json.load(open('$O/$v.c3.json'));print('$v c3',d['value'],d['ms_per_step'])"; grep sweep $O/$v.sweep.txt
done

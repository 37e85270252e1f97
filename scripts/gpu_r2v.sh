#!/bin/bash
# E1 engine-phase threshold A/B (SEL_XTH 12 / 16 default / 24 / 32): c3 and the sweep at 8192 runs/point.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r2v}; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -k overlapped -m gpu -x -q --timeout 200 --timeout-method thread > $O/pytest_overlap.log 2>&1 || { tail -30 $O/pytest_overlap.log; exit 1; }
tail -1 $O/pytest_overlap.log
for v in default x12 x24 x32; do
  if [ $v = default ]; then L=miningsimulation_amd/libmsim.so; else L=miningsimulation_amd/variants/libmsim_$v.so; fi
  MSIM_LIB=$L timeout -k 10 120 python -u scripts/stage_c3.py > $O/c3_$v.txt 2>&1 || { cat $O/c3_$v.txt; exit 1; }
  echo "$v $(grep '^c3' $O/c3_$v.txt | cut -c1-130)"
  MSIM_LIB=$L timeout -k 10 200 python -u scripts/stage_sweep.py 8192 > $O/sweep_$v.txt 2>&1 || { cat $O/sweep_$v.txt; exit 1; }
  echo "$v $(grep sweep $O/sweep_$v.txt)"
done

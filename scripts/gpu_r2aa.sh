#!/bin/bash
# Settled-form steps per exit test: 2 (default) vs 1 (variant m1): c3 and the sweep; selfish GPU tests.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r2aa}; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_selfish.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for v in default m1; do
  if [ $v = default ]; then L=miningsimulation_amd/libmsim.so; else L=miningsimulation_amd/variants/libmsim_$v.so; fi
  MSIM_LIB=$L timeout -k 10 120 python -u scripts/stage_c3.py > $O/c3_$v.txt 2>&1 || { cat $O/c3_$v.txt; exit 1; }
  echo "$v $(grep '^c3' $O/c3_$v.txt | cut -c1-130)"
  MSIM_LIB=$L timeout -k 10 200 python -u scripts/stage_sweep.py 8192 > $O/sweep_$v.txt 2>&1 || { cat $O/sweep_$v.txt; exit 1; }
  echo "$v $(grep sweep $O/sweep_$v.txt)"
done

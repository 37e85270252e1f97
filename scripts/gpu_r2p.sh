#!/bin/bash
# Mixed selfish schedule with the mixed retry kernel: selfish GPU parity, c3/sweep timing of the default
# (1,4,1) and (1,2,1) classes, per-wave phase timing (SEL_PROF variant).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r2p}; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_selfish.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
for v in default c121; do
  if [ $v = default ]; then L=miningsimulation_amd/libmsim.so; else L=miningsimulation_amd/variants/libmsim_$v.so; fi
  MSIM_LIB=$L timeout -k 10 120 python -u scripts/stage_c3.py > $O/c3_$v.txt 2>&1 || { cat $O/c3_$v.txt; exit 1; }
  echo "$v $(grep '^c3' $O/c3_$v.txt | cut -c1-200)"
  MSIM_LIB=$L timeout -k 10 120 python -u scripts/stage_sweep.py 2048 > $O/sweep_$v.txt 2>&1 || { cat $O/sweep_$v.txt; exit 1; }
  echo "$v $(grep sweep $O/sweep_$v.txt)"
done
MSIM_LIB=miningsimulation_amd/variants/libmsim_prof.so timeout -k 10 120 python -u scripts/stage_c3.py > $O/c3_prof.txt 2>&1 || { tail $O/c3_prof.txt; exit 1; }
grep SELPROF $O/c3_prof.txt | head -20

#!/bin/bash
# E1 diagnostics on configs[2]: engine-step section cycles (variant engprof) and per-wave phase timing
# (variant selprof).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/${TAG:-e1diag}; mkdir -p $O
for v in engprof selprof; do
  [ -f miningsimulation_amd/variants/libmsim_$v.so ] || continue
  MSIM_LIB=$PWD/miningsimulation_amd/variants/libmsim_$v.so timeout -k 10 120 python -u scripts/stage_c3.py > $O/$v.txt 2>&1 || { tail -20 $O/$v.txt; exit 1; }
  grep -E "ENGPROF|SELPROF" $O/$v.txt | head -8
done

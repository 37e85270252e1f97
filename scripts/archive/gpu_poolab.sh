#!/bin/bash
# E1 pool parameter A/B (MSIM_SEL_POOL="q,lmin,iters") on configs[2] (serial), plus the per-wave schedule
# (variant nopool) as the reference point.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/${TAG:-poolab}; mkdir -p $O
MSIM_LIB=$PWD/miningsimulation_amd/variants/libmsim_nopool.so timeout -k 10 100 python -u scripts/stage_c3.py > $O/nopool.txt 2>&1 || { tail -5 $O/nopool.txt; exit 1; }
echo nopool $(grep -o "'engine_ms': [0-9.]*" $O/nopool.txt)
for p in ${POOLS:-"8,4,8" "16,8,8" "4,2,4" "32,16,8" "64,32,8" "16,16,4" "8,8,2"}; do
  MSIM_SEL_POOL=$p timeout -k 10 100 python -u scripts/stage_c3.py > $O/p_$p.txt 2>&1 || { tail -5 $O/p_$p.txt; exit 1; }
  echo pool $p $(grep -o "'engine_ms': [0-9.]*" $O/p_$p.txt)
done

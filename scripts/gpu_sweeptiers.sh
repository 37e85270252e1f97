#!/bin/bash
# configs[3] sweep A/B of the per-point engine-phase threshold tiers (MSIM_XTH_MID / MSIM_XTH_HI, msim_api.hip
# build_sel_params): the shipped library against variant libraries in VARIANTS, alternating, 2048 runs per point.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/${TAG:-sweeptiers}; mkdir -p $O
for rep in 1 2; do
  for v in base ${VARIANTS}; do
    L=""; [ $v != base ] && L="MSIM_LIB=miningsimulation_amd/variants/libmsim_$v.so"
    env $L timeout -k 10 300 python3 scripts/bench_sweep.py --runs-per-point 2048 --steps 2 --warmup 1 > $O/sweep_${v}_$rep.json 2> $O/sweep_${v}_$rep.err || { tail -5 $O/sweep_${v}_$rep.err; exit 1; }
    python3 -c "import json;d=json.load(open('$O/sweep_${v}_$rep.json'));print('sweep $v $rep',d['value'],d['ms_per_step'])"
  done
done

#!/bin/bash
# configs[3] sweep A/B (round 5): the sweep bench at 8 192 runs per point with MSIM_SEL_XTH in XTHS (every point's
# engine-phase threshold; "tier" = the per-point tiers of msim_api.hip build_sel_params).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r05/sweepxth}; mkdir -p $O
for x in ${XTHS}; do
  E=""; [ $x != tier ] && E="MSIM_SEL_XTH=$x"
  env $E timeout -k 10 300 python3 scripts/bench_sweep.py --runs-per-point 8192 > $O/sweep_$x.json 2> $O/sweep_$x.err || { tail -5 $O/sweep_$x.err; exit 1; }
  python3 -c "import json;d=json.load(open('$O/sweep_$x.json'));print('xth $x',d['value'],d['ms_per_step'])"
done

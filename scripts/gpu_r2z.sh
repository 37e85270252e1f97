#!/bin/bash
# Stream-count A/B for the honest configs (c2, c5): 2 (default) vs 3 overlapping steps.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r2z}; mkdir -p $O
for c in c2 c5; do for st in 2 3; do
  timeout -k 10 300 python -u bench.py --config $c --streams $st --no-cpu-baseline > $O/bench_${c}_s$st.json 2> $O/bench_${c}_s$st.err || { tail -30 $O/bench_${c}_s$st.err; exit 1; }
  python3 -c "import json;d=json.load(open('$O/bench_${c}_s$st.json'));print('$c streams=$st',d['value'],d['ms_per_step'])"
done; done

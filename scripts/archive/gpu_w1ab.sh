#!/bin/bash
# W1 runs-per-workgroup / histogram packing A/B on configs[4] (serial bench lines).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/${TAG:-w1ab}; mkdir -p $O
for cfg in ${W1CFGS:-"auto 1" "1 1" "2 1" "4 1" "8 1" "4 0" "8 0" "2 0"}; do
  set -- $cfg
  if [ $1 = auto ]; then unset MSIM_W1_RUNS; else export MSIM_W1_RUNS=$1; fi
  export MSIM_W1_PACK=$2 MSIM_DEBUG=1
  timeout -k 10 200 python -u bench.py --config c5 --streams 1 --steps 10 --warmup 2 --no-cpu-baseline > $O/r$1p$2.json 2> $O/r$1p$2.err || { tail -20 $O/r$1p$2.err; exit 1; }
  python3 -c "import json;d=json.load(open('$O/r$1p$2.json'));print('runs $1 pack $2',d['value'],d['ms_per_step'],d['roofline']['k1_ms'])"; grep "W1 runs" $O/r$1p$2.err | head -1
done

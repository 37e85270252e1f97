#!/bin/bash
# c2 A/B (round 5): K1 kernel stats of the serial c2 bench for the shipped library and each variant in VARIANTS,
# alternating, twice each (no tests).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r05/c2ab}; mkdir -p $O
for v in default $VARIANTS default $VARIANTS; do
  if [ $v = default ]; then unset MSIM_LIB; else export MSIM_LIB=$PWD/miningsimulation_amd/variants/libmsim_$v.so; fi
  timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/p_$v -o prof -- python3 bench.py --config c2 --streams 1 --no-cpu-baseline > $O/$v.json 2> $O/$v.err || { tail -20 $O/$v.err; exit 1; }
  python3 scripts/rocprof_summary.py $O/p_$v > $O/rocprof_$v.md
  rm -rf $O/p_$v
  echo "== $v $(python3 -c "import json;d=json.load(open('$O/$v.json'));print(d['value'],d['ms_per_step'])")"; grep -E "draws_kernel|episode|combine" $O/rocprof_$v.md
done

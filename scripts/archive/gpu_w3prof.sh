#!/bin/bash
# c5 tail kernels: W3 phase timing (variant w3prof), then rocprof kernel stats of the serial c5 bench for the
# default library and each variant in VARIANTS.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/${TAG:-w3prof}; mkdir -p $O
if [ -f miningsimulation_amd/variants/libmsim_w3prof.so ]; then
  MSIM_LIB=$PWD/miningsimulation_amd/variants/libmsim_w3prof.so timeout -k 10 120 python -u bench.py --config c5 --steps 1 --warmup 0 --streams 1 --no-cpu-baseline > $O/w3.out 2> $O/w3.err || { tail -20 $O/w3.err; exit 1; }
  grep -a W3PROF $O/w3.out | head -8
fi
for v in default $VARIANTS; do
  if [ $v = default ]; then unset MSIM_LIB; else export MSIM_LIB=$PWD/miningsimulation_amd/variants/libmsim_$v.so; fi
  timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/p_$v -o prof -- python3 bench.py --config c5 --streams 1 --steps 6 --warmup 2 --no-cpu-baseline > $O/$v.json 2> $O/$v.err || { tail -20 $O/$v.err; exit 1; }
  python3 scripts/rocprof_summary.py $O/p_$v > $O/rocprof_$v.md
  echo "== $v $(python3 -c "import json;d=json.load(open('$O/$v.json'));print(d['value'],d['ms_per_step'])")"; grep -E "wide" $O/rocprof_$v.md
done

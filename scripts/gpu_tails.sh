#!/bin/bash
# c2 tail kernels (K2 episodes, K3 combine): rocprof kernel stats of the serial bench for the default library
# and each variant in VARIANTS (e.g. K2 occupancy), and K3's phase timing (variant k3prof) when present.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/${TAG:-tails}; mkdir -p $O
if [ -f miningsimulation_amd/variants/libmsim_k3prof.so ]; then
  MSIM_LIB=$PWD/miningsimulation_amd/variants/libmsim_k3prof.so timeout -k 10 120 python -u bench.py --config c2 --steps 1 --warmup 0 --streams 1 --no-cpu-baseline > $O/k3.json 2> $O/k3.err || { tail -20 $O/k3.err; exit 1; }
  grep -a K3PROF $O/k3.json | head -12
fi
for v in default $VARIANTS; do
  if [ $v = default ]; then unset MSIM_LIB; else export MSIM_LIB=$PWD/miningsimulation_amd/variants/libmsim_$v.so; fi
  timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/p_$v -o prof -- python3 bench.py --config c2 --streams 1 --steps 10 --warmup 2 --no-cpu-baseline > $O/$v.json 2> $O/$v.err || { tail -20 $O/$v.err; exit 1; }
  python3 scripts/rocprof_summary.py $O/p_$v > $O/rocprof_$v.md
  echo "== $v $(python3 -c "import json;d=json.load(open('$O/$v.json'));print(d['value'],d['ms_per_step'])")"; grep -E "episode|combine|runs_kernel|draws" $O/rocprof_$v.md
done

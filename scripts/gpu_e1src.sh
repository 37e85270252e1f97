#!/bin/bash
# E1 A/B of the draw source parked in LDS during engine phases (shipped library) against the register-resident
# one (variant library "regsrc", SEL_SRC_LDS=0): selfish GPU tests, then alternating serial c3 bench lines and
# configs[3] sweep steps (2048 runs per point). Output gpurun_out/$TAG.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/${TAG:-e1src}; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_selfish.py tests/test_gpu_parity.py tests/test_selkat.py tests/test_gpu_general.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for rep in 1 2; do
  for v in lds regsrc; do
    if [ $v = lds ]; then L=""; else L="MSIM_LIB=miningsimulation_amd/variants/libmsim_$v.so"; fi
    env $L timeout -k 10 300 python3 bench.py --config c3 --streams 1 --no-cpu-baseline > $O/c3_${v}_$rep.json 2> $O/c3_${v}_$rep.err || { tail -5 $O/c3_${v}_$rep.err; exit 1; }
    python3 -c "import json;d=json.load(open('$O/c3_${v}_$rep.json'));print('c3 $v $rep',d['value'],d['ms_per_step'])"
    env $L timeout -k 10 300 python3 scripts/bench_sweep.py --runs-per-point 2048 --steps 2 --warmup 1 > $O/sweep_${v}_$rep.json 2> $O/sweep_${v}_$rep.err || { tail -5 $O/sweep_${v}_$rep.err; exit 1; }
    python3 -c "import json;d=json.load(open('$O/sweep_${v}_$rep.json'));print('sweep $v $rep',d['value'],d['ms_per_step'])"
  done
done

#!/bin/bash
# Selfish-pipeline S2 diagnostics (round 5): the SP GPU tests, then per variant library named in VARIANTS
# (miningsimulation_amd/variants/libmsim_<name>.so; "main" = the shipped libmsim.so) one c3 step with its SP_PROF
# phase timing (variants built with -DSP_PROF=1) and a rocprof summary of a short c3 bench.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r05/spdiag}; mkdir -p $O
timeout -k 10 600 python -u -m pytest ${PYTEST_FILES:-tests/test_gpu_selpipe.py tests/test_selkat.py} -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for v in ${VARIANTS}; do
L=miningsimulation_amd/variants/libmsim_$v.so; [ $v = main ] && L=miningsimulation_amd/libmsim.so
if [ $v != main ]; then
MSIM_LIB=$L timeout -k 10 300 python3 bench.py --config c3 --steps 1 --warmup 0 --streams 1 --no-cpu-baseline > $O/spprof_$v.txt 2>&1 || { tail -20 $O/spprof_$v.txt; exit 1; }
echo "== $v"; grep SPPROF $O/spprof_$v.txt | head -4
fi
MSIM_LIB=$L timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_$v -o prof -- python3 bench.py --config c3 --steps 3 --warmup 1 --streams 1 --no-cpu-baseline > $O/bench_$v.json 2> $O/bench_$v.err || { tail -20 $O/bench_$v.err; exit 1; }
python3 scripts/rocprof_summary.py $O/prof_$v > $O/rocprof_$v.md && rm -rf $O/prof_$v; head -6 $O/rocprof_$v.md
python3 -c "import json;d=json.load(open('$O/bench_$v.json'));print('$v c3 s1',d['value'],d['ms_per_step'])"
done

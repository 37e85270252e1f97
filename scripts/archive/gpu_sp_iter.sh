#!/bin/bash
# Selfish-pipeline iteration (round 5): its GPU tests, c3 bench lines with rocprof summaries (two streams and
# serial), the SP_PROF phase timing of S2 (variant library), and (CFGS) more configs' bench lines.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r05/sp}; mkdir -p $O
timeout -k 10 600 python -u -m pytest ${PYTEST_FILES:-tests/test_gpu_selpipe.py} -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for c in c3 ${CFGS}; do for st in 0 1; do B=""; [ $st = 1 ] && B="--streams 1"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_${c}_s$st -o prof -- python3 bench.py --config $c $B --no-cpu-baseline > $O/bench_${c}_s$st.json 2> $O/bench_${c}_s$st.err || { tail -20 $O/bench_${c}_s$st.err; exit 1; }
python3 scripts/rocprof_summary.py $O/prof_${c}_s$st > $O/rocprof_${c}_s$st.md && rm -rf $O/prof_${c}_s$st; head -6 $O/rocprof_${c}_s$st.md
python3 -c "import json;d=json.load(open('$O/bench_${c}_s$st.json'));print('$c s$st',d['value'],d['ms_per_step'])"
done; done
if [ -f miningsimulation_amd/variants/libmsim_spprof.so ]; then
MSIM_LIB=miningsimulation_amd/variants/libmsim_spprof.so timeout -k 10 300 python3 bench.py --config c3 --steps 1 --warmup 0 --streams 1 --no-cpu-baseline > $O/spprof.txt 2>&1 || { tail -20 $O/spprof.txt; exit 1; }
grep SPPROF $O/spprof.txt | head -8
fi

#!/bin/bash
# Iteration: selected GPU tests (TESTS), bench lines (BENCHES "cfg streams"), K1 variants (VARIANTS), and a
# rocprofv3 --kernel-trace --stats pass of one bench line (PROF "cfg streams"). Stops at the first failure.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/${TAG:-iter}; mkdir -p $O
if [ -n "$TESTS" ]; then
  timeout -k 10 700 python -u -m pytest $TESTS -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
  tail -1 $O/pytest.log
fi
for spec in $BENCHES; do
  c=${spec%:*}; s=${spec#*:}
  timeout -k 10 300 python -u bench.py --config $c --streams $s --no-cpu-baseline > $O/bench_${c}_s$s.json 2> $O/bench_${c}_s$s.err || { tail -30 $O/bench_${c}_s$s.err; exit 1; }
  python3 -c "import json;d=json.load(open('$O/bench_${c}_s$s.json'));r=d['roofline'];print('$c streams=$s',d['value'],d['ms_per_step'],'kernel',r['kernel_ms'],'k1',r['k1_ms'],'frac',r['frac'])"
done
for v in $VARIANTS; do
  for s in 1 0; do
    MSIM_LIB=$PWD/miningsimulation_amd/variants/libmsim_$v.so timeout -k 10 120 python -u bench.py --config ${VCONFIG:-c2} --streams $s --no-cpu-baseline > $O/$v.s$s.json 2> $O/$v.s$s.err || { tail -20 $O/$v.s$s.err; exit 1; }
    python3 -c "import json;d=json.load(open('$O/$v.s$s.json'));r=d['roofline'];print('$v streams=$s',d['value'],d['ms_per_step'],'k1',r['k1_ms'],'kern',r['kernel_ms'],r['pipeline'].get('segments'),r['pipeline'].get('segment_blocks'))"
  done
done
if [ -n "$PROF" ]; then
  c=${PROF%:*}; s=${PROF#*:}
  [ -n "$PROFLIB" ] && export MSIM_LIB=$PWD/miningsimulation_amd/variants/libmsim_$PROFLIB.so
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o prof -- python3 bench.py --config $c --streams $s --steps 10 --warmup 2 --no-cpu-baseline > $O/prof.log 2>&1 || { tail -20 $O/prof.log; exit 1; }
  python3 scripts/rocprof_summary.py $O/prof | head -8
fi

#!/bin/bash
# Iteration check: the whole GPU suite, then bench lines (c2 serial / default, c3, c5) and an optional
# K1 grid sweep (SLOTS="..."). Stops at the first failure.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/${TAG:-check}; mkdir -p $O
if [ -z "$NOTEST" ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
  tail -1 $O/pytest.log
fi
for spec in ${BENCHES:-"c2 1" "c2 0" "c3 0" "c5 0"}; do
  set -- $spec
  timeout -k 10 300 python -u bench.py --config $1 --streams $2 --no-cpu-baseline > $O/bench_$1_s$2.json 2> $O/bench_$1_s$2.err || { tail -30 $O/bench_$1_s$2.err; exit 1; }
  python3 -c "import json;d=json.load(open('$O/bench_$1_s$2.json'));r=d['roofline'];print('$1 streams=$2',d['value'],d['ms_per_step'],'kernel',r['kernel_ms'],'k1',r['k1_ms'],'frac',r['frac'])"
done
for s in $SLOTS; do
  MSIM_K1_SLOTS=$s timeout -k 10 120 python -u bench.py --config c2 --streams 1 --no-cpu-baseline > $O/slots$s.json 2> $O/slots$s.err || { tail -20 $O/slots$s.err; exit 1; }
  python3 -c "import json;d=json.load(open('$O/slots$s.json'));r=d['roofline'];print('slots $s',d['value'],d['ms_per_step'],'k1',r['k1_ms'])"
done

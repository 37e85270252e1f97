#!/bin/bash
# Selfish-path iteration: selfish GPU tests, the c3 bench line, the configs[3] sweep (words / in-lane).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/${TAG:-sel}; mkdir -p $O
if [ -z "$NOTEST" ]; then
  timeout -k 10 400 python -u -m pytest tests/test_gpu_selfish.py tests/test_gpu_parity.py -m gpu -x -q --timeout 200 --timeout-method thread > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
  tail -1 $O/pytest.log
fi
timeout -k 10 300 python -u bench.py --config c3 --no-cpu-baseline > $O/bench_c3.json 2> $O/bench_c3.err || { tail -30 $O/bench_c3.err; exit 1; }
python3 -c "import json;d=json.load(open('$O/bench_c3.json'));r=d['roofline'];print('c3',d['value'],d['ms_per_step'],'frac',r['frac'])"
for wv in ${SWEEP_WORDS:-1 0}; do
  MSIM_SEL_WORDS=$wv timeout -k 10 300 python -u scripts/stage_sweep.py ${SWEEP_RPP:-8192} > $O/sweep_w$wv.txt 2>&1 || { cat $O/sweep_w$wv.txt; exit 1; }
  echo "words=$wv $(grep sweep $O/sweep_w$wv.txt)"
done

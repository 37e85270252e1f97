#!/bin/bash
# W1 A/B on configs[4]: the wide GPU tests, then the c5 bench line (serial and default) of the default library
# and of each variant in VARIANTS.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/${TAG:-c5ab}; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_wide.py -x -q --timeout 240 --timeout-method thread > $O/pytest_wide.log 2>&1 || { tail -30 $O/pytest_wide.log; exit 1; }
tail -1 $O/pytest_wide.log
for v in default $VARIANTS; do
  if [ $v = default ]; then unset MSIM_LIB; else export MSIM_LIB=$PWD/miningsimulation_amd/variants/libmsim_$v.so; fi
  for s in 1 2; do
    timeout -k 10 200 python -u bench.py --config c5 --streams $s --no-cpu-baseline > $O/$v.c5s$s.json 2> $O/$v.c5s$s.err || { tail -20 $O/$v.c5s$s.err; exit 1; }
    python3 -c "import json;d=json.load(open('$O/$v.c5s$s.json'));print('$v c5 s$s',d['value'],d['ms_per_step'],d['roofline']['k1_ms'])"
  done
done

#!/bin/bash
# A/B of K1 builds (miningsimulation_amd/variants/libmsim_<V>.so via MSIM_LIB): c2 serial and default.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/${TAG:-k1var}; mkdir -p $O
for v in ${VARIANTS:-}; do
  for s in 1 0; do
    MSIM_LIB=$PWD/miningsimulation_amd/variants/libmsim_$v.so timeout -k 10 120 python -u bench.py --config c2 --streams $s --no-cpu-baseline > $O/$v.s$s.json 2> $O/$v.s$s.err || { tail -20 $O/$v.s$s.err; exit 1; }
    python3 -c "import json;d=json.load(open('$O/$v.s$s.json'));r=d['roofline'];print('$v streams=$s',d['value'],d['ms_per_step'],'k1',r['k1_ms'],'kern',r['kernel_ms'],r['pipeline'].get('segments'),r['pipeline'].get('segment_blocks'))"
  done
done

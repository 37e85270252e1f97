#!/bin/bash
# Selfish pipeline (MSIM_SELPIPE=1) A/B on configs[2], serial: the engine-phase threshold (MSIM_SEL_XTH values in
# XTHS) on the shipped library, and the variant libraries in VARIANTS (SP_PROF phase timing + bench line).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp MSIM_SELPIPE=1
O=gpurun_out/${TAG:-r05/spxth}; mkdir -p $O
for x in ${XTHS}; do
  MSIM_SEL_XTH=$x timeout -k 10 300 python3 bench.py --config c3 --steps 3 --warmup 1 --streams 1 --no-cpu-baseline > $O/xth_$x.json 2> $O/xth_$x.err || { tail -5 $O/xth_$x.err; exit 1; }
  python3 -c "import json;d=json.load(open('$O/xth_$x.json'));print('xth $x',d['value'],d['ms_per_step'])"
done
for v in ${VARIANTS}; do
  MSIM_LIB=miningsimulation_amd/variants/libmsim_$v.so timeout -k 10 300 python3 bench.py --config c3 --steps 1 --warmup 0 --streams 1 --no-cpu-baseline > $O/spprof_$v.txt 2>&1 || { tail -20 $O/spprof_$v.txt; exit 1; }
  echo "== $v"; grep SPPROF $O/spprof_$v.txt | head -3
  MSIM_LIB=miningsimulation_amd/variants/libmsim_$v.so timeout -k 10 300 python3 bench.py --config c3 --steps 3 --warmup 1 --streams 1 --no-cpu-baseline > $O/bench_$v.json 2> $O/bench_$v.err || { tail -5 $O/bench_$v.err; exit 1; }
  python3 -c "import json;d=json.load(open('$O/bench_$v.json'));print('$v',d['value'],d['ms_per_step'])"
done

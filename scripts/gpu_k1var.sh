#!/bin/bash
# K1 variant libraries (VARIANTS, scripts/build_variant.sh NAME msim_drawgen.hip ...) against the shipped one on
# c2, two streams and serial, alternating twice. Output gpurun_out/$TAG.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/${TAG:-k1var}; mkdir -p $O
for rep in 1 2; do
  for v in base ${VARIANTS}; do
    L=""; [ $v != base ] && L="MSIM_LIB=miningsimulation_amd/variants/libmsim_$v.so"
    for st in 2 1; do
      env $L timeout -k 10 300 python3 bench.py --config c2 --streams $st --no-cpu-baseline > $O/c2_${v}_s${st}_$rep.json 2> $O/c2_${v}_s${st}_$rep.err || { tail -5 $O/c2_${v}_s${st}_$rep.err; exit 1; }
      python3 -c "import json;d=json.load(open('$O/c2_${v}_s${st}_$rep.json'));r=d['roofline'];print('$v streams $st rep $rep',d['value'],d['ms_per_step'],r['dominant_ms'])"
    done
  done
done

#!/bin/bash
# K1 grid A/B on c2 (serial and two-stream bench lines): the resident-slot count the segment planner assumes
# (MSIM_K1_SLOTS; the shipped value is the occupancy API's), i.e. how many segments per run and rounds of waves.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/${TAG:-k1slots}; mkdir -p $O
for rep in 1 2; do
  for v in ${SLOTS:-default 10240 20480}; do
    for st in 1 2; do
      if [ $v = default ]; then E=""; else E="MSIM_K1_SLOTS=$v"; fi
      env $E timeout -k 10 300 python3 bench.py --config c2 --streams $st --no-cpu-baseline > $O/c2_${v}_s${st}_$rep.json 2> $O/c2_${v}_s${st}_$rep.err || { tail -5 $O/c2_${v}_s${st}_$rep.err; exit 1; }
      python3 -c "import json;d=json.load(open('$O/c2_${v}_s${st}_$rep.json'));r=d['roofline'];print('slots $v streams $st rep $rep',d['value'],d['ms_per_step'],r['dominant_ms'])"
    done
  done
done

#!/bin/bash
# A/B of the K1 grid geometry: MSIM_K1_SLOTS overrides the wave slots pipe_layout_for sizes the
# (run, segment) grid for (segments per run = whole rounds of that many waves).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${TAG:-k1slots}; mkdir -p $O
for s in ${SLOTS:-6144 5120 4096 12288 24576}; do
  MSIM_K1_SLOTS=$s timeout -k 10 120 python -u bench.py --config c2 --streams 1 --steps 10 --warmup 2 --no-cpu-baseline > $O/s$s.json 2> $O/s$s.err || { tail -20 $O/s$s.err; exit 1; }
  python3 -c "import json;d=json.load(open('$O/s$s.json'));r=d['roofline'];print('slots $s',d['value'],d['ms_per_step'],'k1',r['k1_ms'],'nseg',r['pipeline'].get('nseg'),'seg',r['pipeline'].get('seg'))"
done

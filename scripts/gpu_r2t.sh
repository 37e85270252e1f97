#!/bin/bash
# Rehearsal part 2 (after gpu_r2r.sh's tests/smoke/c3 A-B): K1 occupancy A/B, default bench, c3/c5 lines,
# kernel stats of c2 and c3, the configs[3] sweep at 8192 runs/point.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r2t}; mkdir -p $O
for v in k7 k8; do
  MSIM_LIB=miningsimulation_amd/variants/libmsim_$v.so timeout -k 10 300 python -u bench.py --config c2 --no-cpu-baseline > $O/bench_c2_$v.json 2> $O/bench_c2_$v.err || { tail -30 $O/bench_c2_$v.err; exit 1; }
  python3 -c "import json;d=json.load(open('$O/bench_c2_$v.json'));print('c2 $v',d['value'],d['ms_per_step'],d['roofline']['k1_ms'])"
done
timeout -k 10 400 python -u bench.py > $O/bench_default.json 2> $O/bench_default.err || { tail -30 $O/bench_default.err; exit 1; }
cut -c1-300 $O/bench_default.json
for c in c3 c5; do
  timeout -k 10 300 python -u bench.py --config $c --no-cpu-baseline > $O/bench_$c.json 2> $O/bench_$c.err || { tail -30 $O/bench_$c.err; exit 1; }
  python3 -c "import json;d=json.load(open('$O/bench_$c.json'));print('$c',d['value'],d['ms_per_step'],d['roofline'].get('valu_issue_frac_pmc'))"
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_c2 -o c2 -- python3 bench.py --config c2 --no-cpu-baseline > $O/prof_c2.log 2>&1 || { tail -20 $O/prof_c2.log; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_c3 -o c3 -- python3 bench.py --config c3 --no-cpu-baseline > $O/prof_c3.log 2>&1 || { tail -20 $O/prof_c3.log; exit 1; }
timeout -k 10 300 python -u scripts/stage_sweep.py 8192 > $O/sweep8192.txt 2>&1 || { cat $O/sweep8192.txt; exit 1; }
cat $O/sweep8192.txt | grep sweep
find $O -name "*kernel_stats.csv" -exec cut -c1-120 {} \;

#!/bin/bash
# E1 per-wave phase timing (SEL_PROF variant libraries in VARIANTS, built with scripts/build_variant.sh NAME
# msim_sel_kernels.hip "-DSEL_PROF=1 ..."): one short serial c3 bench per variant, the SELPROF lines kept and
# summarised (settled-form cycles per iteration, engine cycles per phase). Output under gpurun_out/$TAG.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/${TAG:-selprof}; mkdir -p $O
for v in ${VARIANTS}; do
  MSIM_LIB=miningsimulation_amd/variants/libmsim_$v.so timeout -k 10 300 python3 bench.py --config c3 --streams 1 --steps 2 --warmup 1 --no-cpu-baseline > $O/bench_$v.json 2> $O/bench_$v.err || { tail -5 $O/bench_$v.err; exit 1; }
  grep SELPROF $O/bench_$v.json $O/bench_$v.err > $O/selprof_$v.txt || true
  python3 - $O/selprof_$v.txt $v <<'PY'
import re, sys
tm = ti = te = tn = tot = 0; lanes = 0
for ln in open(sys.argv[1]):
    m = re.search(r"total (\d+) \| macro phases (\d+) cyc (\d+) iters (\d+) lanes (\d+) \| engine phases (\d+) cyc (\d+) iters (\d+)", ln)
    if m:
        t, pm, cm, im, lm, pe, ce, ie = map(int, m.groups())
        tot += t; tm += cm; ti += im; te += ce; tn += pe; lanes += lm
print(sys.argv[2], "waves-sampled cycles", tot, "settled", tm, "iters", ti, "cyc/iter", round(tm / max(ti, 1)),
      "lanes/iter", round(lanes / max(ti, 1), 1), "| engine", te, "phases", tn, "cyc/phase", round(te / max(tn, 1)))
PY
done

#!/bin/bash
# Memory-side counters of the c2 tail kernels (serial bench, 2 steps): L2 hit rate, and the TCP's L2 read
# requests with their summed latency and its L1 TLB translations, to tell latency from miss handling.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/${TAG:-k3pmc}; mkdir -p $O
P="python3 bench.py --config c2 --steps 2 --warmup 0 --streams 1 --no-cpu-baseline"
timeout -s KILL 90 rocprofv3 --pmc TCP_TCC_READ_REQ_LATENCY_sum TCP_TCC_READ_REQ_sum TCP_UTCL1_TRANSLATION_MISS_sum TCP_UTCL1_TRANSLATION_HIT_sum --output-format csv -d $O/t -o t -- $P > $O/t.log 2>&1 || { tail -5 $O/t.log; exit 1; }
timeout -s KILL 90 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum --output-format csv -d $O/c -o c -- $P > $O/c.log 2>&1 || { tail -5 $O/c.log; exit 1; }
python3 scripts/pmc_csv.py $O/t $O/c > $O/pmc_k23.txt
grep -A6 -E "episode|combine|draws_kernel" $O/pmc_k23.txt

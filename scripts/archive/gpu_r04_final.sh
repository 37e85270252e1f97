#!/bin/bash
# Round-4 final evidence in one call: GPU suite + default bench + rocprof of the exact bench commands
# (gpu_r04_base.sh), smoke, the configs[3] sweep, and the PMC passes behind the bench constants.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
TAG=final bash scripts/archive/gpu_r04_base.sh || exit 1
O=gpurun_out/final
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -30 $O/smoke.log; exit 1; }
tail -3 $O/smoke.log
timeout -k 10 300 python -u scripts/stage_sweep.py 8192 > $O/sweep.txt 2>&1 || { cat $O/sweep.txt; exit 1; }
grep sweep $O/sweep.txt
TAG=final/pmc bash scripts/archive/gpu_pmc_r04.sh > $O/pmc.log 2>&1 || { tail -20 $O/pmc.log; exit 1; }
echo pmc done

#!/bin/bash
# K3 phase timing (variant k3prof, -DK3_PROF=1) on configs[1], serial.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/${TAG:-k3prof}; mkdir -p $O
MSIM_LIB=$PWD/miningsimulation_amd/variants/libmsim_k3prof.so timeout -k 10 120 python -u bench.py --config c2 --steps 1 --warmup 0 --streams 1 --no-cpu-baseline > $O/k3.json 2> $O/k3.err || { tail -20 $O/k3.err; exit 1; }
grep -c K3PROF $O/k3.err; grep K3PROF $O/k3.err | head -12

#!/bin/bash
# A/B variant of libmsim.so with the 9-miner entity-engine kernels rebuilt under extra flags (not shipped):
#   scripts/build_sel_variant.sh NAME "-DSEL_XTH=8 ..."  ->  miningsimulation_amd/variants/libmsim_NAME.so
set -e
cd "$(dirname "$0")/../miningsimulation_amd/csrc"
make -s obj/msim_common.o obj/msim_api.o obj/msim_drawgen.o obj/msim_wide.o obj/msim_multi.o $(for m in $(seq 1 15); do echo obj/msim_kernels_m$m.o obj/msim_sel_kernels_m$m.o; done)
/opt/rocm/bin/hipcc -O3 -std=c++17 --offload-arch=gfx950 -ffp-contract=off -fPIC -Wall -DMSIM_M=9 $2 -c msim_sel_kernels.hip -o obj/sel9_$1.o
OBJS=$(ls obj/*.o | grep -v -e msim_sel_kernels_m9.o -e 'sel9_' -e drawgen_)
mkdir -p ../variants
/opt/rocm/bin/hipcc -shared --offload-arch=gfx950 -fPIC -o ../variants/libmsim_$1.so $OBJS obj/sel9_$1.o -L/opt/rocm/lib -lrccl -Wl,-rpath,/opt/rocm/lib
echo built ../variants/libmsim_$1.so

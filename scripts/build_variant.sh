#!/bin/bash
# A/B variant of libmsim.so with ONE translation unit rebuilt under extra flags (not shipped):
#   scripts/build_variant.sh NAME SOURCE.hip "-DX=1" [MSIM_M]  ->  miningsimulation_amd/variants/libmsim_NAME.so
# SOURCE is a file of miningsimulation_amd/csrc; for msim_kernels.hip / msim_sel_kernels.hip give the miner
# count whose object is replaced (default 9).
set -e
cd "$(dirname "$0")/../miningsimulation_amd/csrc"
make -s -j8
SRC=$2
BASE=${SRC%.hip}
M=${4:-9}
case $BASE in
  msim_kernels|msim_sel_kernels) OBJ=obj/${BASE}_m$M.o; MF="-DMSIM_M=$M" ;;
  *) OBJ=obj/$BASE.o; MF="" ;;
esac
/opt/rocm/bin/hipcc -O3 -std=c++17 --offload-arch=gfx950 -ffp-contract=off -fPIC -Wall $MF $3 -c $SRC -o obj/var_$1.vo
ALL="$(for m in $(seq 1 15); do echo obj/msim_kernels_m$m.o obj/msim_sel_kernels_m$m.o; done) obj/msim_common.o obj/msim_api.o obj/msim_drawgen.o obj/msim_wide.o obj/msim_multi.o obj/msim_general.o"
OBJS=$(for o in $ALL; do [ "$o" = "$OBJ" ] || echo $o; done)
mkdir -p ../variants
/opt/rocm/bin/hipcc -shared --offload-arch=gfx950 -fPIC -o ../variants/libmsim_$1.so $OBJS obj/var_$1.vo -L/opt/rocm/lib -lrccl -Wl,-rpath,/opt/rocm/lib
echo built ../variants/libmsim_$1.so

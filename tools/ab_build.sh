#!/bin/bash
# Builds libslu_mi355x_full.so variants with extra compile flags into
# ablib/NAME/ for A/B runs (bench.py / tests pick one with
# SLU_LIB=ablib/NAME/libslu_mi355x_full.so).  Host objects come from the
# product build (superlu_dist_amd/lib/obj); only engine.hip is recompiled.
# usage: bash tools/ab_build.sh NAME "-DFLAG=..."
set -e
NAME=$1; FLAGS=$2
ROOT=$(cd $(dirname $0)/.. && pwd)
OUT=$ROOT/ablib/$NAME
mkdir -p $OUT/obj
cd $ROOT/superlu_dist_amd/csrc
make -s -j8 >/dev/null
INC="-I../../include -I/opt/conda/include -I."
/opt/rocm/bin/hipcc -O3 -gline-tables-only -fPIC -std=c++17 --offload-arch=gfx950 -munsafe-fp-atomics \
    $INC -Wno-unused-result $FLAGS -c engine.hip -o $OUT/obj/engine.o
HOST=""
for o in abi amalg amalg_grid distribute frontend symbolic ordering amalg_api symbolic_dev; do HOST="$HOST ../lib/obj/$o.o"; done
/opt/rocm/bin/hipcc -shared -fPIC --offload-arch=gfx950 -Wl,--version-script=full.map \
    -o $OUT/libslu_mi355x_full.so $HOST $OUT/obj/engine.o -L/opt/rocm/lib -lamdhip64 -lrccl -ldl \
    -Wl,-rpath,/opt/rocm/lib
echo built $OUT/libslu_mi355x_full.so

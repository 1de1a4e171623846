#!/bin/bash
# Builds libslu_mi355x.so variants with extra compile flags into ablib/NAME/
# for A/B runs (bench.py / tests pick one with SLU_LIB=ablib/NAME/libslu_mi355x.so).
# usage: bash tools/ab_build.sh NAME "-DFLAG=..."
set -e
NAME=$1; FLAGS=$2
ROOT=$(cd $(dirname $0)/.. && pwd)
OUT=$ROOT/ablib/$NAME
mkdir -p $OUT/obj
cd $ROOT/superlu_dist_amd/csrc
INC="-I../../include -I/opt/conda/include -I."
g++ -O3 -fPIC -std=c++17 $INC -I/opt/rocm/include -D__HIP_PLATFORM_AMD__ -c frontend.cpp -o $OUT/obj/frontend.o
g++ -O3 -fPIC -std=c++17 $INC -I/opt/rocm/include -D__HIP_PLATFORM_AMD__ -c abi.cpp -o $OUT/obj/abi.o
/opt/rocm/bin/hipcc -O3 -fPIC -std=c++17 --offload-arch=gfx950 -munsafe-fp-atomics $INC -Wno-unused-result $FLAGS -c engine.hip -o $OUT/obj/engine.o
/opt/rocm/bin/hipcc -shared -fPIC --offload-arch=gfx950 -o $OUT/libslu_mi355x.so $OUT/obj/*.o -L/opt/rocm/lib -lamdhip64 -lrccl -ldl -Wl,-rpath,/opt/rocm/lib
echo built $OUT/libslu_mi355x.so

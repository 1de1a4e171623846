#!/bin/bash
# the rocBLAS dgemm kernel the micro compares against: its Tensile name
# (macro tile, MFMA shape, depth, prefetch, LDS options) and its duration
OUT=gpurun_out/r05_rbname
rm -rf $OUT; mkdir -p $OUT
export TMPDIR=/tmp
cd tools/micro && timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d ../../$OUT/prof -o run -- ./gemm_glds > ../../$OUT/gemm.txt 2>&1; rc=$?
cd ../.. && find $OUT/prof -name "*kernel_stats.csv" | head -1 | xargs cat | cut -c1-400 | head -20
exit $rc

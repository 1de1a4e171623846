#!/bin/bash
# k_schur_big per-tile stamps of one 100^3 factorization for each stamp
# build named (tools/ab_build.sh NAME "-DSLU_SB_STAMP ..."), summarised on
# the box (the raw stamps stay there).  usage: TAG=t LIBS="stamp ..." bash tools/gpu_stamp.sh
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${TAG:-stamp}; mkdir -p $O
for L in ${LIBS:-stamp}; do
  SLU_LIB=ablib/$L/libslu_mi355x_full.so SLU_STAMP_OUT=/tmp/stamps_$L.bin timeout -k 10 300 python -u bench.py --steps 1 --warmup 1 --no-cpu --no-next --no-abi > $O/bench_$L.json 2> $O/bench_$L.err || { tail -20 $O/bench_$L.err; exit 1; }
  timeout -k 10 300 python -u tools/stamp_analyze.py /tmp/stamps_$L.bin > $O/stamps_$L.txt || exit 1
  echo "== $L"; cat $O/stamps_$L.txt
done

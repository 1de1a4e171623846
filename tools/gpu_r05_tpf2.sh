#!/bin/bash
# rocprofv3 kernel stats of the TRSM prefetch build against the TR_PREFETCH=0 build
set -o pipefail
OUT=gpurun_out/r05tpf2
rm -rf $OUT; mkdir -p $OUT
export TMPDIR=/tmp
for v in prod nopf pf16; do
  lib=""; [ $v != prod ] && lib="SLU_LIB=ablib/$v/libslu_mi355x_full.so"
  env $lib timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_$v -o run \
    -- python3 bench.py --no-cpu --roofline-only --warmup 0 > $OUT/prof_$v.json 2> $OUT/prof_$v.err || { echo "FAILED $v"; exit 1; }
  python3 tools/rocprof_summary.py $OUT/prof_$v > $OUT/stats_$v.txt && head -12 $OUT/stats_$v.txt
done

#!/bin/bash
# Round 4: k_diag_strips with 16-byte sc1 hand-offs, the LDS-broadcast panel
# LU and per-column inverses: micro (times, phases, agreement with
# k_diag_lu_f), then the strips parity tests.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r04l; rm -rf $O; mkdir -p $O
for a in "256 1" "256 4" "128 1" "64 1" "200 2"; do
  timeout -k 10 60 ./tools/micro/diag_strips_micro $a 7 >> $O/micro.txt 2>&1 || { cat $O/micro.txt; exit 1; }
done
cat $O/micro.txt
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu \
    tests/test_gpu_parity.py tests/test_refdump.py -k "strips" > $O/tests.log 2>&1 \
    || { tail -40 $O/tests.log; exit 1; }
tail -2 $O/tests.log

#!/bin/bash
# Round 4: diag strips micro only.
set -o pipefail
O=gpurun_out/r04c; mkdir -p $O; rm -f $O/micro.txt
for a in "256 1" "256 4" "128 1" "64 1"; do
  timeout -k 10 60 ./tools/micro/diag_strips_micro $a 5 >> $O/micro.txt 2>&1 || { echo "FAIL $a rc=$?" >> $O/micro.txt; cat $O/micro.txt; exit 1; }
done
cat $O/micro.txt

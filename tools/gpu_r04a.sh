#!/bin/bash
# Round 4: multi-workgroup diagonal LU micro (k_diag_strips vs k_diag_lu_f).
set -o pipefail
O=gpurun_out/r04a; mkdir -p $O
for a in "256 1" "256 4" "256 16" "224 1" "192 2" "128 1" "100 3" "64 1" "40 2"; do
  timeout -k 10 60 ./tools/micro/diag_strips_micro $a 5 >> $O/micro.txt 2>&1 || { echo "FAIL $a rc=$?" >> $O/micro.txt; cat $O/micro.txt; exit 1; }
done
cat $O/micro.txt

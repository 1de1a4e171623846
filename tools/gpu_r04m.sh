#!/bin/bash
# Round 4: k_diag_strips A/B micro (current vs batched inverse reads)
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r04m; rm -rf $O; mkdir -p $O
for b in diag_strips_micro diag_strips_micro_batch diag_strips_micro_batch2; do
  for a in "256 1" "64 1"; do
    echo "== $b $a" >> $O/micro.txt
    timeout -k 10 60 ./tools/micro/$b $a 7 >> $O/micro.txt 2>&1 || { cat $O/micro.txt; exit 1; }
  done
done
cat $O/micro.txt

#!/bin/bash
# Cold drop-in first calls at 100^3 with the fresh-HBM mapping order as is and
# with the coarse storage's touch after the caller-layout buffers' (SLU_MAP_ORDER=1).
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/$1; mkdir -p $O
for i in 1 2; do
  for mo in 0 1; do
    SLU_MAP_ORDER=$mo SUPERLU_MI355X_TIMING=1 SLU_PROFILE_PLAN=1 timeout -k 10 300 python -u tools/dropin_cold.py 100 \
        > $O/mo$mo.$i.json 2> $O/mo$mo.$i.err || { tail -5 $O/mo$mo.$i.err; exit 1; }
    echo "map_order $mo: $(cat $O/mo$mo.$i.json)"
  done
done

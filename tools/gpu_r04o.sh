#!/bin/bash
# Round 4: where the drop-in's plan build goes (cold process, 100^3), twice.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r04o; rm -rf $O; mkdir -p $O
for i in 1 2; do
SUPERLU_MI355X_TIMING=1 SLU_AMALG_TIME=1 SLU_PROFILE_PLAN=1 timeout -k 10 600 python -u tools/dropin_cold.py 100 > $O/cold$i.json 2> $O/cold$i.err || { tail -20 $O/cold$i.err; exit 1; }
cat $O/cold$i.json; grep -E "PDGSTRF|slu amalg|slu plan" $O/cold$i.err
done

#!/bin/bash
# First-call breakdown of the drop-in device-resident leg at 100^3: for each
# SUPERLU_MI355X_DEFER_A setting in DEFERS (default "1"), the timing of
# pdgstrf's phases and (SLU_PROFILE_PLAN) of its plan build.
set -o pipefail
O=gpurun_out/${TAG:-devres_ab}; mkdir -p $O
for d in ${DEFERS:-1}; do
SLU_PROFILE_PLAN=1 SUPERLU_MI355X_DEFER_A=$d SUPERLU_MI355X_TIMING=1 timeout -k 10 400 python -u bench.py --device-resident-child --nx 100 > $O/devres_$d.json 2> $O/devres_$d.err || { tail -30 $O/devres_$d.err; exit 1; }
echo "== DEFER_A=$d"; grep -v "^\[slu rank" $O/devres_$d.err | head -80; cat $O/devres_$d.json
done

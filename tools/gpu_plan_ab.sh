#!/bin/bash
# One GPU session: host first-touch micro (4 KB vs huge pages), two cold
# drop-in first calls at 100^3 with the plan-build phase ticks, then the
# Schur-kernel A/B builds named on the command line (tools/ab_bench.sh).
# usage: bash tools/gpu_plan_ab.sh TAG [NAME...]
set -o pipefail
export TMPDIR=/tmp
TAG=$1; shift
O=gpurun_out/$TAG; mkdir -p $O
timeout -k 10 120 tools/micro/thp_micro 16 > $O/thp_micro.txt 2>&1 || exit 1
for i in 1 2; do
  SUPERLU_MI355X_TIMING=1 SLU_PROFILE_PLAN=1 SLU_AMALG_TIME=1 timeout -k 10 300 python -u tools/dropin_cold.py 100 \
      > $O/cold$i.json 2> $O/cold$i.err || { tail -5 $O/cold$i.err; exit 1; }
  cat $O/cold$i.json
done
[ $# -gt 0 ] && bash tools/ab_bench.sh $TAG/ab "$@"
exit 0

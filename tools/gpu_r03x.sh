#!/bin/bash
# Round 3: 16-byte B loads in k_schur_big by default -- the whole GPU suite,
# an A/B of 16-byte A loads (ablib/a16, -DSLU_SB_A16), then the 100^3
# drop-in with the timing breakdown.
set -o pipefail
export TMPDIR=/tmp
T=${1:-r03x}; O=gpurun_out/$T; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
    > $O/pytest_gpu.log 2>&1; rc=$?; tail -3 $O/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
bash tools/ab_bench.sh ${T}_ab a16 || exit 1
bash tools/dropin_solve_n100.sh ${T}_solve100

#!/bin/bash
# k_schur_pers (SLU_SB_PERSIST=1): GPU parity tests with it on, then the
# 100^3 bench A/B against k_schur_big
set -o pipefail
OUT=gpurun_out/${1:-r05p}
rm -rf $OUT; mkdir -p $OUT
export TMPDIR=/tmp
SLU_SB_PERSIST=1 timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_amalg.py tests/test_grid_lifecycle.py -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/pytest_pers.log 2>&1; rc=$?
tail -3 $OUT/pytest_pers.log; grep -E "FAILED|Error" $OUT/pytest_pers.log | head -5
[ $rc -ne 0 ] && exit $rc
bash tools/ab_env.sh ${1:-r05p}/ab "big:SLU_SB_PERSIST=0" "pers:SLU_SB_PERSIST=1"

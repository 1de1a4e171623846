#!/bin/bash
# TRSM prefetch only on the levels with few slabs (SLU_TRSM_PF): parity with
# it forced everywhere, then A/B on 100^3
set -o pipefail
OUT=gpurun_out/r05tpf3
rm -rf $OUT; mkdir -p $OUT
export TMPDIR=/tmp
SLU_TRSM_PF=1000000 timeout -k 10 700 python -u -m pytest tests/test_gpu_parity.py tests/test_amalg.py tests/test_gpu_fill.py tests/test_gpu_solve.py -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1; rc=$?
tail -3 $OUT/pytest.log; grep -E "FAILED|Error" $OUT/pytest.log | head -5
[ $rc -ne 0 ] && exit $rc
bash tools/ab_env.sh r05tpf3/ab "f:SLU_TRSM_PF=0" "p256:SLU_TRSM_PF=256" "p600:SLU_TRSM_PF=600"

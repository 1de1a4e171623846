#!/bin/bash
# k_diag_strips received-panel staging depth (DS_TU 16 vs 32): parity with the
# variant (strips forced on every level), then A/B on 100^3
set -o pipefail
OUT=gpurun_out/r05ds
rm -rf $OUT; mkdir -p $OUT
export TMPDIR=/tmp
SLU_LIB=ablib/ds32/libslu_mi355x_full.so SLU_DIAG_STRIPS=2 timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py -m gpu -k "not reference_structure and not dropin" -x -q --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1; rc=$?
tail -3 $OUT/pytest.log; grep -E "FAILED|Error" $OUT/pytest.log | head -5
[ $rc -ne 0 ] && exit $rc
bash tools/ab_env.sh r05ds/ab "f:SLU_REST_SPLIT=30" "ds32:SLU_LIB=ablib/ds32/libslu_mi355x_full.so"
timeout -k 10 300 python -u bench.py --no-cpu --no-abi --no-next --steps 1 --warmup 1 --level-log > $OUT/lv_f.json 2> $OUT/lv_f.err && \
SLU_LIB=ablib/ds32/libslu_mi355x_full.so timeout -k 10 300 python -u bench.py --no-cpu --no-abi --no-next --steps 1 --warmup 1 --level-log > $OUT/lv_ds32.json 2> $OUT/lv_ds32.err

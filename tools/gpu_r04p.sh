#!/bin/bash
# Round 4: the streamed upload of cached refactorizations: parity (plan cache
# tests, drop-in tests), then the drop-in leg and D2H knob runs at 100^3.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r04p; rm -rf $O; mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu \
    tests/test_gpu_parity.py tests/test_dropin.py tests/test_amalg.py -k "cache or dropin or amalg or refactor" > $O/tests.log 2>&1 \
    || { tail -40 $O/tests.log; exit 1; }
tail -2 $O/tests.log
SUPERLU_MI355X_TIMING=1 timeout -k 10 600 python -u tools/d2h_variants.py 100 > $O/var.txt 2> $O/var.err || { tail -20 $O/var.err; exit 1; }
cat $O/var.txt; grep -E "^rep|PDGSTRF" $O/var.err | head -12
SUPERLU_MI355X_TIMING=1 SUPERLU_MI355X_STREAM=0 timeout -k 10 600 python -u tools/dropin_cold.py 100 > $O/cold_nostream.json 2> $O/cold_nostream.err || { tail -20 $O/cold_nostream.err; exit 1; }
cat $O/cold_nostream.json
SUPERLU_MI355X_TIMING=1 timeout -k 10 600 python -u tools/dropin_cold.py 100 > $O/cold.json 2> $O/cold.err || { tail -20 $O/cold.err; exit 1; }
cat $O/cold.json; grep PDGSTRF $O/cold.err

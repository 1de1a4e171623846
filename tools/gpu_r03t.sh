#!/bin/bash
# Round 3: device-resident build in libslu_mi355x_solve.so (pddistribute keeps
# A, pdgstrf fills on the device, the factors stay in HBM for pdgstrs) --
# drop-in tests, then the 100^3 drop-in run.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${1:-r03t}; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_dropin.py -m gpu -v -s --timeout 300 -k "solve or reentry or factorization" \
    --timeout-method thread > $O/pytest.log 2>&1; rc=$?
grep -E "pddrive|psdrive|pzdrive|passed|failed" $O/pytest.log | cut -c1-300 | tail -40
[ $rc -eq 0 ] || exit $rc
bash tools/dropin_solve_n100.sh ${1:-r03t}_solve100

#!/bin/bash
# Round 3: the drop-in tests after the s / z distribute fix.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${1:-r03o}; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_dropin.py -m gpu -v -s --timeout 300 \
    --timeout-method thread > $O/pytest.log 2>&1; rc=$?
grep -E "pddrive|psdrive|pzdrive|passed|failed" $O/pytest.log | cut -c1-300 | tail -60; exit $rc

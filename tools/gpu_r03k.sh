#!/bin/bash
# Round 3: pdgstrf3d drop-in (reference pddrive3d with our pdgstrf3d) + the
# 3D engine tests + the 2D drop-in regressions.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${1:-r03k}; mkdir -p $O
timeout -k 10 800 python -u -m pytest tests/test_dropin.py tests/test_grid3d.py -m gpu -v -s --timeout 300 \
    --timeout-method thread > $O/pytest.log 2>&1; rc=$?; grep -E "pddrive|passed|failed" $O/pytest.log | tail -70; exit $rc

#!/bin/bash
# Round 3: drop-in tests (pdgstrf, pdgstrs on the device factors, pdgstrf3d
# with the reference's pddrive3d) + 3D engine tests, then the 100^3 solve
# drop-in measurement.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${1:-r03m}; mkdir -p $O
timeout -k 10 700 python -u -m pytest tests/test_dropin.py tests/test_grid3d.py -m gpu -v -s --timeout 300 \
    --timeout-method thread > $O/pytest.log 2>&1; rc=$?
grep -E "pddrive|psdrive|pzdrive|passed|failed" $O/pytest.log | tail -80
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
bash tools/dropin_solve_n100.sh ${1:-r03m}_solve100

#!/bin/bash
# Round 4: diag strips micro, then the grid GPU tests (grid amalgamation:
# reference-structure fingerprints on 2x2 / 2x4, the oracle / fixture grid
# suites through the coarse path, the grid solve tests, the 2x2 drop-in
# drivers).
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r04b; mkdir -p $O
for a in "256 1" "256 4" "128 1" "64 1"; do
  timeout -k 10 60 ./tools/micro/diag_strips_micro $a 5 >> $O/micro.txt 2>&1 || { echo "FAIL $a rc=$?" >> $O/micro.txt; cat $O/micro.txt; exit 1; }
done
cat $O/micro.txt
timeout -k 10 1200 python -u -m pytest tests/test_grid.py tests/test_solve_ref.py tests/test_refdump.py -m gpu -x -v \
    --timeout 600 --timeout-method thread > $O/pytest_grid.log 2>&1; rc=$?
tail -25 $O/pytest_grid.log; exit $rc

#!/bin/bash
# Round 3: 3D grids (pdgstrf3d) -- the 3D tests on one GPU (host p2p
# transport), the 2D grid regressions, the 1x1 parity subset.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${1:-r03j}; mkdir -p $O
timeout -k 10 500 python -u -m pytest tests/test_grid3d.py -m gpu -x -v --timeout 240 --timeout-method thread \
    > $O/pytest_3d.log 2>&1; rc=$?; tail -3 $O/pytest_3d.log; [ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 500 python -u -m pytest tests/test_grid.py tests/test_gpu_parity.py -m gpu -x -q --timeout 240 \
    --timeout-method thread > $O/pytest_reg.log 2>&1; tail -3 $O/pytest_reg.log
grep -q " passed" $O/pytest_3d.log && ! grep -q "failed" $O/pytest_3d.log && \
timeout -k 10 400 python -u tools/model3d.py --nx 100 --pz 2,4,8 > $O/model3d.json 2> $O/model3d.err && cat $O/model3d.json

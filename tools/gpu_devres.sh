#!/bin/bash
# Drop-in device-resident checks: the solve-library tests (reference
# drivers, eviction, grids, the device-resident system), then the 100^3
# first-call breakdown (SLU_DIST_TIME).  usage: TAG=t bash tools/gpu_devres.sh
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${TAG:-devres}; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_dropin.py -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest_dropin.log 2>&1 || { tail -40 $O/pytest_dropin.log; exit 1; }
tail -3 $O/pytest_dropin.log
SLU_DIST_TIME=1 timeout -k 10 400 python -u bench.py --device-resident-child --nx 100 > $O/devres.json 2> $O/devres.err || { tail -30 $O/devres.err; exit 1; }
grep -E "pxdistribute|distribute\]" $O/devres.err | head -30
cat $O/devres.json

#!/bin/bash
# small rest tiles beside the big ones: parity tests, then A/B on 100^3 and 2D 1000^2
set -o pipefail
OUT=gpurun_out/${1:-r05r2s}
rm -rf $OUT; mkdir -p $OUT
export TMPDIR=/tmp
SLU_REST_2STREAM=1 timeout -k 10 700 python -u -m pytest tests/test_gpu_parity.py tests/test_amalg.py tests/test_gpu_fill.py tests/test_gpu_solve.py -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1; rc=$?
tail -3 $OUT/pytest.log; grep -E "FAILED|Error" $OUT/pytest.log | head -5
[ $rc -ne 0 ] && exit $rc
for round in 1 2; do
  for v in 0 1; do
    SLU_REST_2STREAM=$v timeout -k 10 300 python -u bench.py --workload lap2d --nx 1000 --no-cpu --no-abi --no-next --steps 5 > $OUT/lap2d_$v.$round.json 2> $OUT/lap2d_$v.$round.err || exit 1
    python3 -c "import json; d=json.load(open('$OUT/lap2d_$v.$round.json')); print('lap2d wave=$v round $round', d['ms_per_step'])"
  done
done
bash tools/ab_env.sh ${1:-r05r2s}/ab "f:SLU_REST_2STREAM=0" "w:SLU_REST_2STREAM=1"

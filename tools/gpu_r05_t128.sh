#!/bin/bash
set -o pipefail
OUT=gpurun_out/${1:-r05t128}
rm -rf $OUT; mkdir -p $OUT
export TMPDIR=/tmp
SLU_TRSM_NARROW=2 timeout -k 10 700 python -u -m pytest tests/test_gpu_parity.py tests/test_amalg.py -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1; rc=$?
tail -2 $OUT/pytest.log; [ $rc -ne 0 ] && exit $rc
for round in 1 2; do
  for v in 1 2; do
    SLU_TRSM_NARROW=$v timeout -k 10 300 python -u bench.py --workload lap2d --nx 1000 --no-cpu --no-abi --no-next --steps 5 > $OUT/lap2d_$v.$round.json 2> $OUT/lap2d_$v.$round.err || exit 1
    python3 -c "import json; d=json.load(open('$OUT/lap2d_$v.$round.json')); print('lap2d narrow=$v round $round', d['ms_per_step'])"
  done
done
bash tools/ab_env.sh ${1:-r05t128}/ab "n1:SLU_TRSM_NARROW=1" "n2:SLU_TRSM_NARROW=2"

#!/bin/bash
# K split of root-level Schur tiles (SLU_KSPLIT_TILES): parity with it forced on, then A/B
set -o pipefail
OUT=gpurun_out/${1:-r05ks}
rm -rf $OUT; mkdir -p $OUT
export TMPDIR=/tmp
SLU_KSPLIT_TILES=100000 timeout -k 10 700 python -u -m pytest tests/test_gpu_parity.py tests/test_amalg.py tests/test_gpu_solve.py -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1; rc=$?
tail -2 $OUT/pytest.log; grep -E "FAILED|Error" $OUT/pytest.log | head -3; [ $rc -ne 0 ] && exit $rc
for round in 1 2; do
  for v in 0 128 256; do
    SLU_KSPLIT_TILES=$v timeout -k 10 300 python -u bench.py --workload lap2d --nx 1000 --no-cpu --no-abi --no-next --steps 5 > $OUT/lap2d_$v.$round.json 2> $OUT/lap2d_$v.$round.err || exit 1
    python3 -c "import json; d=json.load(open('$OUT/lap2d_$v.$round.json')); print('lap2d ksplit=$v round $round', d['ms_per_step'])"
  done
done
bash tools/ab_env.sh ${1:-r05ks}/ab "k0:SLU_KSPLIT_TILES=0" "k128:SLU_KSPLIT_TILES=128" "k256:SLU_KSPLIT_TILES=256"

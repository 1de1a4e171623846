#!/bin/bash
# pipelined k_schur (small tiles): parity, lap2d and 100^3 factor-only timings, lap2d level log
set -o pipefail
OUT=gpurun_out/${1:-r05sc}
rm -rf $OUT; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 700 python -u -m pytest tests/test_gpu_parity.py tests/test_amalg.py tests/test_gpu_solve.py tests/test_grid.py -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1; rc=$?
tail -2 $OUT/pytest.log; grep -E "FAILED|Error" $OUT/pytest.log | head -3; [ $rc -ne 0 ] && exit $rc
for round in 1 2; do
  timeout -k 10 300 python -u bench.py --workload lap2d --nx 1000 --no-cpu --no-abi --no-next --steps 5 > $OUT/lap2d.$round.json 2> $OUT/lap2d.$round.err || exit 1
  python3 -c "import json; d=json.load(open('$OUT/lap2d.$round.json')); print('lap2d round $round', d['ms_per_step'])"
  timeout -k 10 300 python -u bench.py --steps 3 --warmup 1 --no-cpu --no-next --no-abi > $OUT/n100.$round.json 2> $OUT/n100.$round.err || exit 1
  python3 -c "import json; d=json.load(open('$OUT/n100.$round.json')); print('n100 round $round', d['ms_per_step'], d['roofline']['frac'])"
done
timeout -k 10 300 python -u bench.py --workload lap2d --nx 1000 --no-cpu --no-abi --no-next --level-log --steps 3 > $OUT/lap2d_lv.json 2> $OUT/lap2d_lv.err

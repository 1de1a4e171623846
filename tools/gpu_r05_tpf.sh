#!/bin/bash
# TRSM register prefetch of the next block (TR_PREFETCH): parity tests, then
# A/B against a TR_PREFETCH=0 build on 100^3 and 2D 1000^2, and a level log
set -o pipefail
OUT=gpurun_out/${1:-r05tpf}
rm -rf $OUT; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 700 python -u -m pytest tests/test_gpu_parity.py tests/test_amalg.py tests/test_gpu_fill.py tests/test_gpu_solve.py -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1; rc=$?
tail -3 $OUT/pytest.log; grep -E "FAILED|Error" $OUT/pytest.log | head -5
[ $rc -ne 0 ] && exit $rc
for round in 1 2; do
  for v in prod nopf; do
    lib=""; [ $v != prod ] && lib="SLU_LIB=ablib/$v/libslu_mi355x_full.so"
    env $lib timeout -k 10 300 python -u bench.py --no-cpu --no-abi --no-next --steps 3 --warmup 1 > $OUT/n100_$v.$round.json 2> $OUT/n100_$v.$round.err || { echo "FAILED $v"; exit 1; }
    env $lib timeout -k 10 300 python -u bench.py --workload lap2d --nx 1000 --no-cpu --no-abi --no-next --steps 5 > $OUT/lap2d_$v.$round.json 2> $OUT/lap2d_$v.$round.err || { echo "FAILED $v"; exit 1; }
    python3 -c "import json; a=json.load(open('$OUT/n100_$v.$round.json')); b=json.load(open('$OUT/lap2d_$v.$round.json')); print('$v round $round: n100', a['ms_per_step'], 'serial', a['roofline']['serial_factor_ms'], 'trsm span', a['phases_ms_per_step_rank0']['trsm'], '| lap2d', b['ms_per_step'])"
  done
done
timeout -k 10 300 python -u bench.py --no-cpu --no-abi --no-next --steps 1 --warmup 1 --level-log > $OUT/n100_levels.json 2> $OUT/n100_levels.err

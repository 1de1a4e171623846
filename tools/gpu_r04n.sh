#!/bin/bash
# Round 4: k_diag_strips (branch-free full-width LU) micro + strips tests, then
# the bulk stream's CU reservation A/B on the 100^3 factorization.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r04n; rm -rf $O; mkdir -p $O
for a in "256 1" "256 4" "128 1" "64 1" "200 2"; do
  timeout -k 10 60 ./tools/micro/diag_strips_micro $a 7 >> $O/micro.txt 2>&1 || { cat $O/micro.txt; exit 1; }
done
grep -v "^  strips" $O/micro.txt; grep "strips phases" $O/micro.txt | head -2
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu \
    tests/test_gpu_parity.py tests/test_refdump.py -k "strips" > $O/tests.log 2>&1 \
    || { tail -40 $O/tests.log; exit 1; }
tail -2 $O/tests.log
for r in 0 1 2 0 1 2; do
  SLU_SCHUR_CU_RESERVE=$r timeout -k 10 300 python -u bench.py --steps 5 --warmup 2 --no-cpu --no-next > $O/bench_$r.json 2> $O/bench_$r.err || { tail -20 $O/bench_$r.err; exit 1; }
  python3 -c "import json; d=json.load(open('$O/bench_$r.json')); print('reserve $r', d['ms_per_step'], d.get('phases_ms_per_step_rank0'), d['roofline']['frac'])"
done

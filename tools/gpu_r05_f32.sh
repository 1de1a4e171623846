#!/bin/bash
# fp32 Schur tile configurations on C5 (st27 120^3, psgstrf), factor only
set -o pipefail
OUT=gpurun_out/r05f32
rm -rf $OUT; mkdir -p $OUT
export TMPDIR=/tmp
for round in 1 2; do
  for v in prod bk16m4 bk32m4 bk32m6; do
    lib=""; [ $v != prod ] && lib="SLU_LIB=ablib/$v/libslu_mi355x_full.so"
    env $lib timeout -k 10 400 python -u bench.py --workload st27 --nx 120 --no-cpu --no-abi --no-next --steps 3 --warmup 1 > $OUT/$v.$round.json 2> $OUT/$v.$round.err || { echo "FAILED $v"; tail -3 $OUT/$v.$round.err; exit 1; }
    python3 -c "import json; d=json.load(open('$OUT/$v.$round.json')); print('$v round $round', d['ms_per_step'], 'frac', d['roofline']['frac'])"
  done
done

#!/bin/bash
# TRSM staging depth (TR_TU) A/B: 100^3 and lap2d, factor only
set -o pipefail
OUT=gpurun_out/r05tu
rm -rf $OUT; mkdir -p $OUT
export TMPDIR=/tmp
for round in 1 2; do
  for v in prod tu16 tu32; do
    lib=""; [ $v != prod ] && lib="SLU_LIB=ablib/$v/libslu_mi355x_full.so"
    env $lib timeout -k 10 300 python -u bench.py --no-cpu --no-abi --no-next --steps 3 --warmup 1 > $OUT/n100_$v.$round.json 2> $OUT/n100_$v.$round.err || { echo "FAILED $v"; exit 1; }
    env $lib timeout -k 10 300 python -u bench.py --workload lap2d --nx 1000 --no-cpu --no-abi --no-next --steps 5 > $OUT/lap2d_$v.$round.json 2> $OUT/lap2d_$v.$round.err || { echo "FAILED $v"; exit 1; }
    python3 -c "import json; a=json.load(open('$OUT/n100_$v.$round.json')); b=json.load(open('$OUT/lap2d_$v.$round.json')); print('$v round $round: n100', a['ms_per_step'], 'serial', a['roofline']['serial_factor_ms'], 'trsm span', a['phases_ms_per_step_rank0']['trsm'], '| lap2d', b['ms_per_step'])"
  done
done

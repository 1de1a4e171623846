#!/bin/bash
# A/B of engine builds on the GPU box: the 100^3 bench (factor only) for the
# product library ("base") and each ablib/NAME/libslu_mi355x.so, two rounds
# interleaved (box clocks drift).  usage: bash tools/ab_bench.sh TAG NAME...
set -o pipefail
export TMPDIR=/tmp
TAG=$1; shift
O=gpurun_out/$TAG; mkdir -p $O
for round in 1 2; do
  for v in base "$@"; do
    lib=""; [ "$v" != base ] && lib=ablib/$v/libslu_mi355x_full.so
    SLU_LIB=$lib timeout -k 10 300 python -u bench.py --steps 3 --warmup 1 --no-cpu --no-next --no-abi \
        > $O/$v.$round.json 2> $O/$v.$round.err || { echo "FAILED $v"; tail -5 $O/$v.$round.err; exit 1; }
    python -c "import json; d=json.load(open('$O/$v.$round.json')); r=d['roofline']; print('$v round $round: ms_per_step', d['ms_per_step'], 'frac', r['frac'], 'launch_ms', r['avg_launch_ms'], 'serial', r['serial_factor_ms'])"
  done
done

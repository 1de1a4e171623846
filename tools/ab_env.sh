#!/bin/bash
# A/B of engine settings given as environment assignments, on the 100^3
# bench (factor only), two interleaved rounds.
# usage: bash tools/ab_env.sh TAG "NAME1:VAR=val VAR2=val" "NAME2:..." ...
set -o pipefail
export TMPDIR=/tmp
TAG=$1; shift
O=gpurun_out/$TAG; mkdir -p $O
for round in 1 2; do
  for spec in "$@"; do
    name=${spec%%:*}; envs=${spec#*:}
    env $envs timeout -k 10 300 python -u bench.py --steps 3 --warmup 1 --no-cpu --no-next --no-abi \
        > $O/$name.$round.json 2> $O/$name.$round.err || { echo "FAILED $name"; tail -5 $O/$name.$round.err; exit 1; }
    python -c "import json; d=json.load(open('$O/$name.$round.json')); r=d['roofline']; print('$name round $round: ms_per_step', d['ms_per_step'], 'frac', r['frac'], 'serial', r['serial_factor_ms'])"
  done
done

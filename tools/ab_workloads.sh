#!/bin/bash
# A/B of the product library against ablib/NAME on every bench workload.
# usage: bash tools/ab_workloads.sh TAG NAME
set -o pipefail
export TMPDIR=/tmp
TAG=$1; V=$2
O=gpurun_out/$TAG; mkdir -p $O
for w in st27 lap2d helm3d; do
  for v in base $V; do
    lib=""; [ "$v" != base ] && lib=ablib/$v/libslu_mi355x.so
    SLU_LIB=$lib timeout -k 10 400 python -u bench.py --workload $w --steps 3 --warmup 1 --no-next --no-abi \
        > $O/$w.$v.json 2> $O/$w.$v.err || { echo "FAILED $w $v"; tail -5 $O/$w.$v.err; exit 1; }
    python -c "import json; d=json.load(open('$O/$w.$v.json')); r=d['roofline']; print('$w $v', d['ms_per_step'], d['value'], r['frac'], r['serial_factor_ms'])"
  done
done

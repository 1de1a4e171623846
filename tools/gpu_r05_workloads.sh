#!/bin/bash
# The other BASELINE configs on one GPU (factor only): C2 lap2d 1000^2, C4 helm3d 80^3 (complex),
# C5 st27 120^3 (fp32)
set -o pipefail
OUT=gpurun_out/${1:-r05wl}
rm -rf $OUT; mkdir -p $OUT
export TMPDIR=/tmp
for w in "lap2d --nx 1000" "helm3d --nx 80" "st27 --nx 120"; do
  name=${w%% *}
  timeout -k 10 400 python -u bench.py --workload $w --no-cpu --no-abi --steps 3 --warmup 1 > $OUT/$name.json 2> $OUT/$name.err || { echo "FAILED $name"; tail -5 $OUT/$name.err; exit 1; }
  python3 -c "import json; d=json.load(open('$OUT/$name.json')); print('$name', d['ms_per_step'], d['value'], d['unit'], d['dtype'], 'frac', d['roofline']['frac'])"
done

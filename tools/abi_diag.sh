#!/bin/bash
# Diagnostics of the drop-in path's overlapped D2H (bench.py abi leg
# breakdown under the SLU_D2H_* knobs of engine.hip).  GPU box only.
set -o pipefail
OUT=gpurun_out/${1:-abi_diag}
mkdir -p $OUT
export SLU_ABI_BREAKDOWN_ONLY=1
for cfg in "base:" "after:SLU_D2H_AFTER=1" "push:SLU_D2H_MODE=push" "pushafter:SLU_D2H_MODE=push SLU_D2H_AFTER=1"; do
  name=${cfg%%:*}; envs=${cfg#*:}
  env $envs timeout -k 10 300 python -u bench.py --no-cpu --no-next --steps 1 --warmup 1 > $OUT/$name.json 2> $OUT/$name.err || exit 1
  python -c "import json,sys;d=json.load(open('$OUT/$name.json'));print('$name', json.dumps(d['abi_pdgstrf']['breakdown_ms']))"; grep 'slu d2h' $OUT/$name.err || true
done

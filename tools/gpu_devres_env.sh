#!/bin/bash
# The device-resident first call (standalone child) under each env setting
# in ENVS, twice each, with pdgstrf's timing line.  usage: ENVS="A=1 A=0" bash tools/gpu_devres_env.sh
set -o pipefail
O=gpurun_out/${TAG:-devres_env}; mkdir -p $O
for rep in 1 2; do
for e in ${ENVS:-X=0}; do
  n=$(echo "$e" | tr '/=' '_-')
  env $e SUPERLU_MI355X_TIMING=1 timeout -k 10 400 python -u bench.py --device-resident-child --nx 100 > $O/devres_${n}_$rep.json 2> $O/devres_${n}_$rep.err || { tail -20 $O/devres_${n}_$rep.err; exit 1; }
  python3 -c "import json,re; d=json.load(open('$O/devres_${n}_$rep.json')); t=open('$O/devres_${n}_$rep.err').read(); m=re.search(r'plan built ([0-9.]+) ms \(amalg ([0-9.]+)', t); print('$e rep $rep symbolic', d['symbolic_s'], 'dist', d['calls'][0]['distribute_ms'], 'utime', d['calls'][0]['utime_fact_ms'], 'plan', m.group(1), 'amalg', m.group(2))"
done
done

#!/bin/bash
# The device-resident first call as bench.py runs it (a child of the bench
# process, after the headline and drop-in legs), with its timing breakdowns.
set -o pipefail
O=gpurun_out/${TAG:-devres_ctx}; mkdir -p $O
SUPERLU_MI355X_TIMING=1 SLU_PROFILE_PLAN=1 SLU_DIST_TIME=1 SLU_BENCH_CHILD_ERR=$O/child.err \
  timeout -k 10 600 python -u bench.py --no-cpu > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
grep -v "^\[slu rank" $O/child.err | grep -E "PDGSTRF|amalg plan\] (analysis|coarse|programs)|distribute\]|pxdistribute" | head -40
python3 -c "import json; d=json.load(open('$O/bench.json')); print(json.dumps(d['abi_pdgstrf']['device_resident']['calls'][0]))"

#!/bin/bash
# Round 4: the D2H slots warmed beside the plan build: drop-in / cache parity,
# then the cold-process first call at 100^3 (twice) and the bench's drop-in leg.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r04r; rm -rf $O; mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu \
    tests/test_gpu_parity.py tests/test_dropin.py -k "cache or dropin or abi" > $O/tests.log 2>&1 \
    || { tail -40 $O/tests.log; exit 1; }
tail -2 $O/tests.log
for i in 1 2; do
SUPERLU_MI355X_TIMING=1 SLU_PROFILE_PLAN=1 timeout -k 10 600 python -u tools/dropin_cold.py 100 > $O/cold$i.json 2> $O/cold$i.err || { tail -20 $O/cold$i.err; exit 1; }
cat $O/cold$i.json; grep -E "PDGSTRF|slu d2h" $O/cold$i.err
done
timeout -k 10 600 python -u bench.py --steps 2 --warmup 1 --no-cpu --no-next > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
python3 -c "import json; d=json.load(open('$O/bench.json')); print(d['abi_pdgstrf']); print(d['value'], d['ms_per_step'])"

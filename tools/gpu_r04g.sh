#!/bin/bash
# Round 4: where the drop-in pdgstrf's first call spends its time at 100^3
# (SUPERLU_MI355X_TIMING / SLU_AMALG_TIME / SLU_PROFILE_PLAN breakdowns).
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r04g; mkdir -p $O
SUPERLU_MI355X_TIMING=1 SLU_AMALG_TIME=1 SLU_PROFILE_PLAN=1 timeout -k 10 600 python -u bench.py --steps 2 --warmup 1 --no-cpu --no-next \
    > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
grep -E "slu amalg|slu plan|PDGSTRF|slu d2h|amalg" $O/bench.err > $O/summary.txt || true; head -c 6000 $O/summary.txt
python -c "import json; d=json.load(open('$O/bench.json')); print(d['abi_pdgstrf'])"

#!/bin/bash
# Round 4: compact U relayout program + faster analysis + shallow digest:
# parity of the relayout paths, then the drop-in first-call breakdown at 100^3.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r04h; mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu \
    tests/test_gpu_parity.py tests/test_grid.py tests/test_amalg.py tests/test_dropin.py > $O/tests.log 2>&1 \
    || { tail -40 $O/tests.log; exit 1; }
tail -3 $O/tests.log
SUPERLU_MI355X_TIMING=1 SLU_AMALG_TIME=1 SLU_PROFILE_PLAN=1 timeout -k 10 600 python -u bench.py --steps 2 --warmup 1 --no-cpu --no-next \
    > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
grep -E "slu amalg|slu plan|PDGSTRF|slu d2h" $O/bench.err > $O/summary.txt || true; head -c 8000 $O/summary.txt
python -c "import json; d=json.load(open('$O/bench.json')); print(d['abi_pdgstrf']); print(d['value'], d['ms_per_step'])"

#!/bin/bash
# Round 4: fresh-HBM allocation cost, the drop-in's first call in a cold
# process, the relayout / cache parity tests, and the bench's drop-in leg.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r04i; mkdir -p $O
timeout -k 10 120 ./tools/micro/alloc_micro > $O/alloc.txt 2>&1 || { cat $O/alloc.txt; exit 1; }
cat $O/alloc.txt
SUPERLU_MI355X_TIMING=1 SLU_PROFILE_PLAN=1 timeout -k 10 600 python -u tools/dropin_cold.py 100 > $O/cold.json 2> $O/cold.err || { tail -20 $O/cold.err; exit 1; }
cat $O/cold.json; grep -E "PDGSTRF|slu amalg plan|layout \+ alloc" $O/cold.err
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu \
    tests/test_gpu_parity.py tests/test_amalg.py -k "amalg or cache or dropin" > $O/tests.log 2>&1 \
    || { tail -40 $O/tests.log; exit 1; }
tail -2 $O/tests.log
SUPERLU_MI355X_TIMING=1 SLU_PROFILE_PLAN=1 timeout -k 10 600 python -u bench.py --steps 2 --warmup 1 --no-cpu --no-next \
    > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
grep -E "slu amalg plan|layout \+ alloc|PDGSTRF" $O/bench.err > $O/summary.txt || true; cat $O/summary.txt
python -c "import json; d=json.load(open('$O/bench.json')); print(d['abi_pdgstrf']); print(d['value'], d['ms_per_step'])"

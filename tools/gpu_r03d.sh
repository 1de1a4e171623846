#!/bin/bash
# Round 3: small-width diagonal LU variant (parity + bench), and where the
# drop-in path's time goes on the amalgamated plan.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${1:-r03d}; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_refdump.py -m gpu -x -v \
    --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 && tail -2 $O/pytest.log && \
timeout -k 10 400 python -u bench.py --no-cpu --no-abi --no-next > $O/bench.json 2> $O/bench.err && cat $O/bench.json && \
SLU_PROFILE_PLAN=1 timeout -k 10 300 python -u tools/abi_amalg_diag.py > $O/diag.json 2> $O/diag.err && cat $O/diag.json && \
SLU_PROFILE_PLAN=1 SLU_D2H_PRIO=hi timeout -k 10 300 python -u tools/abi_amalg_diag.py > $O/diag_hi.json 2> $O/diag_hi.err && cat $O/diag_hi.json
grep "slu d2h" $O/diag.err $O/diag_hi.err

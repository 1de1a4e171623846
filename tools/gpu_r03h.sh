#!/bin/bash
# Round 3: chunked U relayout -- the whole GPU suite, the drop-in
# diagnostics, then the default bench line (CPU baseline + full-size parity).
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${1:-r03h}; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread \
    > $O/pytest_gpu.log 2>&1 && tail -2 $O/pytest_gpu.log && \
SLU_PROFILE_PLAN=1 timeout -k 10 300 python -u tools/abi_amalg_diag.py 100 0,1,1 > $O/diag.json 2> $O/diag.err && cat $O/diag.json && \
grep "slu d2h" $O/diag.err && \
timeout -k 10 900 python -u bench.py > $O/bench.json 2> $O/bench.err && cat $O/bench.json

#!/bin/bash
# Round 3: wave-per-row U relayout -- parity of the amalgamated paths, then
# the drop-in diagnostics.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${1:-r03e}; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_refdump.py tests/test_dropin.py -m gpu -x -v \
    --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 && tail -2 $O/pytest.log && \
SLU_PROFILE_PLAN=1 timeout -k 10 300 python -u tools/abi_amalg_diag.py > $O/diag.json 2> $O/diag.err && cat $O/diag.json
grep "slu d2h" $O/diag.err

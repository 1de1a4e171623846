#!/bin/bash
# Round 3: flattened U relayout -- amalgamation parity, drop-in diagnostics
# with the relayout kernels profiled.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${1:-r03g}; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_refdump.py tests/test_dropin.py -m gpu -x -v \
    --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 && tail -2 $O/pytest.log && \
SLU_PROFILE_PLAN=1 timeout -k 10 300 python -u tools/abi_amalg_diag.py 100 0,1,1 > $O/diag.json 2> $O/diag.err && cat $O/diag.json && \
grep "slu d2h" $O/diag.err && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_diag -o run \
    -- python3 tools/abi_amalg_diag.py 100 0,1 > $O/diag_prof.json 2> $O/diag_prof.err && cat $O/diag_prof.json

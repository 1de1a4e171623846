#!/bin/bash
# Round 3: diag LU trailing update transposed (coalesced A22 loads / stores)
# -- parity suites that run the diagonal kernel, then the bench line.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${1:-r03r}; mkdir -p $O
timeout -k 10 700 python -u -m pytest tests/test_gpu_parity.py tests/test_refdump.py tests/test_grid.py -m gpu -x -q \
    --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 && tail -2 $O/pytest.log && \
timeout -k 10 300 python -u bench.py --no-cpu --no-abi --no-next > $O/bench.json 2> $O/bench.err && cut -c1-1200 $O/bench.json

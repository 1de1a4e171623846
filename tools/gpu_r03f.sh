#!/bin/bash
# Round 3: K-loop loads issued ahead of the MFMAs (branch-free LDS-store
# masks) -- parity, bench, kernel stats; relayout kernel times.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${1:-r03f}; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_refdump.py -m gpu -x -v \
    --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 && tail -2 $O/pytest.log && \
timeout -k 10 400 python -u bench.py --no-cpu --no-abi --no-next > $O/bench.json 2> $O/bench.err && cat $O/bench.json && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run \
    -- python3 bench.py --no-cpu --roofline-only --warmup 0 > $O/prof_bench.json 2> $O/prof.err && \
timeout -s KILL 300 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE --kernel-trace --output-format csv -d $O/pmc_mfma -o run \
    -- python3 bench.py --no-cpu --roofline-only --warmup 0 > $O/pmc_mfma.json 2> $O/pmc_mfma.err && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_diag -o run \
    -- python3 tools/abi_amalg_diag.py 100 0,1 > $O/diag.json 2> $O/diag.err && cat $O/diag.json

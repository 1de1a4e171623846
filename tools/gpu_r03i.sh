#!/bin/bash
# Round 3: pipelined staging loops in the diagonal LU / TRSM kernels --
# factor parity subset, bench line (no CPU leg), kernel-time summary.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${1:-r03i}; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_dropin.py -m gpu -x -v \
    --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 && tail -2 $O/pytest.log && \
timeout -k 10 300 python -u bench.py --no-cpu --no-abi --no-next > $O/bench.json 2> $O/bench.err && cat $O/bench.json && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run \
    -- python3 bench.py --no-cpu --no-abi --no-next --steps 2 --warmup 1 > $O/bench_prof.json 2> $O/bench_prof.err && \
python3 tools/rocprof_summary.py $O/prof > $O/stats.txt 2>/dev/null; head -12 $O/stats.txt

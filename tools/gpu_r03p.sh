#!/bin/bash
# Round 3 evidence: the whole GPU suite, then rocprofv3 kernel statistics and
# the PMC passes (FETCH_SIZE / WRITE_SIZE / MFMA busy) of the roofline step.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${1:-r03p}; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
    > $O/pytest_gpu.log 2>&1 && tail -2 $O/pytest_gpu.log && \
bash tools/gpu_round_b.sh ${1:-r03p}

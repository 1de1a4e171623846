#!/bin/bash
# Round 3: the headline on the reference's own symbolic structure.
# GPU parity of the new cases, then the bench on both structures.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${1:-refs}; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -v --timeout 300 --timeout-method thread \
    -k "reference_structure" > $O/pytest.log 2>&1 && tail -3 $O/pytest.log && \
timeout -k 10 900 python -u bench.py --level-log > $O/bench_ref.json 2> $O/bench_ref.err && cat $O/bench_ref.json && \
timeout -k 10 300 python -u bench.py --symbolic frontend --no-cpu --no-next --no-abi > $O/bench_fe.json 2> $O/bench_fe.err && cat $O/bench_fe.json

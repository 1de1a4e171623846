#!/bin/bash
# Round-end evidence, part 1: the whole GPU suite and the default bench line
# (CPU baseline + full-size parity included).
set -o pipefail
TAG=${1:-run}; shift
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
echo "== pytest -m gpu" && \
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread \
    > $OUT/pytest_gpu.log 2>&1 && tail -3 $OUT/pytest_gpu.log && \
echo "== bench" && \
timeout -k 10 900 python -u bench.py "$@" > $OUT/bench.json 2> $OUT/bench.err && cat $OUT/bench.json

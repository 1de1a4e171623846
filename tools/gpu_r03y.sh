#!/bin/bash
# Round 3 evidence with the 16-byte A and B loads in k_schur_big: the whole
# GPU suite, the default bench line (with its CPU baseline), then rocprofv3
# statistics + PMC passes of the roofline step.
set -o pipefail
export TMPDIR=/tmp
T=${1:-r03y}; O=gpurun_out/$T; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
    > $O/pytest_gpu.log 2>&1; rc=$?; tail -3 $O/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -u bench.py > $O/bench.json 2> $O/bench.err || { tail -5 $O/bench.err; exit 1; }
cut -c1-400 $O/bench.json
bash tools/gpu_round_b.sh $T

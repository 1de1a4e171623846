#!/bin/bash
# Round 3: per-level breakdown of the 100^3 factorization (pipelined step and
# the serialized roofline step), for the critical-path analysis.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${1:-r03q}; mkdir -p $O
timeout -k 10 400 python -u bench.py --no-cpu --no-abi --no-next --level-log --steps 1 --warmup 1 \
    > $O/bench.json 2> $O/level.log && cat $O/bench.json | cut -c1-400 && grep -c "slu rank" $O/level.log

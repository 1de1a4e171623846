#!/bin/bash
# Round 5 GPU session b: grid life cycle + grid suites, the 2x2 host-transport
# rehearsal with the parity preflight, the 100^3 level log, symbfact timing on
# the box's host against the reference, the graph ordering on the reference
# structure.  Each GPU step has its own limit; steps chained with &&.
set -o pipefail
OUT=gpurun_out/${1:-r05b}
rm -rf $OUT; mkdir -p $OUT
export TMPDIR=/tmp
echo "== symbfact timing (host)" && \
timeout -k 10 300 python -u tools/symb_timing.py 100 > $OUT/symb_timing_100.jsonl 2> $OUT/symb_timing.err && \
cat $OUT/symb_timing_100.jsonl && \
echo "== pytest (grid life cycle, grids)" && \
timeout -k 10 700 python -u -m pytest tests/test_dropin.py tests/test_grid.py -m gpu -x -v --timeout 300 \
    --timeout-method thread -k "evicts or grid_matches or fingerprints or device_resident" > $OUT/pytest_gpu.log 2>&1 && \
tail -3 $OUT/pytest_gpu.log && \
echo "== 2x2 host-transport rehearsal with parity preflight" && \
timeout -k 10 400 python -u bench.py --gpus 4 --host-transport --nx 40 --steps 2 --warmup 1 \
    > $OUT/rehearse_n4.json 2> $OUT/rehearse_n4.err && cat $OUT/rehearse_n4.json && \
echo "== bench 100^3 level log" && \
timeout -k 10 400 python -u bench.py --no-cpu --no-abi --no-next --level-log --steps 1 --warmup 1 \
    > $OUT/bench_levels.json 2> $OUT/bench_levels.err && \
echo "== bench 100^3 graph ordering, reference structure" && \
timeout -k 10 500 python -u bench.py --ordering graph --no-cpu --no-abi --no-next --steps 2 --warmup 1 \
    > $OUT/bench_graph.json 2> $OUT/bench_graph.err && cat $OUT/bench_graph.json && \
echo "== done"

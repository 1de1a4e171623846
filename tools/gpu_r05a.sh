#!/bin/bash
# Round 5 first GPU session: the new grid life-cycle test, the grid suites,
# the 2x2 host-transport rehearsal with the parity preflight, and a 100^3
# bench with the per-level log (pipelined and serialized).
set -o pipefail
OUT=gpurun_out/${1:-r05a}
rm -rf $OUT; mkdir -p $OUT
export TMPDIR=/tmp
echo "== pytest (grid life cycle, grids)" && \
timeout -k 10 600 python -u -m pytest tests/test_dropin.py tests/test_grid.py -m gpu -x -v --timeout 300 \
    --timeout-method thread -k "evicts or grid_matches or fingerprints" > $OUT/pytest_gpu.log 2>&1 && \
tail -3 $OUT/pytest_gpu.log && \
echo "== 2x2 host-transport rehearsal with parity preflight" && \
timeout -k 10 400 python -u bench.py --gpus 4 --host-transport --nx 40 --steps 2 --warmup 1 \
    > $OUT/rehearse_n4.json 2> $OUT/rehearse_n4.err && cat $OUT/rehearse_n4.json && \
echo "== bench 100^3 level log" && \
timeout -k 10 400 python -u bench.py --no-cpu --no-abi --no-next --level-log --steps 1 --warmup 1 \
    > $OUT/bench_levels.json 2> $OUT/bench_levels.err && cat $OUT/bench_levels.json && \
echo "== done"

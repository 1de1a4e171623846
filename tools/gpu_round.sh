#!/bin/bash
# One GPU-box session: parity tests, bench line, rocprofv3 kernel stats and
# the HBM-traffic PMC passes for the dominant kernel.  Every GPU step has its
# own time limit; the steps are chained with && so the first failure ends it.
# usage: bash tools/gpu_round.sh TAG [bench args...]
set -o pipefail
TAG=${1:-run}; shift
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
echo "== pytest -m gpu" && \
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread \
    > $OUT/pytest_gpu.log 2>&1 && tail -3 $OUT/pytest_gpu.log && \
echo "== bench" && \
timeout -k 10 600 python -u bench.py "$@" > $OUT/bench.json 2> $OUT/bench.err && cat $OUT/bench.json && \
echo "== rocprofv3 kernel stats" && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o run \
    -- python3 bench.py --no-cpu --roofline-only --warmup 0 "$@" > $OUT/prof_bench.json 2> $OUT/prof.err && \
echo "== pmc FETCH_SIZE" && \
timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d $OUT/pmc_fetch -o run \
    -- python3 bench.py --no-cpu --roofline-only --warmup 0 "$@" > $OUT/pmc_fetch.json 2> $OUT/pmc_fetch.err && \
echo "== pmc WRITE_SIZE" && \
timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d $OUT/pmc_write -o run \
    -- python3 bench.py --no-cpu --roofline-only --warmup 0 "$@" > $OUT/pmc_write.json 2> $OUT/pmc_write.err && \
echo "== pmc MFMA busy" && \
timeout -s KILL 300 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE --kernel-trace --output-format csv -d $OUT/pmc_mfma -o run \
    -- python3 bench.py --no-cpu --roofline-only --warmup 0 "$@" > $OUT/pmc_mfma.json 2> $OUT/pmc_mfma.err && \
echo "== done"

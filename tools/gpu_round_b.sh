#!/bin/bash
# Round-end evidence, part 2: rocprofv3 kernel statistics and the PMC passes
# (FETCH_SIZE, WRITE_SIZE, MFMA busy) of the serialized roofline step.
set -o pipefail
TAG=${1:-run}; shift
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
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

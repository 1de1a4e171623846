#!/bin/bash
# End-of-round GPU session: the whole GPU suite, the bench line,
# rocprofv3 kernel statistics, the HBM-traffic and MFMA-busy PMC passes of the
# dominant kernel, and their summaries into profiles/ (TAG prefix).  Every GPU
# step has its own time limit and the steps are chained with &&.
# usage: [SKIP_TESTS=1] bash tools/gpu_round.sh TAG [bench args...]
set -o pipefail
TAG=${1:-r06z}; shift
OUT=gpurun_out/$TAG
rm -rf $OUT; mkdir -p $OUT
export TMPDIR=/tmp
{ [ "$SKIP_TESTS" = 1 ] || { echo "== pytest -m gpu" && \
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread \
    > $OUT/pytest_gpu.log 2>&1 && tail -3 $OUT/pytest_gpu.log; }; } && \
echo "== bench" && \
timeout -k 10 600 python -u bench.py "$@" > $OUT/bench.json 2> $OUT/bench.err && cat $OUT/bench.json && \
echo "== rocprofv3 kernel stats" && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o run \
    -- python3 bench.py --no-cpu --roofline-only --warmup 0 "$@" > $OUT/prof_bench.json 2> $OUT/prof.err && \
python3 tools/rocprof_summary.py $OUT/prof > $OUT/rocprof_stats.txt && head -20 $OUT/rocprof_stats.txt && \
echo "== pmc FETCH_SIZE" && \
timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d $OUT/pmc_fetch -o run \
    -- python3 bench.py --no-cpu --roofline-only --warmup 0 "$@" > $OUT/pmc_fetch.json 2> $OUT/pmc_fetch.err && \
echo "== pmc WRITE_SIZE" && \
timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d $OUT/pmc_write -o run \
    -- python3 bench.py --no-cpu --roofline-only --warmup 0 "$@" > $OUT/pmc_write.json 2> $OUT/pmc_write.err && \
python3 tools/pmc_traffic.py $OUT/pmc_fetch $OUT/pmc_write $OUT/pmc_traffic.txt && head -12 $OUT/pmc_traffic.txt && \
echo "== pmc MFMA busy" && \
timeout -s KILL 300 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE --kernel-trace --output-format csv -d $OUT/pmc_mfma -o run \
    -- python3 bench.py --no-cpu --roofline-only --warmup 0 "$@" > $OUT/pmc_mfma.json 2> $OUT/pmc_mfma.err && \
python3 tools/pmc_mfma.py $OUT/pmc_mfma k_schur_big $OUT/pmc_mfma_busy.txt && cat $OUT/pmc_mfma_busy.txt && \
rm -rf $OUT/prof $OUT/pmc_fetch $OUT/pmc_write $OUT/pmc_mfma && \
echo "== done"

#!/bin/bash
# Round 3: the amalgamated plan (csrc/amalg.h) -- the whole GPU suite, then
# the headline bench on the reference's structure.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${1:-amalg}; mkdir -p $O
nproc > $O/nproc.txt; lscpu > $O/lscpu.txt 2>&1
timeout -k 10 700 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread \
    > $O/pytest.log 2>&1; rc=$?; tail -3 $O/pytest.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
SLU_AMALG_TIME=1 timeout -k 10 1000 python -u bench.py > $O/bench_ref.json 2> $O/bench_ref.err && cat $O/bench_ref.json

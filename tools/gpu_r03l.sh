#!/bin/bash
# Round 3: the failing 3D drop-in case (2D layers) with a host backtrace.
export TMPDIR=/tmp OMP_NUM_THREADS=1 MKL_NUM_THREADS=1 SUPERLU_MI355X_SEGV_TRACE=1
O=gpurun_out/${1:-r03l}; mkdir -p $O
timeout -k 10 120 /opt/conda/bin/mpiexec -n 4 oracle/_ref/pddrive3d_mi355x -r 1 -c 2 -d 2 -q 2 \
    tests/golden/matrices/g20.rua > $O/run.txt 2>&1; echo rc=$?; grep -v "^\*\*" $O/run.txt | tail -60

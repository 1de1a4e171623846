#!/bin/bash
# The headline matrix through the reference's own EXAMPLE/pddrive.c (MC64,
# MMD_AT_PLUS_A, symbfact, pddistribute, pdgssvx's SOLVE + pdgsrfs), 1 rank:
# (a) our pddistribute + pdgstrf + pdgstrs (libslu_mi355x_solve.so), (b) our
# pdgstrf only (libslu_mi355x.so).  VERDICT r2 #5: DISTRIBUTE < 3 s;
# #7: SOLVE + REFINEMENT < 0.5 s.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${1:-solve100}; mkdir -p $O
( while sleep 45; do date >> $O/tick; done ) & TICK=$!
trap "kill $TICK" EXIT
CONDA=/opt/conda
timeout -k 10 120 python -u tools/write_mtx.py 100 /tmp/lap3d_100.mtx > $O/mtx.log 2>&1 || exit 1
export SUPERLU_MI355X_TIMING=1 SLU_PROFILE_PLAN=1 SLU_AMALG_TIME=1
export MKL_NUM_THREADS=1 MKL_THREADING_LAYER=SEQUENTIAL OMP_NUM_THREADS=1
export LD_LIBRARY_PATH=/usr/lib/x86_64-linux-gnu:/opt/rocm/lib:$CONDA/lib:$LD_LIBRARY_PATH
timeout -k 10 400 $CONDA/bin/mpiexec -n 1 oracle/_ref/pddrive_mi355x_solve -r 1 -c 1 -q 2 /tmp/lap3d_100.mtx > $O/mi355x_solve_1x1.log 2>&1 || { tail -20 $O/mi355x_solve_1x1.log; exit 1; }
grep -E "time|flops|Sol|Steps|digest" $O/mi355x_solve_1x1.log
timeout -k 10 400 $CONDA/bin/mpiexec -n 1 oracle/_ref/pddrive_mi355x -r 1 -c 1 -q 2 /tmp/lap3d_100.mtx > $O/mi355x_1x1.log 2>&1 || { tail -20 $O/mi355x_1x1.log; exit 1; }
grep -E "time|flops|Sol|Steps|digest" $O/mi355x_1x1.log

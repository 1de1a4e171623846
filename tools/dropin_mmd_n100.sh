#!/bin/bash
# The headline matrix through the reference's OWN driver and front-end
# (EXAMPLE/pddrive.c: MC64, MMD_AT_PLUS_A, symbfact, pddistribute, pdgstrs,
# pdgsrfs) with the factorization swapped for libslu_mi355x (1 rank, 1 GPU),
# then the all-reference driver on 2x4 ranks (BASELINE.md's 167.3 s row).
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/mmd100; mkdir -p $O
( while sleep 45; do date >> $O/tick; done ) & TICK=$!
trap "kill $TICK" EXIT
CONDA=/opt/conda
timeout -k 10 120 python -u tools/write_mtx.py 100 /tmp/lap3d_100.mtx > $O/mtx.log 2>&1 || exit 1
export MKL_NUM_THREADS=1 MKL_THREADING_LAYER=SEQUENTIAL OMP_NUM_THREADS=1
export LD_LIBRARY_PATH=/usr/lib/x86_64-linux-gnu:/opt/rocm/lib:$CONDA/lib:$LD_LIBRARY_PATH
timeout -k 10 400 $CONDA/bin/mpiexec -n 1 oracle/_ref/pddrive_mi355x -r 1 -c 1 -q 2 /tmp/lap3d_100.mtx > $O/mi355x_1x1.log 2>&1 || { tail -20 $O/mi355x_1x1.log; exit 1; }
grep -E "time|flops|Sol|Steps" $O/mi355x_1x1.log
timeout -k 10 500 $CONDA/bin/mpiexec -n 8 oracle/_ref/pddrive_ref -r 2 -c 4 -q 2 /tmp/lap3d_100.mtx > $O/ref_2x4.log 2>&1 || { tail -20 $O/ref_2x4.log; exit 1; }
grep -E "time|flops|Sol|Steps" $O/ref_2x4.log

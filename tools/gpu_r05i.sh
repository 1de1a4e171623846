#!/bin/bash
OUT=gpurun_out/${1:-r05i}
rm -rf $OUT; mkdir -p $OUT
export TMPDIR=/tmp
step() { local name=$1 lim=$2; shift 2; echo "== $name"
    timeout -k 10 $lim "$@" > $OUT/$name.out 2> $OUT/$name.err; local rc=$?
    echo "   rc=$rc"; grep -v "^Time to" $OUT/$name.out | tail -${TAILN:-12} | cut -c1-600
    if [ $rc -ge 124 ]; then echo "stopping after rc=$rc"; exit $rc; fi; return 0; }
export OMP_NUM_THREADS=1 MKL_NUM_THREADS=1 MKL_THREADING_LAYER=SEQUENTIAL
M=tests/golden/matrices/big.rua
TAILN=30 step regrid_wrap 200 env REGRID_WRAP=1 /opt/conda/bin/mpiexec -n 4 oracle/_ref/regrid $M 2 2
TAILN=30 step regrid_wrap_noov 200 env REGRID_WRAP=1 SUPERLU_MI355X_OVERLAP=0 SLU_H2D_THREADS=1 /opt/conda/bin/mpiexec -n 4 oracle/_ref/regrid $M 2 2
echo "== done"

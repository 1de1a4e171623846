#!/bin/bash
OUT=gpurun_out/${1:-r05k}
rm -rf $OUT; mkdir -p $OUT
export TMPDIR=/tmp
step() { local name=$1 lim=$2; shift 2; echo "== $name"
    timeout -k 10 $lim "$@" > $OUT/$name.out 2> $OUT/$name.err; local rc=$?
    echo "   rc=$rc"; grep -v "^Time to" $OUT/$name.out | tail -${TAILN:-12} | cut -c1-600; tail -3 $OUT/$name.err | cut -c1-300
    if [ $rc -ge 124 ]; then echo "stopping after rc=$rc"; exit $rc; fi; return 0; }
export OMP_NUM_THREADS=1 MKL_NUM_THREADS=1 MKL_THREADING_LAYER=SEQUENTIAL
M=tests/golden/matrices/big.rua
TAILN=8 step probe 100 env REGRID_REFROUND=-1 REGRID_HIPINIT=4 /opt/conda/bin/mpiexec -n 2 oracle/_ref/regrid_mix $M 1 2
TAILN=5 step regrid_fixed 200 /opt/conda/bin/mpiexec -n 4 oracle/_ref/regrid $M 2 2
TAILN=5 step regrid_fixed_samegrid 200 env REGRID_SAMEGRID=1 /opt/conda/bin/mpiexec -n 4 oracle/_ref/regrid $M 2 2
unset OMP_NUM_THREADS MKL_NUM_THREADS MKL_THREADING_LAYER
TAILN=8 step pytest_regrid 600 python -u -m pytest tests/test_dropin.py -x -v --timeout 300 --timeout-method thread -m gpu -k "evicts or without_plan_cache or regrid"
echo "== done"

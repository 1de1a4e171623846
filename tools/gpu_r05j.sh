#!/bin/bash
OUT=gpurun_out/${1:-r05j}
rm -rf $OUT; mkdir -p $OUT
export TMPDIR=/tmp
step() { local name=$1 lim=$2; shift 2; echo "== $name"
    timeout -k 10 $lim "$@" > $OUT/$name.out 2> $OUT/$name.err; local rc=$?
    echo "   rc=$rc"; grep -v "^Time to" $OUT/$name.out | tail -${TAILN:-12} | cut -c1-600
    if [ $rc -ge 124 ]; then echo "stopping after rc=$rc"; exit $rc; fi; return 0; }
export OMP_NUM_THREADS=1 MKL_NUM_THREADS=1 MKL_THREADING_LAYER=SEQUENTIAL
M=tests/golden/matrices/big.rua
#step regrid_pure 200 /opt/conda/bin/mpiexec -n 4 oracle/_ref/regrid_pure $M 2 2
step mix_ref1 200 env REGRID_REFROUND=1 /opt/conda/bin/mpiexec -n 4 oracle/_ref/regrid_mix $M 2 2
step mix_ref0 200 env REGRID_REFROUND=0 /opt/conda/bin/mpiexec -n 4 oracle/_ref/regrid_mix $M 2 2
step mix_none 200 /opt/conda/bin/mpiexec -n 4 oracle/_ref/regrid_mix $M 2 2
echo "== done"

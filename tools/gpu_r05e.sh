#!/bin/bash
# Round 5 GPU session e: regrid factor sums, watchdog off, lifecycle, devres diagnostic.
OUT=gpurun_out/${1:-r05e}
rm -rf $OUT; mkdir -p $OUT
export TMPDIR=/tmp
step() { local name=$1 lim=$2; shift 2; echo "== $name"
    timeout -k 10 $lim "$@" > $OUT/$name.out 2> $OUT/$name.err; local rc=$?
    echo "   rc=$rc"; grep -v "^Time to" $OUT/$name.out | tail -${TAILN:-12} | cut -c1-600
    if [ $rc -ge 124 ]; then echo "stopping after rc=$rc"; exit $rc; fi; return 0; }
export OMP_NUM_THREADS=1 MKL_NUM_THREADS=1 MKL_THREADING_LAYER=SEQUENTIAL
M=tests/golden/matrices/big.rua
TAILN=20 step regrid_sums 200 env REGRID_SUMS=1 /opt/conda/bin/mpiexec -n 4 oracle/_ref/regrid $M 2 2
step regrid_nowd 200 env SLU_WATCHDOG_S=0 /opt/conda/bin/mpiexec -n 4 oracle/_ref/regrid $M 2 2
step diag_devres 200 python -u tools/diag_devres.py 12
step lifecycle 700 python -u -m pytest tests/test_grid_lifecycle.py -m gpu -v --timeout 400 --timeout-method thread
echo "== done"

#!/bin/bash
# Round 5 GPU session d: the regrid / lifecycle / device-resident issues.
OUT=gpurun_out/${1:-r05d}
rm -rf $OUT; mkdir -p $OUT
export TMPDIR=/tmp
step() { local name=$1 lim=$2; shift 2; echo "== $name"
    timeout -k 10 $lim "$@" > $OUT/$name.out 2> $OUT/$name.err; local rc=$?
    echo "   rc=$rc"; tail -6 $OUT/$name.out | cut -c1-600
    if [ $rc -ge 124 ]; then echo "stopping after rc=$rc"; exit $rc; fi; return 0; }
step diag_devres 200 python -u tools/diag_devres.py 12
step lifecycle 700 python -u -m pytest tests/test_grid_lifecycle.py -m gpu -v --timeout 400 --timeout-method thread
export OMP_NUM_THREADS=1 MKL_NUM_THREADS=1 MKL_THREADING_LAYER=SEQUENTIAL SUPERLU_MI355X_TIMING=1
M=tests/golden/matrices/big.rua
step regrid_amalg0 200 env SLU_AMALG=0 /opt/conda/bin/mpiexec -n 4 oracle/_ref/regrid $M 2 2
step regrid_nocache_1x1 200 env SUPERLU_MI355X_PLAN_CACHE=0 /opt/conda/bin/mpiexec -n 1 oracle/_ref/regrid $M 1 1
step regrid_2x2 200 /opt/conda/bin/mpiexec -n 4 oracle/_ref/regrid $M 2 2
step regrid_1x2 200 /opt/conda/bin/mpiexec -n 2 oracle/_ref/regrid $M 1 2
echo "== done"

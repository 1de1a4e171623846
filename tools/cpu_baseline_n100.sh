#!/bin/bash
# CPU baseline on the actual C3 workload (3D 7-pt Laplacian 100^3), box host cores:
#  (1) reference pdgstrf on the same ND perm_c as the GPU run (oracle/_ref/ref_pdgstrf, 4x4 ranks)
#  (2) the reference's own pddrive, MMD_AT_PLUS_A ordering, 4x4 ranks
# Writes gpurun_out/cpu100/*; a ticker keeps the directory fresh for long silent phases.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/cpu100; mkdir -p $O
( while sleep 45; do date >> $O/tick; done ) & TICK=$!
trap "kill $TICK" EXIT
CONDA=/opt/conda
timeout -k 10 400 python -u -c "
import json, sys; sys.path.insert(0, '.')
import bench
print(json.dumps(bench.cpu_baseline(100, 16, 380)))" > $O/nd.json 2> $O/nd.err || { tail $O/nd.err; exit 1; }
cat $O/nd.json
timeout -k 10 120 python -u tools/write_mtx.py 100 /tmp/lap3d_100.mtx > $O/mtx.log 2>&1 || exit 1
export MKL_NUM_THREADS=1 MKL_THREADING_LAYER=SEQUENTIAL OMP_NUM_THREADS=1
export LD_LIBRARY_PATH=/usr/lib/x86_64-linux-gnu:/opt/rocm/lib:$CONDA/lib:$LD_LIBRARY_PATH
timeout -k 10 700 $CONDA/bin/mpiexec -n 16 oracle/_ref/pddrive_ref -r 4 -c 4 -q 2 /tmp/lap3d_100.mtx > $O/mmd_4x4.log 2>&1 || { tail -20 $O/mmd_4x4.log; exit 1; }
grep -E "time|flops|Mflops|nnz|Sol|error" $O/mmd_4x4.log | head -30

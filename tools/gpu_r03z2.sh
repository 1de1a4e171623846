#!/bin/bash
# Round 3: is the slower plan build after this library's pddistribute the
# malloc state?  The solve library's 100^3 drop-in with glibc's mmap
# threshold pinned high, and with one malloc arena.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${1:-r03z2}; mkdir -p $O
timeout -k 10 120 python -u tools/write_mtx.py 100 /tmp/lap3d_100.mtx > $O/mtx.log 2>&1 || exit 1
export SUPERLU_MI355X_TIMING=1 SLU_PROFILE_PLAN=1 SLU_AMALG_TIME=1 MKL_NUM_THREADS=1 OMP_NUM_THREADS=1
export LD_LIBRARY_PATH=/usr/lib/x86_64-linux-gnu:/opt/rocm/lib:/opt/conda/lib:$LD_LIBRARY_PATH
for v in mmap32M:glibc.malloc.mmap_threshold=33554432 arena1:glibc.malloc.arena_max=1; do
  n=${v%%:*}; t=${v#*:}
  GLIBC_TUNABLES=$t timeout -k 10 400 /opt/conda/bin/mpiexec -n 1 oracle/_ref/pddrive_mi355x_solve -r 1 -c 1 -q 2 /tmp/lap3d_100.mtx \
      > $O/solve_$n.log 2>&1 || exit 1
  echo "== $n"; grep -E "PDGSTRF|slu amalg|slu plan|FACTOR time|DISTRIBUTE time" $O/solve_$n.log
done

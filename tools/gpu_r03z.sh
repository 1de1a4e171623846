#!/bin/bash
# Round 3: the 100^3 drop-in (both libraries) with the timing line that
# reports process CPU time and threads over the plan build, and the solve
# library once more with one plan thread (is the slower build contention?).
set -o pipefail
export TMPDIR=/tmp
T=${1:-r03z}
bash tools/dropin_solve_n100.sh ${T}_solve100 || exit 1
O=gpurun_out/${T}_solve100
export SUPERLU_MI355X_TIMING=1 SLU_PROFILE_PLAN=1 SLU_AMALG_TIME=1 MKL_NUM_THREADS=1 OMP_NUM_THREADS=1
export LD_LIBRARY_PATH=/usr/lib/x86_64-linux-gnu:/opt/rocm/lib:/opt/conda/lib:$LD_LIBRARY_PATH
cat /proc/self/status | grep -E "Cpus_allowed_list|Mems_allowed_list" > $O/cpus.txt
SLU_PLAN_THREADS=1 timeout -k 10 400 /opt/conda/bin/mpiexec -n 1 oracle/_ref/pddrive_mi355x_solve -r 1 -c 1 -q 2 /tmp/lap3d_100.mtx \
    > $O/mi355x_solve_1x1_t1.log 2>&1 || exit 1
grep -E "PDGSTRF|slu amalg|slu plan|FACTOR time" $O/mi355x_solve_1x1_t1.log

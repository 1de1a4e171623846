#!/bin/bash
# which processes of an MPI launch hold GPU device files open
show() { for p in $(pgrep -u $(id -u) -f "$1" 2>/dev/null); do n=$(ls -l /proc/$p/fd 2>/dev/null | grep -cE "kfd|dri"); echo "  pid $p ($(cat /proc/$p/comm)): $n gpu fds"; done; }
/opt/conda/bin/mpiexec -n 2 tools/micro/mpi_sleep 4 &
sleep 2; echo "== mpi_sleep ranks"; show mpi_sleep; wait
echo done

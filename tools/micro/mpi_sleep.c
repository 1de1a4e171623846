/* Diagnostics: MPI_Init, then sleep, so that a script can list which device
 * files an MPI rank holds open (the GPU box's per-GPU process limit). */
#include <mpi.h>
#include <stdlib.h>
#include <unistd.h>
int main(int argc, char **argv) {
    MPI_Init(&argc, &argv);
    sleep(argc > 1 ? atoi(argv[1]) : 4);
    MPI_Finalize();
    return 0;
}

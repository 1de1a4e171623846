/* Test infrastructure (not product code): the ownership contract of this
 * library's p[dsz]distribute (libslu_mi355x_solve.so) against the
 * reference's p[dsz]Destroy_LU (SRC/pdutil.c:485, psutil.c:435,
 * pzutil.c:483), which free the LUstruct's arrays the way the reference's
 * own pddistribute allocated them (the d version its *_dat arrays, the s / z
 * versions every block on its own).
 *
 * The reference's p?gssvx with nrhs = 0 (factorization only) runs its
 * front-end and calls OUR p?distribute, then OUR p?gstrf, which the test
 * hook SUPERLU_MI355X_FACTOR_SKIP=1 returns from at once (no GPU here);
 * with -r the driver calls p?gssvx again with Fact =
 * SamePattern_SameRowPerm (the value refill of the same structure).  Then
 * the reference's p?Destroy_LU / LUstructFree.  Built with
 * -fsanitize=address (oracle/Makefile asan): ASAN's allocator sees every
 * malloc / free of the process, so a block freed that was never malloc'ed
 * on its own, freed twice, or read past its end aborts the run.
 *
 * usage: mpiexec -n P distribute_destroy_asan -t d|s|z -r? -R nprow -C npcol file
 */
#include <stdlib.h>
#include <string.h>

#include "superlu_ddefs.h"
#include "superlu_sdefs.h"
#include "superlu_zdefs.h"

int dcreate_matrix(SuperMatrix *, int, double **, int *, double **, int *, FILE *, gridinfo_t *);
int screate_matrix(SuperMatrix *, int, float **, int *, float **, int *, FILE *, gridinfo_t *);
int zcreate_matrix(SuperMatrix *, int, doublecomplex **, int *, doublecomplex **, int *, FILE *,
                   gridinfo_t *);

#define RUN(P, T, BERR)                                                                           \
    do {                                                                                       \
        SuperMatrix A;                                                                         \
        T *b, *xtrue;                                                                          \
        int ldb, ldx, info = 0;                                                                \
        P##ScalePermstruct_t sp;                                                               \
        P##LUstruct_t lu;                                                                      \
        P##SOLVEstruct_t solve;                                                                \
        SuperLUStat_t stat;                                                                    \
        P##create_matrix(&A, 1, &b, &ldb, &xtrue, &ldx, fp, &grid);                            \
        const int_t m = A.nrow, n = A.ncol;                                                    \
        P##ScalePermstructInit(m, n, &sp);                                                     \
        P##LUstructInit(n, &lu);                                                               \
        PStatInit(&stat);                                                                      \
        p##P##gssvx(&options, &A, &sp, b, ldb, 0, &grid, &lu, &solve, BERR, &stat, &info);     \
        if (info) fprintf(stderr, "p%sgssvx: info %d\n", #P, info);                            \
        if (refill) {                                                                          \
            options.Fact = SamePattern_SameRowPerm;                                            \
            p##P##gssvx(&options, &A, &sp, b, ldb, 0, &grid, &lu, &solve, BERR, &stat, &info); \
            if (info) fprintf(stderr, "p%sgssvx (refill): info %d\n", #P, info);               \
        }                                                                                      \
        P##Destroy_LU(n, &grid, &lu);                                                          \
        P##LUstructFree(&lu);                                                                  \
        P##ScalePermstructFree(&sp);                                                           \
        Destroy_CompRowLoc_Matrix_dist(&A);                                                    \
        SUPERLU_FREE(b);                                                                       \
        SUPERLU_FREE(xtrue);                                                                   \
        PStatFree(&stat);                                                                      \
        ok = info == 0;                                                                        \
    } while (0)

int main(int argc, char **argv) {
    int nprow = 1, npcol = 1, refill = 0, ok = 0;
    char type = 'd';
    const char *file = NULL;
    for (int i = 1; i < argc; ++i) {
        if (!strcmp(argv[i], "-t") && i + 1 < argc) type = argv[++i][0];
        else if (!strcmp(argv[i], "-r")) refill = 1;
        else if (!strcmp(argv[i], "-R") && i + 1 < argc) nprow = atoi(argv[++i]);
        else if (!strcmp(argv[i], "-C") && i + 1 < argc) npcol = atoi(argv[++i]);
        else file = argv[i];
    }
    MPI_Init(&argc, &argv);
    gridinfo_t grid;
    superlu_gridinit(MPI_COMM_WORLD, nprow, npcol, &grid);
    if (grid.iam < nprow * npcol) {
        FILE *fp = fopen(file, "r");
        if (!fp) ABORT("cannot open the matrix file");
        superlu_dist_options_t options;
        set_default_options_dist(&options);
        options.ColPerm = MMD_AT_PLUS_A; /* (METIS is not in this image) */
        options.PrintStat = NO;
        double berr[1];
        float sberr[1];
        if (type == 'd') RUN(d, double, berr);
        else if (type == 's') RUN(s, float, sberr);
        else RUN(z, doublecomplex, berr);
        fclose(fp);
        printf("distribute_destroy %c %dx%d%s: %s\n", type, nprow, npcol, refill ? " refill" : "",
               ok ? "OK" : "FAILED");
    }
    else ok = 1; /* (ranks outside the grid) */
    superlu_gridexit(&grid);
    MPI_Finalize();
    return ok ? 0 : 1;
}

/* Test infrastructure (not product code): the grid life cycle twice in one
 * process, through libslu_mi355x.so.  Each round: superlu_gridinit on a
 * Pr x Pc grid, pdgssvx (DOFACT), then a second pdgssvx with Fact =
 * SamePattern_SameRowPerm on the same LUstruct (a plan-cache hit), then
 * dDestroy_LU and superlu_gridexit.  superlu_gridexit frees grid->comm,
 * which destroys the engine communicators cached on it: the cached plan built
 * on them must go with them, so the next round's first
 * call builds a new plan on the new grid's transport even if MPI reuses the
 * communicator handle and malloc the LUstruct addresses.
 *
 * usage: mpiexec -n Pr*Pc regrid file Pr Pc   (prints "round r call c: err e")
 */
#include <stdlib.h>
#include <string.h>

#include "superlu_ddefs.h"

int dcreate_matrix(SuperMatrix *, int, double **, int *, double **, int *, FILE *, gridinfo_t *);

int main(int argc, char **argv) {
    if (argc < 4) return 2;
    MPI_Init(&argc, &argv);
    const int pr = atoi(argv[2]), pc = atoi(argv[3]);
    for (int round = 0; round < 2; ++round) {
        gridinfo_t grid;
        superlu_gridinit(MPI_COMM_WORLD, pr, pc, &grid);
        SuperMatrix A;
        double *b, *xtrue;
        int ldb, ldx;
        FILE *fp = fopen(argv[1], "r");
        if (!fp) ABORT("cannot open the matrix file");
        dcreate_matrix(&A, 1, &b, &ldb, &xtrue, &ldx, fp, &grid);
        fclose(fp);
        /* pdgssvx scales and permutes A in place: keep its arrays for the
         * second call, which rebuilds A from them (EXAMPLE/pddrive3.c) */
        NRformat_loc *As = (NRformat_loc *)A.Store;
        const int m = A.nrow, n = A.ncol, m_loc = As->m_loc, fst_row = As->fst_row;
        const int_t nnz_loc = As->nnz_loc;
        double *nzval1 = doubleMalloc_dist(nnz_loc);
        int_t *colind1 = intMalloc_dist(nnz_loc), *rowptr1 = intMalloc_dist(m_loc + 1);
        memcpy(nzval1, As->nzval, sizeof(double) * nnz_loc);
        memcpy(colind1, As->colind, sizeof(int_t) * nnz_loc);
        memcpy(rowptr1, As->rowptr, sizeof(int_t) * (m_loc + 1));
        double *b0 = doubleMalloc_dist(ldb);
        memcpy(b0, b, sizeof(double) * ldb);
        superlu_dist_options_t opt;
        set_default_options_dist(&opt);
        opt.ColPerm = MMD_AT_PLUS_A; /* (METIS is not in this image) */
        opt.PrintStat = NO;
        dScalePermstruct_t sp;
        dLUstruct_t lu;
        dSOLVEstruct_t solve;
        dScalePermstructInit(A.nrow, A.ncol, &sp);
        dLUstructInit(A.ncol, &lu);
        for (int call = 0; call < 2; ++call) {
            SuperLUStat_t stat;
            double berr[1];
            int info = 0;
            memcpy(b, b0, sizeof(double) * ldb);
            PStatInit(&stat);
            pdgssvx(&opt, &A, &sp, b, ldb, 1, &grid, &lu, &solve, berr, &stat, &info);
            PStatFree(&stat);
            double dmax = 0, xmax = 0, g[2];
            for (int i = 0; i < m_loc; ++i) {
                const double d = fabs(b[i] - xtrue[i]);
                if (d > dmax) dmax = d;
                if (fabs(b[i]) > xmax) xmax = fabs(b[i]);
            }
            double l[2] = {dmax, xmax};
            MPI_Allreduce(l, g, 2, MPI_DOUBLE, MPI_MAX, grid.comm);
            if (grid.iam == 0) {
                printf("round %d call %d: info %d err %.3e\n", round, call, info, g[0] / g[1]);
                fflush(stdout);
            }
            if (call == 0) { /* the same pattern and values, from the saved arrays */
                opt.Fact = SamePattern_SameRowPerm;
                Destroy_CompRowLoc_Matrix_dist(&A);
                dZeroLblocks(grid.iam, n, &grid, &lu);
                dZeroUblocks(grid.iam, n, &grid, &lu);
                dCreate_CompRowLoc_Matrix_dist(&A, m, n, nnz_loc, m_loc, fst_row, nzval1, colind1,
                                               rowptr1, SLU_NR_loc, SLU_D, SLU_GE);
            }
        }
        dSolveFinalize(&opt, &solve);
        dDestroy_LU(A.ncol, &grid, &lu);
        dLUstructFree(&lu);
        dScalePermstructFree(&sp);
        Destroy_CompRowLoc_Matrix_dist(&A); /* (frees nzval1 / colind1 / rowptr1) */
        SUPERLU_FREE(b);
        SUPERLU_FREE(b0);
        SUPERLU_FREE(xtrue);
        superlu_gridexit(&grid);
    }
    MPI_Finalize();
    return 0;
}

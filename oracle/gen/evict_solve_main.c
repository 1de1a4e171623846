/* Test infrastructure (not product code): one process holding two
 * factorizations, through libslu_mi355x_solve.so (our p?distribute keeps A
 * for a device-side fill, our pdgstrf keeps 1x1 factors in HBM only, our
 * pdgstrs solves on them).  System 1 is factored and solved, then system 2
 * (another structure) is factored, which evicts system 1's cached plan and
 * with it the only copy of system 1's factors; then pdgssvx with Fact =
 * FACTORED solves system 1 again (the EXAMPLE/pddrive1.c re-entry).  The
 * library must refuse that solve loudly (its host L/U arrays hold A, not the
 * factors) unless SUPERLU_MI355X_HOST_FACTORS=1 wrote the factors back, in
 * which case the solve must be accurate.
 *
 * usage: evict_solve fileA fileB   (one MPI rank, 1x1 grid; prints one
 * "system k: err" line per completed solve)
 */
#include <stdlib.h>
#include <string.h>

#include "superlu_ddefs.h"

int dcreate_matrix(SuperMatrix *, int, double **, int *, double **, int *, FILE *, gridinfo_t *);

typedef struct {
    SuperMatrix A;
    double *b, *b0, *xtrue;
    int ldb, ldx;
    dScalePermstruct_t sp;
    dLUstruct_t lu;
    dSOLVEstruct_t solve;
    superlu_dist_options_t opt;
} System;

static int load(System *s, const char *file, gridinfo_t *grid) {
    FILE *fp = fopen(file, "r");
    if (!fp) return 0;
    dcreate_matrix(&s->A, 1, &s->b, &s->ldb, &s->xtrue, &s->ldx, fp, grid);
    fclose(fp);
    s->b0 = doubleMalloc_dist(s->ldb);
    memcpy(s->b0, s->b, sizeof(double) * s->ldb);
    set_default_options_dist(&s->opt);
    s->opt.ColPerm = MMD_AT_PLUS_A; /* (METIS is not in this image) */
    s->opt.PrintStat = NO;
    dScalePermstructInit(s->A.nrow, s->A.ncol, &s->sp);
    dLUstructInit(s->A.ncol, &s->lu);
    return 1;
}

static double solve(System *s, int k, gridinfo_t *grid) {
    SuperLUStat_t stat;
    double berr[1];
    int info = 0;
    memcpy(s->b, s->b0, sizeof(double) * s->ldb);
    PStatInit(&stat);
    pdgssvx(&s->opt, &s->A, &s->sp, s->b, s->ldb, 1, grid, &s->lu, &s->solve, berr, &stat, &info);
    PStatFree(&stat);
    if (info) {
        printf("system %d: info %d\n", k, info);
        return -1;
    }
    /* ||x - xtrue|| / ||x|| on the one rank */
    double dmax = 0, xmax = 0;
    for (int i = 0; i < ((NRformat_loc *)s->A.Store)->m_loc; ++i) {
        const double d = fabs(s->b[i] - s->xtrue[i]);
        if (d > dmax) dmax = d;
        if (fabs(s->b[i]) > xmax) xmax = fabs(s->b[i]);
    }
    printf("system %d: err %.3e\n", k, dmax / xmax);
    fflush(stdout);
    return dmax / xmax;
}

int main(int argc, char **argv) {
    if (argc < 3) return 2;
    MPI_Init(&argc, &argv);
    gridinfo_t grid;
    superlu_gridinit(MPI_COMM_WORLD, 1, 1, &grid);
    System s1, s2;
    if (!load(&s1, argv[1], &grid) || !load(&s2, argv[2], &grid)) ABORT("cannot open a matrix file");
    solve(&s1, 1, &grid);      /* DOFACT: factors of system 1 (HBM only) */
    solve(&s2, 2, &grid);      /* DOFACT: another structure, evicts system 1's plan */
    s1.opt.Fact = FACTORED;    /* the factored form of system 1 is supplied */
    solve(&s1, 3, &grid);
    dDestroy_LU(s1.A.ncol, &grid, &s1.lu);
    dDestroy_LU(s2.A.ncol, &grid, &s2.lu);
    superlu_gridexit(&grid);
    MPI_Finalize();
    return 0;
}

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
#define _GNU_SOURCE
#include <stdlib.h>
#include <string.h>

#include "superlu_ddefs.h"

int dcreate_matrix(SuperMatrix *, int, double **, int *, double **, int *, FILE *, gridinfo_t *);

#include <dlfcn.h>
#include <execinfo.h>
#include <signal.h>
#include <unistd.h>
static void segv_bt(int sig) {
    void *f[64];
    const int k = backtrace(f, 64);
    backtrace_symbols_fd(f, k, 2);
    signal(sig, SIG_DFL);
    raise(sig);
}
/* the factors' position-weighted sums of this rank (diagnostics) */
static void factor_sums(dLUstruct_t *lu, gridinfo_t *grid, int n, double *ls, double *us) {
    dLocalLU_t *Llu = lu->Llu;
    const int nsup = lu->Glu_persist->supno[n - 1] + 1;
    *ls = *us = 0;
    for (int lb = 0; lb < CEILING(nsup, grid->npcol); ++lb) {
        const int_t *ix = Llu->Lrowind_bc_ptr[lb];
        if (!ix) continue;
        const int jb = lb * grid->npcol + grid->iam % grid->npcol;
        const int_t cnt = ix[1] * (lu->Glu_persist->xsup[jb + 1] - lu->Glu_persist->xsup[jb]);
        for (int_t i = 0; i < cnt; ++i) *ls += Llu->Lnzval_bc_ptr[lb][i] * (double)(i % 97 + 1);
    }
    for (int lb = 0; lb < CEILING(nsup, grid->nprow); ++lb) {
        const int_t *ix = Llu->Ufstnz_br_ptr[lb];
        if (!ix) continue;
        for (int_t i = 0; i < ix[1]; ++i) *us += Llu->Unzval_br_ptr[lb][i] * (double)(i % 97 + 1);
    }
}

static int g_round;
#ifdef REGRID_MIX
int_t ref_pdgstrf(superlu_dist_options_t *, int, int, double, dLUstruct_t *, gridinfo_t *, SuperLUStat_t *, int *);
#endif
#ifdef REGRID_MIX
/* (regrid_mix only) REGRID_WRAP: this executable's pdgstrf interposes the library's (the
 * reference's pdgssvx binds it first) and checks that the factors do not
 * change after the call returned (no write still in flight) */
int_t pdgstrf(superlu_dist_options_t *options, int m, int n, double anorm, dLUstruct_t *LUstruct,
              gridinfo_t *grid, SuperLUStat_t *stat, int *info) {
    typedef int_t (*fn_t)(superlu_dist_options_t *, int, int, double, dLUstruct_t *, gridinfo_t *,
                          SuperLUStat_t *, int *);
    static fn_t next = NULL;
    if (!next) next = (fn_t)dlsym(RTLD_NEXT, "pdgstrf");
    fn_t f = next;
#ifdef REGRID_MIX
    /* REGRID_REFROUND=r: round r factors with the reference's own pdgstrf
     * (linked in renamed), the other round with the library's */
    const char *rr = getenv("REGRID_REFROUND");
    if (rr && (atoi(rr) == g_round || atoi(rr) < 0)) f = ref_pdgstrf; /* (-1: both rounds) */
#endif
    const int_t rv = f(options, m, n, anorm, LUstruct, grid, stat, info);
    if (getenv("REGRID_WRAP")) {
        double l0, u0, l1, u1;
        factor_sums(LUstruct, grid, n, &l0, &u0);
        usleep(500000);
        factor_sums(LUstruct, grid, n, &l1, &u1);
        printf("pdgstrf returned, rank %d: wsum L %.17g U %.17g, 0.5 s later L %.17g U %.17g%s\n", grid->iam,
               l0, u0, l1, u1, (l0 != l1 || u0 != u1) ? "  CHANGED" : "");
        fflush(stdout);
    }
    return rv;
}
#endif

int main(int argc, char **argv) {
    if (argc < 4) return 2;
    if (getenv("REGRID_BT")) signal(SIGSEGV, segv_bt);
    MPI_Init(&argc, &argv);
#ifdef REGRID_MIX
    /* REGRID_HIPINIT=1: the HIP runtime initialised (one device allocation)
     * before anything else, whatever factors */
    if (getenv("REGRID_HIPINIT")) {
        void *h = dlopen("libamdhip64.so", RTLD_NOW | RTLD_GLOBAL);
        int (*hmalloc)(void **, size_t) = h ? (int (*)(void **, size_t))dlsym(h, "hipMalloc") : NULL;
        void *d = NULL;
        printf("hipMalloc: %d\n", hmalloc ? hmalloc(&d, 1 << 20) : -1);
        /* REGRID_HIPINIT=2: and two streams (priority, non-blocking) created
         * and destroyed; 3: one plain stream */
        const int mode = atoi(getenv("REGRID_HIPINIT"));
        int (*prange)(int *, int *) = (int (*)(int *, int *))dlsym(h, "hipDeviceGetStreamPriorityRange");
        int (*screate)(void **, unsigned, int) = (int (*)(void **, unsigned, int))dlsym(h, "hipStreamCreateWithPriority");
        int (*splain)(void **) = (int (*)(void **))dlsym(h, "hipStreamCreate");
        int (*sdestroy)(void *) = (int (*)(void *))dlsym(h, "hipStreamDestroy");
        void *s1 = NULL, *s2 = NULL;
        int lo = 0, hi = 0;
        if (mode == 2) {
            prange(&lo, &hi);
            printf("streams: %d %d\n", screate(&s1, 1, lo), screate(&s2, 1, hi));
            sdestroy(s1);
            sdestroy(s2);
        } else if (mode == 3) {
            printf("stream: %d\n", splain(&s1));
            sdestroy(s1);
        } else if (mode == 4) { /* which calls move libc rand()'s sequence */
            srand(7);
            const int r0 = rand();
            srand(7);
            splain(&s1);
            const int r1 = rand();
            srand(7);
            sdestroy(s1);
            const int r2 = rand();
            srand(7);
            void *d2 = NULL;
            hmalloc(&d2, 1 << 26);
            const int r3 = rand();
            printf("rand after srand(7): %d; after stream create %d, destroy %d, hipMalloc %d\n", r0, r1, r2, r3);
        }
    }
    /* REGRID_MPITEST=1: broadcasts and all-to-alls of patterned buffers,
     * checked on every rank (after REGRID_HIPINIT's streams, if any) */
    if (getenv("REGRID_MPITEST")) {
        int me, np;
        MPI_Comm_rank(MPI_COMM_WORLD, &me);
        MPI_Comm_size(MPI_COMM_WORLD, &np);
        for (long sz = 8; sz <= (8L << 20); sz *= 8) {
            long bad = 0;
            for (int rep = 0; rep < 3; ++rep) {
                double *buf = (double *)malloc(sz * sizeof(double));
                for (long i = 0; i < sz; ++i) buf[i] = me == 0 ? (double)(i * 7 + rep) : -1.0;
                MPI_Bcast(buf, (int)sz, MPI_DOUBLE, 0, MPI_COMM_WORLD);
                for (long i = 0; i < sz; ++i) bad += buf[i] != (double)(i * 7 + rep);
                free(buf);
                /* all-to-all-v: rank p sends rank q a block of sz/np values p*1e9+q*1e6+i */
                const long blk = sz / np > 0 ? sz / np : 1;
                double *sb = (double *)malloc(blk * np * sizeof(double)), *rb = (double *)malloc(blk * np * sizeof(double));
                int *cnt = (int *)malloc(np * sizeof(int)), *dsp = (int *)malloc(np * sizeof(int));
                for (int q = 0; q < np; ++q) {
                    cnt[q] = (int)blk;
                    dsp[q] = (int)(q * blk);
                    for (long i = 0; i < blk; ++i) sb[q * blk + i] = me * 1e9 + q * 1e6 + i + rep;
                }
                MPI_Alltoallv(sb, cnt, dsp, MPI_DOUBLE, rb, cnt, dsp, MPI_DOUBLE, MPI_COMM_WORLD);
                for (int p = 0; p < np; ++p)
                    for (long i = 0; i < blk; ++i) bad += rb[p * blk + i] != p * 1e9 + me * 1e6 + i + rep;
                free(sb); free(rb); free(cnt); free(dsp);
            }
            long tot = 0;
            MPI_Allreduce(&bad, &tot, 1, MPI_LONG, MPI_SUM, MPI_COMM_WORLD);
            if (me == 0) printf("mpitest %ld doubles: %ld wrong\n", sz, tot);
        }
        fflush(stdout);
    }
#endif
    const int pr = atoi(argv[2]), pc = atoi(argv[3]);
    gridinfo_t keep; /* REGRID_KEEP: round 0's grid stays alive through round 1 */
    for (int round = 0; round < 2; ++round) {
        g_round = round;
        /* REGRID_SKIP0: round 0 runs with this library's factorization skipped
         * (SUPERLU_MI355X_FACTOR_SKIP), round 1 is the first real one */
        if (getenv("REGRID_SKIP0")) {
            if (round == 0) setenv("SUPERLU_MI355X_FACTOR_SKIP", "1", 1);
            else unsetenv("SUPERLU_MI355X_FACTOR_SKIP");
        }
        gridinfo_t grid;
        /* REGRID_SAMEGRID: both rounds on one grid (a second system, new
         * LUstruct and SOLVEstruct, on the same communicators) */
        if (getenv("REGRID_SAMEGRID") && round == 1) grid = keep;
        else superlu_gridinit(MPI_COMM_WORLD, pr, pc, &grid);
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
        if (getenv("REGRID_NOREFINE")) opt.IterRefine = NOREFINE;
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
            if (getenv("REGRID_SUMS")) { /* the factors' sums, per rank (diagnostics) */
                dLocalLU_t *Llu = lu.Llu;
                const int nsup = lu.Glu_persist->supno[n - 1] + 1;
                double ls = 0, us = 0;
                for (int lb = 0; lb < CEILING(nsup, grid.npcol); ++lb) {
                    const int_t *ix = Llu->Lrowind_bc_ptr[lb];
                    if (!ix) continue;
                    const int jb = lb * grid.npcol + grid.iam % grid.npcol;
                    const int_t cnt = ix[1] * (lu.Glu_persist->xsup[jb + 1] - lu.Glu_persist->xsup[jb]);
                    for (int_t i = 0; i < cnt; ++i) ls += Llu->Lnzval_bc_ptr[lb][i] * (double)(i % 97 + 1);
                }
                for (int lb = 0; lb < CEILING(nsup, grid.nprow); ++lb) {
                    const int_t *ix = Llu->Ufstnz_br_ptr[lb];
                    if (!ix) continue;
                    for (int_t i = 0; i < ix[1]; ++i) us += Llu->Unzval_br_ptr[lb][i] * (double)(i % 97 + 1);
                }
                /* and the index arrays (an in-place change would show here) */
                long long li = 0, ui = 0, lv = 0;
                for (int lb = 0; lb < CEILING(nsup, grid.npcol); ++lb) {
                    const int_t *ix = Llu->Lrowind_bc_ptr[lb];
                    if (!ix) continue;
                    int_t p = BC_HEADER;
                    for (int_t b = 0; b < ix[0]; ++b) p += LB_DESCRIPTOR + ix[p + 1];
                    for (int_t i = 0; i < p; ++i) li += (long long)ix[i] * (i + 1);
                    if (Llu->Lindval_loc_bc_ptr && Llu->Lindval_loc_bc_ptr[lb])
                        for (int_t i = 0; i < 3 * ix[0]; ++i) lv += (long long)Llu->Lindval_loc_bc_ptr[lb][i] * (i + 1);
                }
                for (int lb = 0; lb < CEILING(nsup, grid.nprow); ++lb) {
                    const int_t *ix = Llu->Ufstnz_br_ptr[lb];
                    if (!ix) continue;
                    for (int_t i = 0; i < ix[2]; ++i) ui += (long long)ix[i] * (i + 1);
                }
                printf("round %d call %d rank %d: wsum L %.17g wsum U %.17g idx %lld %lld %lld\n", round, call,
                       grid.iam, ls, us, li, ui, lv);
                fflush(stdout);
            }
            /* the reference draws its solve trees' seeds from rand() on every
             * rank (SRC/pddistribute.c:1557): the sequence must not have moved
             * differently on any rank */
            const int rnd = rand();
            int rmin, rmax;
            MPI_Allreduce(&rnd, &rmin, 1, MPI_INT, MPI_MIN, grid.comm);
            MPI_Allreduce(&rnd, &rmax, 1, MPI_INT, MPI_MAX, grid.comm);
            if (grid.iam == 0) {
                printf("round %d call %d: info %d err %.3e rand %s\n", round, call, info, g[0] / g[1],
                       rmin == rmax ? "same" : "DIFFERS");
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
        if (getenv("REGRID_PROBE")) { /* messages nobody received (diagnostics) */
            MPI_Comm cs[4] = {grid.comm, grid.rscp.comm, grid.cscp.comm, MPI_COMM_WORLD};
            const char *nm[4] = {"grid", "row", "column", "world"};
            MPI_Barrier(grid.comm);
            for (int k = 0; k < 4; ++k) {
                int flag = 0;
                MPI_Status st;
                MPI_Iprobe(MPI_ANY_SOURCE, MPI_ANY_TAG, cs[k], &flag, &st);
                if (flag) {
                    int cnt = 0;
                    MPI_Get_count(&st, MPI_BYTE, &cnt);
                    printf("round %d rank %d: pending message on the %s communicator from %d tag %d (%d bytes)\n",
                           round, grid.iam, nm[k], st.MPI_SOURCE, st.MPI_TAG, cnt);
                    fflush(stdout);
                }
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
        if ((getenv("REGRID_KEEP") || getenv("REGRID_SAMEGRID")) && round == 0) keep = grid;
        else if (getenv("REGRID_SAMEGRID")) { /* (freed below) */ }
        else superlu_gridexit(&grid);
    }
    if (getenv("REGRID_KEEP") || getenv("REGRID_SAMEGRID")) superlu_gridexit(&keep);
    MPI_Finalize();
    return 0;
}

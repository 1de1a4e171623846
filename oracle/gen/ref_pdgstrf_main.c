/*
 * ref_pdgstrf_main.c -- MPI harness around the REFERENCE pdgstrf / psgstrf /
 * pzgstrf (compiled from /root/reference/SRC by oracle/Makefile).
 *
 * TEST INFRASTRUCTURE.  Each rank builds its LUstruct with the front-end of
 * libslu_mi355x.so (dlopen'ed RTLD_LOCAL so its own pdgstrf cannot interpose),
 * calls the reference factorization exactly as pdgssvx does
 * (SRC/pdgssvx.c:1174-1180), and writes its factor arrays and statistics.
 *
 * usage: mpiexec -n P ref_pdgstrf -lib LIB -f MATRIX.bin -r PR -c PC
 *          [-x relax] [-m maxsup] [-l lookaheads] [-t replace_tiny]
 *          [-n reps] [-o outprefix] [-s symbolic_flags] [-k blocksums_prefix]
 * -s: slu_symbolic flags (2 = SLU_SYMB_REFERENCE: pdgssvx's own sp_colorder +
 *     symbfact + pddistribute, restated bit-exact in the library).
 * -k: per-block checksums of the factors (oracle/blocksum.h) per rank.
 * MATRIX.bin: int64 {n, nnz, dtype, has_perm}, colptr[n+1], rowind[nnz],
 *             values[nnz] (dtype 0=d,1=s,2=z), perm_c[n] if has_perm.
 */
#include <dlfcn.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "superlu_ddefs.h"
#include "superlu_sdefs.h"
#include "superlu_zdefs.h"

/* the library's flat LUstruct view (include/slu_mi355x.h) */
typedef struct {
    int64_t nsupers;
    int_t *xsup, *supno;
    int_t *Lidx; int64_t Lidx_cnt; long *Lidx_off;
    void *Lval; int64_t Lval_cnt; long *Lval_off;
    int_t *Uidx; int64_t Uidx_cnt; long *Uidx_off;
    void *Uval; int64_t Uval_cnt; long *Uval_off;
    int *ToRecv, *ToSendD, **ToSendR;
    int_t bufmax[5];
} slu_lu_view;
#define SLU_ORACLE_BLOCKSUM_WRITE
#include "../blocksum.h"

typedef struct {
    int64_t n, nnz;
    int64_t *colptr, *rowind;
    void *val;
    int dtype;
} fe_csc;

typedef fe_csc *(*csc_create_t)(int64_t, int64_t, const int64_t *, const int64_t *, const void *, int);
typedef void *(*symbolic_t)(const fe_csc *, const int64_t *, int, int, int);
typedef void *(*distribute_t)(const void *, const fe_csc *, int, int, int, int);
typedef void (*lufree_t)(void *, int);
typedef int (*view_t)(void *, int, slu_lu_view *);

static size_t vsz(int dt) { return dt == 1 ? 4 : dt == 2 ? 16 : 8; }

int main(int argc, char **argv) {
    int prov;
    MPI_Init_thread(&argc, &argv, MPI_THREAD_MULTIPLE, &prov);
    const char *libpath = NULL, *mfile = NULL, *outp = NULL, *sums = NULL;
    int nprow = 1, npcol = 1, relax = 60, maxsup = 256, look = 10, tiny = 0, reps = 1, sflags = 0;
    for (int i = 1; i < argc - 1; ++i) {
        if (!strcmp(argv[i], "-lib")) libpath = argv[++i];
        else if (!strcmp(argv[i], "-f")) mfile = argv[++i];
        else if (!strcmp(argv[i], "-o")) outp = argv[++i];
        else if (!strcmp(argv[i], "-r")) nprow = atoi(argv[++i]);
        else if (!strcmp(argv[i], "-c")) npcol = atoi(argv[++i]);
        else if (!strcmp(argv[i], "-x")) relax = atoi(argv[++i]);
        else if (!strcmp(argv[i], "-m")) maxsup = atoi(argv[++i]);
        else if (!strcmp(argv[i], "-l")) look = atoi(argv[++i]);
        else if (!strcmp(argv[i], "-t")) tiny = atoi(argv[++i]);
        else if (!strcmp(argv[i], "-n")) reps = atoi(argv[++i]);
        else if (!strcmp(argv[i], "-s")) sflags = atoi(argv[++i]);
        else if (!strcmp(argv[i], "-k")) sums = argv[++i];
    }
    void *h = dlopen(libpath, RTLD_NOW | RTLD_LOCAL);
    if (!h) { fprintf(stderr, "dlopen %s: %s\n", libpath, dlerror()); MPI_Abort(MPI_COMM_WORLD, 1); }
    csc_create_t csc_create = (csc_create_t)dlsym(h, "slu_csc_create");
    symbolic_t symbolic = (symbolic_t)dlsym(h, "slu_symbolic");
    distribute_t distribute = (distribute_t)dlsym(h, "slu_distribute");
    lufree_t lufree = (lufree_t)dlsym(h, "slu_lustruct_free");
    view_t get_view = (view_t)dlsym(h, "slu_lu_get_view");

    FILE *fp = fopen(mfile, "rb");
    if (!fp) { fprintf(stderr, "cannot open %s\n", mfile); MPI_Abort(MPI_COMM_WORLD, 1); }
    int64_t hdr[4];
    if (fread(hdr, 8, 4, fp) != 4) MPI_Abort(MPI_COMM_WORLD, 1);
    int64_t n = hdr[0], nnz = hdr[1];
    int dtype = (int)hdr[2];
    int64_t *colptr = malloc((n + 1) * 8), *rowind = malloc(nnz * 8), *perm = NULL;
    void *val = malloc(nnz * vsz(dtype));
    size_t rd = fread(colptr, 8, n + 1, fp);
    rd += fread(rowind, 8, nnz, fp);
    rd += fread(val, vsz(dtype), nnz, fp);
    if (hdr[3]) { perm = malloc(n * 8); rd += fread(perm, 8, n, fp); }
    fclose(fp);
    (void)rd;

    /* anorm = ||A||_1 (pdlangs("1"), SRC/pdgssvx.c:950) */
    double anorm = 0.0;
    for (int64_t j = 0; j < n; ++j) {
        double s = 0.0;
        for (int64_t p = colptr[j]; p < colptr[j + 1]; ++p) {
            if (dtype == 0) s += fabs(((double *)val)[p]);
            else if (dtype == 1) s += fabsf(((float *)val)[p]);
            else s += hypot(((double *)val)[2 * p], ((double *)val)[2 * p + 1]);
        }
        if (s > anorm) anorm = s;
    }

    gridinfo_t grid;
    superlu_gridinit(MPI_COMM_WORLD, nprow, npcol, &grid);
    int iam = grid.iam, myrow = iam / npcol, mycol = iam % npcol;
    fe_csc *A = csc_create(n, nnz, colptr, rowind, val, dtype);
    void *symb = symbolic(A, perm, relax, maxsup, sflags);

    double tbest = 1e30, tsum = 0;
    int info = 0, tinyp = 0;
    double ops = 0;
    for (int rep = 0; rep < reps; ++rep) {
        void *LU = distribute(symb, A, nprow, npcol, myrow, mycol);
        superlu_dist_options_t options;
        set_default_options_dist(&options);
        options.num_lookaheads = look;
        options.ReplaceTinyPivot = tiny ? YES : NO;
        options.superlu_maxsup = maxsup;
        options.superlu_relax = relax;
        SuperLUStat_t stat;
        PStatInit(&stat);
        MPI_Barrier(MPI_COMM_WORLD);
        double t0 = MPI_Wtime();
        if (dtype == 0)
            pdgstrf(&options, (int)n, (int)n, anorm, (dLUstruct_t *)LU, &grid, &stat, &info);
        else if (dtype == 1)
            psgstrf(&options, (int)n, (int)n, (float)anorm, (sLUstruct_t *)LU, &grid, &stat, &info);
        else
            pzgstrf(&options, (int)n, (int)n, anorm, (zLUstruct_t *)LU, &grid, &stat, &info);
        double t = MPI_Wtime() - t0, tmax;
        MPI_Allreduce(&t, &tmax, 1, MPI_DOUBLE, MPI_MAX, MPI_COMM_WORLD);
        if (tmax < tbest) tbest = tmax;
        tsum += tmax;
        double myops = stat.ops[FACT];
        MPI_Allreduce(&myops, &ops, 1, MPI_DOUBLE, MPI_SUM, MPI_COMM_WORLD);
        MPI_Allreduce(&stat.TinyPivots, &tinyp, 1, MPI_INT, MPI_SUM, MPI_COMM_WORLD);
        if (rep == reps - 1 && outp) {
            char fn[1024];
            /* flat factor arrays of this rank (library layout keeps *_dat contiguous) */
            long lcnt, ucnt;
            void *ld, *ud;
            if (dtype == 0) {
                dLocalLU_t *L = ((dLUstruct_t *)LU)->Llu;
                ld = L->Lnzval_bc_dat; lcnt = L->Lnzval_bc_cnt; ud = L->Unzval_br_dat; ucnt = L->Unzval_br_cnt;
            } else if (dtype == 1) {
                sLocalLU_t *L = ((sLUstruct_t *)LU)->Llu;
                ld = L->Lnzval_bc_dat; lcnt = L->Lnzval_bc_cnt; ud = L->Unzval_br_dat; ucnt = L->Unzval_br_cnt;
            } else {
                zLocalLU_t *L = ((zLUstruct_t *)LU)->Llu;
                ld = L->Lnzval_bc_dat; lcnt = L->Lnzval_bc_cnt; ud = L->Unzval_br_dat; ucnt = L->Unzval_br_cnt;
            }
            snprintf(fn, sizeof fn, "%s.rank%d.L.bin", outp, iam);
            fp = fopen(fn, "wb"); fwrite(ld, vsz(dtype), lcnt, fp); fclose(fp);
            snprintf(fn, sizeof fn, "%s.rank%d.U.bin", outp, iam);
            fp = fopen(fn, "wb"); fwrite(ud, vsz(dtype), ucnt, fp); fclose(fp);
        }
        if (rep == reps - 1 && sums) {
            slu_lu_view v;
            get_view(LU, dtype, &v);
            v.nsupers = n > 0 ? v.supno[n - 1] + 1 : 0;
            char fn[1024];
            snprintf(fn, sizeof fn, "%s.rank%d.bin", sums, iam);
            if (blocksum_write(fn, dtype, &v, nprow, npcol, myrow, mycol)) {
                fprintf(stderr, "cannot write %s\n", fn);
                MPI_Abort(MPI_COMM_WORLD, 1);
            }
        }
        PStatFree(&stat);
        lufree(LU, dtype);
    }
    if (iam == 0) {
        int nth = 1;
#ifdef _OPENMP
        nth = omp_get_max_threads();
#endif
        printf("{\"time_best\": %.6f, \"time_mean\": %.6f, \"ops\": %.6e, \"info\": %d, "
               "\"tiny\": %d, \"nprocs\": %d, \"omp_threads\": %d, \"anorm\": %.17g}\n",
               tbest, tsum / reps, ops, info, tinyp, nprow * npcol, nth, anorm);
        fflush(stdout);
    }
    superlu_gridexit(&grid);
    MPI_Finalize();
    return 0;
}

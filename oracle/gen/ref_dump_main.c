/*
 * ref_dump_main.c -- runs the REFERENCE p[dsz]gssvx end to end (compiled from
 * /root/reference/SRC by oracle/Makefile) and dumps what crosses the pdgstrf
 * boundary, for the golden fixtures tests/golden/refdump_*.npz.
 *
 * TEST INFRASTRUCTURE.  The whole front-end is the reference's own: matrix
 * read + xtrue/b (EXAMPLE/[dsz]create_matrix.c), equilibration, MC64 row
 * permutation, MMD/COLAMD column ordering (or MY_PERMC from a file),
 * symbfact and pddistribute (SRC/pdgssvx.c:718-1146).  This file defines
 * pdgstrf / psgstrf / pzgstrf; the reference factorization itself is linked
 * under the name slu_refimpl_p?gstrf (the same source compiled with -D).
 * The interposer writes each rank's LUstruct before the factorization, calls
 * the reference, and writes the factored values, info, TinyPivots and
 * ops[FACT].  After pdgssvx returns (solve + refinement, SRC/pdgssvx.c:1427-
 * 1548) the harness writes x, berr and RefineSteps, then solves once more
 * with Fact = FACTORED and IterRefine = NOREFINE for the unrefined x.
 *
 * usage: mpiexec -n P ref_dump -t d|s|z -o OUTDIR [-r PR] [-c PC] [-x relax]
 *          [-m maxsup] [-p rowperm] [-q colperm] [-e equil] [-y replace_tiny]
 *          [-l lookaheads] [-i iterrefine] [-s nrhs] [-P permc.bin] MATRIX
 * OUTDIR receives r<rank>_<name>.npy per rank and meta_<rank>.json.
 */
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "superlu_ddefs.h"
#include "superlu_sdefs.h"
#include "superlu_zdefs.h"

int_t slu_refimpl_pdgstrf(superlu_dist_options_t *, int, int, double, dLUstruct_t *, gridinfo_t *,
                          SuperLUStat_t *, int *);
int_t slu_refimpl_psgstrf(superlu_dist_options_t *, int, int, float, sLUstruct_t *, gridinfo_t *,
                          SuperLUStat_t *, int *);
int_t slu_refimpl_pzgstrf(superlu_dist_options_t *, int, int, double, zLUstruct_t *, gridinfo_t *,
                          SuperLUStat_t *, int *);

static const char *g_out = NULL;
static int g_iam = 0;
static void *g_sp = NULL; /* the ScalePermstruct pdgssvx is filling */
static char g_dt = 'd';
static FILE *g_meta = NULL;

/* ---- .npy writer (format 1.0) ---- */
static void npy(const char *name, const char *descr, const void *p, long cnt, int esz) {
    char fn[2048], hdr[256];
    snprintf(fn, sizeof fn, "%s/r%d_%s.npy", g_out, g_iam, name);
    FILE *f = fopen(fn, "wb");
    if (!f) { fprintf(stderr, "cannot write %s\n", fn); MPI_Abort(MPI_COMM_WORLD, 1); }
    int hl = snprintf(hdr, sizeof hdr, "{'descr': '%s', 'fortran_order': False, 'shape': (%ld,), }",
                      descr, cnt);
    int tot = 10 + hl + 1;
    int pad = (64 - tot % 64) % 64;
    unsigned short hlen = (unsigned short)(hl + pad + 1);
    fwrite("\x93NUMPY\x01\x00", 1, 8, f);
    fwrite(&hlen, 2, 1, f);
    fwrite(hdr, 1, hl, f);
    for (int i = 0; i < pad; ++i) fputc(' ', f);
    fputc('\n', f);
    if (cnt) fwrite(p, esz, cnt, f);
    fclose(f);
}
static void npy_i64(const char *name, const int_t *p, long cnt) { npy(name, "<i8", p, cnt, 8); }
static void npy_i32(const char *name, const int *p, long cnt) { npy(name, "<i4", p, cnt, 4); }
static void npy_val(const char *name, const void *p, long cnt) {
    if (g_dt == 's') npy(name, "<f4", p, cnt, 4);
    else if (g_dt == 'z') npy(name, "<c16", p, cnt, 16);
    else npy(name, "<f8", p, cnt, 8);
}


/* Re-serialises one rank's LUstruct: the index arrays per local block
 * column / row (offsets -1 where empty) in the formats of SRC/superlu_defs.h:
 * 152-190, the values likewise, and the communication schedule of
 * SRC/pddistribute.c:752-801. */
#define DUMP_LU(P, LocalLU_t, LUstruct_t, T)                                                       \
    static void P##dump_lu(LUstruct_t *LU, gridinfo_t *grid, int n, const char *tag, int structure) \
    {                                                                                             \
        LocalLU_t *Llu = LU->Llu;                                                                 \
        int_t *xsup = LU->Glu_persist->xsup;                                                      \
        int nsupers = (int)LU->Glu_persist->supno[n - 1] + 1;                                     \
        int Pr = (int)grid->nprow, Pc = (int)grid->npcol;                                         \
        int mycol = g_iam % Pc, myrow = g_iam / Pc;                                               \
        int nlc = (nsupers + Pc - 1) / Pc, nlr = (nsupers + Pr - 1) / Pr;                        \
        int_t *loff = malloc(sizeof(int_t) * (nlc + 1)), *lvoff = malloc(sizeof(int_t) * (nlc + 1)); \
        int_t *uoff = malloc(sizeof(int_t) * (nlr + 1)), *uvoff = malloc(sizeof(int_t) * (nlr + 1)); \
        long li = 0, lv = 0, ui = 0, uv = 0;                                                      \
        for (int ljb = 0; ljb < nlc; ++ljb) {                                                     \
            int_t *ix = Llu->Lrowind_bc_ptr[ljb];                                                 \
            loff[ljb] = lvoff[ljb] = -1;                                                          \
            if (!ix) continue;                                                                    \
            int jb = ljb * Pc + mycol;                                                            \
            long len = BC_HEADER;                                                                 \
            for (int b = 0; b < ix[0]; ++b) len += LB_DESCRIPTOR + ix[len + 1];                   \
            loff[ljb] = li; lvoff[ljb] = lv;                                                      \
            li += len; lv += (long)ix[1] * (xsup[jb + 1] - xsup[jb]);                             \
        }                                                                                         \
        for (int lb = 0; lb < nlr; ++lb) {                                                        \
            int_t *ix = Llu->Ufstnz_br_ptr[lb];                                                   \
            uoff[lb] = uvoff[lb] = -1;                                                            \
            if (!ix) continue;                                                                    \
            uoff[lb] = ui; uvoff[lb] = uv;                                                        \
            ui += ix[2]; uv += ix[1];                                                             \
        }                                                                                         \
        int_t *lidx = malloc(sizeof(int_t) * (li + 1)), *uidx = malloc(sizeof(int_t) * (ui + 1)); \
        T *lval = malloc(sizeof(T) * (lv + 1)), *uval = malloc(sizeof(T) * (uv + 1));            \
        for (int ljb = 0; ljb < nlc; ++ljb) {                                                     \
            if (loff[ljb] < 0) continue;                                                          \
            int_t *ix = Llu->Lrowind_bc_ptr[ljb];                                                 \
            int jb = ljb * Pc + mycol;                                                            \
            long len = BC_HEADER;                                                                 \
            for (int b = 0; b < ix[0]; ++b) len += LB_DESCRIPTOR + ix[len + 1];                   \
            memcpy(lidx + loff[ljb], ix, len * sizeof(int_t));                                    \
            memcpy(lval + lvoff[ljb], Llu->Lnzval_bc_ptr[ljb],                                    \
                   sizeof(T) * ix[1] * (xsup[jb + 1] - xsup[jb]));                                \
        }                                                                                         \
        for (int lb = 0; lb < nlr; ++lb) {                                                        \
            if (uoff[lb] < 0) continue;                                                           \
            int_t *ix = Llu->Ufstnz_br_ptr[lb];                                                   \
            memcpy(uidx + uoff[lb], ix, ix[2] * sizeof(int_t));                                   \
            memcpy(uval + uvoff[lb], Llu->Unzval_br_ptr[lb], sizeof(T) * ix[1]);                  \
        }                                                                                         \
        char nm[64];                                                                              \
        snprintf(nm, sizeof nm, "%s_Lval", tag); npy_val(nm, lval, lv);                            \
        snprintf(nm, sizeof nm, "%s_Uval", tag); npy_val(nm, uval, uv);                            \
        if (structure) {                                                                          \
            npy_i64("Lidx", lidx, li); npy_i64("Loff", loff, nlc); npy_i64("Lvoff", lvoff, nlc);  \
            npy_i64("Uidx", uidx, ui); npy_i64("Uoff", uoff, nlr); npy_i64("Uvoff", uvoff, nlr);  \
            npy_i64("xsup", xsup, nsupers + 1);                                                   \
            npy_i64("supno", LU->Glu_persist->supno, n);                                          \
            npy_i32("ToRecv", Llu->ToRecv, nsupers);                                              \
            npy_i32("ToSendD", Llu->ToSendD, nlr);                                                \
            int *tsr = malloc(sizeof(int) * ((long)nlc * Pc + 1));                                \
            for (int i = 0; i < nlc; ++i)                                                         \
                for (int p = 0; p < Pc; ++p) tsr[(long)i * Pc + p] = Llu->ToSendR[i][p];          \
            npy_i32("ToSendR", tsr, (long)nlc * Pc);                                              \
            free(tsr);                                                                            \
            npy_i64("bufmax", Llu->bufmax, NBUFFERS);                                             \
            fprintf(g_meta, "\"nsupers\": %d, \"myrow\": %d, \"mycol\": %d, ", nsupers, myrow,    \
                    mycol);                                                                       \
        }                                                                                         \
        free(loff); free(lvoff); free(uoff); free(uvoff);                                         \
        free(lidx); free(uidx); free(lval); free(uval);                                           \
    }

DUMP_LU(d, dLocalLU_t, dLUstruct_t, double)
DUMP_LU(s, sLocalLU_t, sLUstruct_t, float)
DUMP_LU(z, zLocalLU_t, zLUstruct_t, doublecomplex)

/* perm_r / perm_c / R / C of the ScalePermstruct, as pdgssvx left them for
 * pddistribute (the row permutation Pc*Pr is applied inside it). */
#define DUMP_SP(P, SP_t, RT, descr)                                                                \
    static void P##dump_sp(int m, int n) {                                                        \
        SP_t *sp = (SP_t *)g_sp;                                                                  \
        npy_i64("perm_r", sp->perm_r, m);                                                         \
        npy_i64("perm_c", sp->perm_c, n);                                                         \
        int ds = (int)sp->DiagScale;                                                              \
        fprintf(g_meta, "\"DiagScale\": %d, ", ds);                                               \
        if (ds == ROW || ds == BOTH) npy("R", descr, sp->R, m, sizeof(RT));                       \
        if (ds == COL || ds == BOTH) npy("C", descr, sp->C, n, sizeof(RT));                       \
    }
DUMP_SP(d, dScalePermstruct_t, double, "<f8")
DUMP_SP(s, sScalePermstruct_t, float, "<f4")
DUMP_SP(z, zScalePermstruct_t, double, "<f8")

#define INTERPOSE(P, LUstruct_t, AT)                                                               \
    int_t p##P##gstrf(superlu_dist_options_t *options, int m, int n, AT anorm,                     \
                      LUstruct_t *LU, gridinfo_t *grid, SuperLUStat_t *stat, int *info) {          \
        P##dump_lu(LU, grid, n, "pre", 1);                                                        \
        P##dump_sp(m, n);                                                                         \
        int tiny0 = stat->TinyPivots;                                                             \
        int_t r = slu_refimpl_p##P##gstrf(options, m, n, anorm, LU, grid, stat, info);            \
        P##dump_lu(LU, grid, n, "post", 0);                                                       \
        fprintf(g_meta, "\"anorm\": %.17g, \"info\": %d, \"tiny\": %d, \"ops\": %.9g, "           \
                "\"replace_tiny\": %d, \"num_lookaheads\": %d, \"relax\": %d, \"maxsup\": %d, ",    \
                (double)anorm, *info, stat->TinyPivots - tiny0, (double)stat->ops[FACT],          \
                options->ReplaceTinyPivot == YES, options->num_lookaheads,                        \
                sp_ienv_dist(2, options), sp_ienv_dist(3, options));                              \
        return r;                                                                                 \
    }
INTERPOSE(d, dLUstruct_t, double)
INTERPOSE(s, sLUstruct_t, float)
INTERPOSE(z, zLUstruct_t, double)

static int_t *read_perm(const char *fn, int_t n) {
    FILE *f = fopen(fn, "rb");
    if (!f) { fprintf(stderr, "cannot open %s\n", fn); MPI_Abort(MPI_COMM_WORLD, 1); }
    int_t *p = malloc(sizeof(int_t) * n);
    if ((int_t)fread(p, sizeof(int_t), n, f) != n) MPI_Abort(MPI_COMM_WORLD, 1);
    fclose(f);
    return p;
}

static void set_options(superlu_dist_options_t *o, int rowperm, int colperm, int equil, int tiny,
                        int look, int ir, int relax, int maxsup) {
    set_default_options_dist(o);
    o->ColPerm = MMD_AT_PLUS_A; /* METIS is not in the image */
    o->ParSymbFact = NO;
    o->PrintStat = NO;
    if (rowperm >= 0) o->RowPerm = rowperm;
    if (colperm >= 0) o->ColPerm = colperm;
    if (equil >= 0) o->Equil = equil ? YES : NO;
    if (tiny >= 0) o->ReplaceTinyPivot = tiny ? YES : NO;
    if (look >= 0) o->num_lookaheads = look;
    if (ir >= 0) o->IterRefine = ir;
    if (relax > 0) o->superlu_relax = relax;
    if (maxsup > 0) o->superlu_maxsup = maxsup;
}

/* One solve path per value type: create A/b/xtrue the way p?drive does,
 * call p?gssvx (which calls the interposer), dump x / berr, then solve again
 * from the same factors without refinement. */
#define RUN(P, T, SP_t, BT)                                                                            \
    static void P##run(FILE *fp, char *postfix, gridinfo_t *grid, int nrhs, int_t *permc,         \
                       superlu_dist_options_t *opt) {                                             \
        SuperMatrix A;                                                                            \
        T *b, *xtrue;                                                                             \
        int ldb, ldx, info = 0;                                                                   \
        P##create_matrix_postfix(&A, nrhs, &b, &ldb, &xtrue, &ldx, fp, postfix, grid);            \
        int m = (int)A.nrow, n = (int)A.ncol;                                                     \
        NRformat_loc *S = (NRformat_loc *)A.Store;                                                \
        int m_loc = (int)S->m_loc;                                                                \
        T *b0 = malloc(sizeof(T) * (size_t)ldb * nrhs);                                           \
        memcpy(b0, b, sizeof(T) * (size_t)ldb * nrhs);                                            \
        SP_t SP;                                                                                  \
        P##LUstruct_t LU;                                                                         \
        P##SOLVEstruct_t SV;                                                                      \
        SuperLUStat_t stat;                                                                       \
        P##ScalePermstructInit(m, n, &SP);                                                        \
        if (permc) memcpy(SP.perm_c, permc, sizeof(int_t) * n);                                   \
        P##LUstructInit(n, &LU);                                                                  \
        PStatInit(&stat);                                                                         \
        g_sp = &SP;                                                                               \
        BT *berr = malloc(sizeof(BT) * nrhs);                                                       \
        p##P##gssvx(opt, &A, &SP, b, ldb, nrhs, grid, &LU, &SV, berr, &stat, &info);                 \
        fprintf(g_meta, "\"gssvx_info\": %d, \"refine_steps\": %d, \"m_loc\": %d, "               \
                "\"fst_row\": %lld, \"n\": %d, \"nrhs\": %d, \"ldb\": %d, ",                        \
                info, stat.RefineSteps, m_loc, (long long)S->fst_row, n, nrhs, ldb);              \
        npy_val("x", b, (long)ldb * nrhs);                                                        \
        npy_val("b", b0, (long)ldb * nrhs);                                                       \
        npy_val("xtrue", xtrue, (long)ldx * nrhs);                                                \
        npy("berr", sizeof(BT) == 4 ? "<f4" : "<f8", berr, nrhs, (int)sizeof(BT));                \
        /* A as pdgssvx received it (local rows, CSR), for the refinement */                     \
        npy_i64("A_rowptr", S->rowptr, m_loc + 1);                                                \
        npy_i64("A_colind", S->colind, S->nnz_loc);                                               \
        npy_val("A_val", S->nzval, S->nnz_loc);                                                   \
        if (info == 0) {                                                                          \
            memcpy(b, b0, sizeof(T) * (size_t)ldb * nrhs);                                        \
            opt->Fact = FACTORED;                                                                 \
            opt->IterRefine = NOREFINE;                                                           \
            p##P##gssvx(opt, &A, &SP, b, ldb, nrhs, grid, &LU, &SV, berr, &stat, &info);              \
            npy_val("x_norefine", b, (long)ldb * nrhs);                                           \
        }                                                                                         \
        fprintf(g_meta, "\"dtype\": \"%c\"}\n", g_dt);                                            \
    }
RUN(d, double, dScalePermstruct_t, double)
RUN(s, float, sScalePermstruct_t, float)
RUN(z, doublecomplex, zScalePermstruct_t, double)

int main(int argc, char **argv) {
    int prov;
    MPI_Init_thread(&argc, &argv, MPI_THREAD_MULTIPLE, &prov);
    int nprow = 1, npcol = 1, relax = -1, maxsup = -1, rowperm = -1, colperm = -1, equil = -1;
    int tiny = -1, look = -1, ir = -1, nrhs = 1;
    const char *permfile = NULL, *mfile = NULL;
    for (int i = 1; i < argc; ++i) {
        if (argv[i][0] == '-' && i + 1 < argc) {
            const char *v = argv[i + 1];
            switch (argv[i][1]) {
            case 't': g_dt = v[0]; break;
            case 'o': g_out = v; break;
            case 'r': nprow = atoi(v); break;
            case 'c': npcol = atoi(v); break;
            case 'x': relax = atoi(v); break;
            case 'm': maxsup = atoi(v); break;
            case 'p': rowperm = atoi(v); break;
            case 'q': colperm = atoi(v); break;
            case 'e': equil = atoi(v); break;
            case 'y': tiny = atoi(v); break;
            case 'l': look = atoi(v); break;
            case 'i': ir = atoi(v); break;
            case 's': nrhs = atoi(v); break;
            case 'P': permfile = v; break;
            }
            ++i;
        } else {
            mfile = argv[i];
        }
    }
    if (!g_out || !mfile) {
        fprintf(stderr, "usage: ref_dump -t d|s|z -o OUTDIR [options] MATRIX\n");
        MPI_Abort(MPI_COMM_WORLD, 2);
    }
    gridinfo_t grid;
    superlu_gridinit(MPI_COMM_WORLD, nprow, npcol, &grid);
    g_iam = grid.iam;
    char mfn[2048];
    snprintf(mfn, sizeof mfn, "%s/meta_%d.json", g_out, g_iam);
    g_meta = fopen(mfn, "w");
    fprintf(g_meta, "{\"nprow\": %d, \"npcol\": %d, \"iam\": %d, ", nprow, npcol, g_iam);
    FILE *fp = fopen(mfile, "r");
    if (!fp) { fprintf(stderr, "cannot open %s\n", mfile); MPI_Abort(MPI_COMM_WORLD, 1); }
    char *postfix = strrchr(mfile, '.');
    postfix = postfix ? postfix + 1 : (char *)"rua";
    superlu_dist_options_t opt;
    set_options(&opt, rowperm, colperm, equil, tiny, look, ir, relax, maxsup);
    int_t *permc = NULL;
    if (permfile) {
        /* n from the perm file size */
        FILE *pf = fopen(permfile, "rb");
        fseek(pf, 0, SEEK_END);
        int_t n = ftell(pf) / sizeof(int_t);
        fclose(pf);
        permc = read_perm(permfile, n);
        opt.ColPerm = MY_PERMC;
    }
    if (g_dt == 'd') drun(fp, postfix, &grid, nrhs, permc, &opt);
    else if (g_dt == 's') srun(fp, postfix, &grid, nrhs, permc, &opt);
    else zrun(fp, postfix, &grid, nrhs, permc, &opt);
    fclose(g_meta);
    superlu_gridexit(&grid);
    MPI_Finalize();
    return 0;
}

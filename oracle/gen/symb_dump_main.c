/* TEST INFRASTRUCTURE: runs the REFERENCE's column ordering post-pass and
 * symbolic factorization exactly as pdgssvx does (SRC/pdgssvx.c:1029-1076:
 * get_perm_c_dist, sp_colorder, the Pc relabelling of GAC's rows, symbfact)
 * on a pattern read from a file, and dumps every array they produce.
 * -> tests/golden/symb_*.npz (oracle/gen/make_symb_golden.py).
 *
 *   symb_dump IN OUT COLPERM RELAX MAXSUP
 *     IN   int64 m, n, nnz, colptr[n+1], rowind[nnz]; perm_c[n] follows
 *          when COLPERM = 7 (MY_PERMC)
 *     OUT  records: char name[16], int64 count, int64 data[count]
 *   prints "colperm_s colorder_s symbfact_s" on stdout.
 */
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include "superlu_ddefs.h"

static void put(FILE *f, const char *name, const int_t *v, int64_t n) {
    char nm[16] = {0};
    strncpy(nm, name, 15);
    fwrite(nm, 1, 16, f);
    fwrite(&n, 8, 1, f);
    if (n) fwrite(v, 8, (size_t)n, f);
}

static int64_t rd1(FILE *f) {
    int64_t x;
    if (fread(&x, 8, 1, f) != 1) { fprintf(stderr, "short read\n"); exit(2); }
    return x;
}

int main(int argc, char **argv) {
    if (argc < 6) { fprintf(stderr, "usage: symb_dump IN OUT COLPERM RELAX MAXSUP\n"); return 2; }
    MPI_Init(&argc, &argv);
    FILE *fi = fopen(argv[1], "rb");
    if (!fi) { perror(argv[1]); return 2; }
    const int colperm = atoi(argv[3]);
    int_t m = rd1(fi), n = rd1(fi), nnz = rd1(fi);
    int_t *colptr = intMalloc_dist(n + 1), *rowind = intMalloc_dist(nnz > 0 ? nnz : 1);
    if (fread(colptr, 8, n + 1, fi) != (size_t)(n + 1)) return 2;
    if (nnz && fread(rowind, 8, nnz, fi) != (size_t)nnz) return 2;
    int_t *perm_c = intMalloc_dist(n), *etree = intMalloc_dist(n);
    if (colperm == MY_PERMC)
        if (fread(perm_c, 8, n, fi) != (size_t)n) return 2;
    fclose(fi);
    double *val = doubleMalloc_dist(nnz > 0 ? nnz : 1);
    for (int_t i = 0; i < nnz; ++i) val[i] = 1.0;

    superlu_dist_options_t options;
    set_default_options_dist(&options);
    options.Fact = DOFACT;
    options.ColPerm = colperm;
    options.superlu_relax = atoi(argv[4]);
    options.superlu_maxsup = atoi(argv[5]);

    SuperMatrix A, AC;
    dCreate_CompCol_Matrix_dist(&A, m, n, nnz, val, rowind, colptr, SLU_NC, SLU_D, SLU_GE);

    double t0 = SuperLU_timer_();
    if (colperm == NATURAL)
        for (int_t j = 0; j < n; ++j) perm_c[j] = j;
    else if (colperm != MY_PERMC)
        get_perm_c_dist(0, colperm, &A, perm_c);
    double t1 = SuperLU_timer_();

    FILE *fo = fopen(argv[2], "wb");
    put(fo, "colptr", colptr, n + 1);
    put(fo, "rowind", rowind, nnz);
    put(fo, "perm_c_in", perm_c, n);

    sp_colorder(&options, &A, perm_c, etree, &AC);
    NCPformat *S = (NCPformat *)AC.Store;
    for (int_t j = 0; j < n; ++j)
        for (int_t i = S->colbeg[j]; i < S->colend[j]; ++i) S->rowind[i] = perm_c[S->rowind[i]];
    double t2 = SuperLU_timer_();

    Glu_persist_t gp;
    Glu_freeable_t gf;
    int_t ret = symbfact(&options, 0, &AC, perm_c, etree, &gp, &gf);
    double t3 = SuperLU_timer_();

    put(fo, "perm_c", perm_c, n);
    put(fo, "etree", etree, n);
    put(fo, "colbeg", S->colbeg, n);
    put(fo, "colend", S->colend, n);
    put(fo, "xsup", gp.xsup, gp.supno[n] + 2);
    put(fo, "supno", gp.supno, n + 1);
    put(fo, "xlsub", gf.xlsub, n + 1);
    put(fo, "lsub", gf.lsub, gf.xlsub[n]);
    put(fo, "xusub", gf.xusub, n + 1);
    put(fo, "usub", gf.usub, gf.xusub[n]);
    int_t sc[4] = {ret, gf.nnzLU, sp_ienv_dist(2, &options), sp_ienv_dist(3, &options)};
    put(fo, "scalars", sc, 4);
    fclose(fo);
    printf("%.6f %.6f %.6f\n", t1 - t0, t2 - t1, t3 - t2);
    MPI_Finalize();
    return 0;
}

/*
 * blocksum.h -- TEST INFRASTRUCTURE (the checker, never the product path).
 *
 * Per-block fingerprints of a factored LUstruct, so that factors of the full
 * 100^3 headline problem (17 GB) can be compared between the reference's
 * pdgstrf on a CPU grid and the GPU factorization on another grid without
 * moving either set of factors: every L block (ib, jb) and U block (ib, jb) of
 * a rank gives one record keyed by its GLOBAL block coordinates, so records of
 * different process grids match up one to one.
 *
 *   cnt     stored values of the block
 *   maxabs  max |v| (complex: |re| + |im|, slud_z_abs1)
 *   wre/wim sum of w(r, c) * v over the block, w a fixed pseudo-random weight
 *           in [-1, 1) of the value's global (row, column): a random
 *           projection, so |wsum_gpu - wsum_ref| ~ the block's 2-norm error
 *
 * Layouts walked (the library's flat view of the reference layout,
 * SRC/superlu_defs.h:152-198; SRC/pddistribute.c:1283-1340, 1465-1493):
 *   L block column ljb (jb = ljb*Pc + mycol): index at Loff[ljb] =
 *     [nblocks, nsupr, {gb, nrows, rows[nrows]}...], values nsupr x nsupc
 *     column major at Lvoff[ljb], block rows stacked in index order.
 *   U block row lb (ib = lb*Pr + myrow): index at Uoff[lb] =
 *     [nblocks, len(nzval), len(index), {jb, nnz, fstnz[nsupc(jb)]}...],
 *     values = the column segments [fstnz, xsup[ib+1]) in (block, column)
 *     order at Uvoff[lb].
 */
#ifndef SLU_ORACLE_BLOCKSUM_H
#define SLU_ORACLE_BLOCKSUM_H
#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

typedef struct {
    int64_t kind; /* 0 = L block, 1 = U block */
    int64_t ib, jb, cnt;
    double maxabs, wre, wim;
} blocksum_rec;

static inline double blocksum_weight(int64_t r, int64_t c) {
    uint64_t z = ((uint64_t)r << 32) ^ (uint64_t)c;
    z += 0x9E3779B97F4A7C15ull; /* splitmix64 */
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    z ^= z >> 31;
    return (double)(z >> 11) * (2.0 / 9007199254740992.0) - 1.0;
}

static inline void blocksum_val(int dtype, const void *vals, int64_t i, double *re, double *im) {
    if (dtype == 1) { *re = ((const float *)vals)[i]; *im = 0; }
    else if (dtype == 2) { *re = ((const double *)vals)[2 * i]; *im = ((const double *)vals)[2 * i + 1]; }
    else { *re = ((const double *)vals)[i]; *im = 0; }
}

static inline void blocksum_add(blocksum_rec *b, double re, double im, int64_t r, int64_t c) {
    const double w = blocksum_weight(r, c), a = fabs(re) + fabs(im);
    b->cnt++;
    if (a > b->maxabs) b->maxabs = a;
    b->wre += w * re;
    b->wim += w * im;
}

/* Records of one block column (L, ljb) or block row (U, lb) into out + at. */
static inline int64_t blocksum_lcol(int dtype, const int64_t *xsup, const int64_t *ix,
                                    const void *Lval, int64_t voff, int64_t jb, blocksum_rec *out) {
    const int64_t nb = ix[0], nsupr = ix[1], fc = xsup[jb], w = xsup[jb + 1] - fc;
    int64_t p = 2, r0 = 0;
    for (int64_t b = 0; b < nb; ++b) {
        const int64_t gb = ix[p], nr = ix[p + 1];
        if (out) {
            blocksum_rec *o = &out[b];
            o->kind = 0; o->ib = gb; o->jb = jb; o->cnt = 0;
            o->maxabs = o->wre = o->wim = 0;
            for (int64_t c = 0; c < w; ++c)
                for (int64_t i = 0; i < nr; ++i) {
                    double re, im;
                    blocksum_val(dtype, Lval, voff + c * nsupr + r0 + i, &re, &im);
                    blocksum_add(o, re, im, ix[p + 2 + i], fc + c);
                }
        }
        r0 += nr;
        p += 2 + nr;
    }
    return nb;
}

static inline int64_t blocksum_urow(int dtype, const int64_t *xsup, const int64_t *ix,
                                    const void *Uval, int64_t v, int64_t ib, blocksum_rec *out) {
    const int64_t nb = ix[0], last = xsup[ib + 1];
    int64_t p = 3;
    for (int64_t b = 0; b < nb; ++b) {
        const int64_t jb = ix[p], fc = xsup[jb], w = xsup[jb + 1] - fc;
        if (out) {
            blocksum_rec *o = &out[b];
            o->kind = 1; o->ib = ib; o->jb = jb; o->cnt = 0;
            o->maxabs = o->wre = o->wim = 0;
            int64_t q = v;
            for (int64_t c = 0; c < w; ++c)
                for (int64_t r = ix[p + 2 + c]; r < last; ++r) {
                    double re, im;
                    blocksum_val(dtype, Uval, q++, &re, &im);
                    blocksum_add(o, re, im, r, fc + c);
                }
        }
        for (int64_t c = 0; c < w; ++c) v += last - ix[p + 2 + c];
        p += 2 + w;
    }
    return nb;
}

/* Records of one rank's blocks into out (NULL: count only), L block columns
 * then U block rows in local order; block columns / rows in parallel where
 * built with OpenMP.  Returns the number of records. */
static inline int64_t blocksum_compute(int dtype, int64_t nsupers, const int64_t *xsup,
                                       const int64_t *Lidx, const long *Loff, const void *Lval,
                                       const long *Lvoff, const int64_t *Uidx, const long *Uoff,
                                       const void *Uval, const long *Uvoff, int nprow, int npcol,
                                       int myrow, int mycol, blocksum_rec *out) {
    const int64_t nlc = (nsupers + npcol - 1) / npcol, nlr = (nsupers + nprow - 1) / nprow;
    int64_t *at = (int64_t *)calloc(nlc + nlr + 1, sizeof(int64_t)); /* record offsets */
    if (!at) return -1;
    for (int64_t e = 0; e < nlc + nlr; ++e) {
        int64_t nb = 0;
        if (e < nlc) {
            const int64_t jb = e * npcol + mycol;
            if (jb < nsupers && Loff[e] >= 0) nb = Lidx[Loff[e]];
        } else {
            const int64_t lb = e - nlc, ib = lb * nprow + myrow;
            if (ib < nsupers && Uoff[lb] >= 0) nb = Uidx[Uoff[lb]];
        }
        at[e + 1] = at[e] + nb;
    }
    const int64_t nrec = at[nlc + nlr];
    if (out) {
#pragma omp parallel for schedule(dynamic, 8)
        for (int64_t e = 0; e < nlc + nlr; ++e) {
            if (at[e + 1] == at[e]) continue;
            if (e < nlc)
                blocksum_lcol(dtype, xsup, Lidx + Loff[e], Lval, Lvoff[e], e * npcol + mycol,
                              out + at[e]);
            else
                blocksum_urow(dtype, xsup, Uidx + Uoff[e - nlc], Uval, Uvoff[e - nlc],
                              (e - nlc) * nprow + myrow, out + at[e]);
        }
    }
    free(at);
    return nrec;
}

#ifdef SLU_ORACLE_BLOCKSUM_WRITE
/* file: int64 nrec, then nrec records */
static inline int blocksum_write(const char *fn, int dtype, const slu_lu_view *v, int nprow,
                                 int npcol, int myrow, int mycol) {
    const int64_t n = blocksum_compute(dtype, v->nsupers, v->xsup, v->Lidx, v->Lidx_off, v->Lval,
                                       v->Lval_off, v->Uidx, v->Uidx_off, v->Uval, v->Uval_off,
                                       nprow, npcol, myrow, mycol, NULL);
    blocksum_rec *r = (blocksum_rec *)calloc(n > 0 ? n : 1, sizeof(blocksum_rec));
    if (!r) return -1;
    blocksum_compute(dtype, v->nsupers, v->xsup, v->Lidx, v->Lidx_off, v->Lval, v->Lval_off,
                     v->Uidx, v->Uidx_off, v->Uval, v->Uval_off, nprow, npcol, myrow, mycol, r);
    FILE *fp = fopen(fn, "wb");
    if (!fp) { free(r); return -1; }
    int ok = fwrite(&n, 8, 1, fp) == 1 && (int64_t)fwrite(r, sizeof *r, n, fp) == n;
    ok = (fclose(fp) == 0) && ok;
    free(r);
    return ok ? 0 : -1;
}
#endif
#endif

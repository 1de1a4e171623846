/*
 * oracle.c -- CPU restatement of SuperLU_DIST 8.1.1 pdgstrf / psgstrf /
 * pzgstrf (SRC/pdgstrf.c:242-2002 and the files it includes:
 * SRC/pdgstrf2.c, SRC/dscatter.c, SRC/dSchCompUdt-2Ddynamic.c,
 * SRC/dlook_ahead_update.c; s/z variants are type substitutions).
 *
 * TEST INFRASTRUCTURE: this is the checker.  Only tests/, __graft_entry__.smoke()
 * and bench.py's cpu_baseline leg may load oracle/_build/liboracle.so.  The
 * product path (libslu_mi355x.so) never links or calls it.
 *
 * Pinned against the reference itself: tests/golden/ref_*.npz hold the factors
 * produced by the reference pdgstrf (compiled from /root/reference/SRC by
 * oracle/Makefile into oracle/_ref/, run by oracle/gen/make_golden.py) on the
 * same LUstructs; tests/test_oracle.py checks this restatement against them.
 *
 * Entry points (all ranks of a Pr x Pc grid simulated in one process):
 *   int oracle_dfactor(int Pr, int Pc, void **LUs, int n, int replace_tiny,
 *                      double anorm, int *info, int *tiny, double *flops);
 *   int oracle_sfactor(...), oracle_zfactor(...)
 * LUs[p] is rank p's dLUstruct_t / sLUstruct_t / zLUstruct_t (p = row*Pc+col).
 */
#include <float.h>
#include <math.h>
#include <stdlib.h>
#include <string.h>

#include "slu_abi.h"

/* ---------------- double ---------------- */
#define F_SCALE(x) (x)
#define F_RANK1 2.0
#define F_TRSM 1.0
#define F_SCHUR 2.0
#define VT double
#define LUS dLUstruct_t
#define OR_NAME(x) d_##x
#define V_ZERO 0.0
#define V_ADD(a, b) ((a) + (b))
#define V_SUB(a, b) ((a) - (b))
#define V_MUL(a, b) ((a) * (b))
#define V_DIV(a, b) ((a) / (b))
#define V_ABS(a) fabs(a)
#define V_ISZERO(a) ((a) == 0.0)
#define V_RECIP(a) (1.0 / (a))
#define V_SET_THRESH(a, t) ((a) = ((a) < 0 ? -(t) : (t)))
#include "oracle_impl.h"
#undef VT
#undef LUS
#undef OR_NAME
#undef V_ZERO
#undef V_ADD
#undef V_SUB
#undef V_MUL
#undef V_DIV
#undef V_ABS
#undef V_ISZERO
#undef V_RECIP
#undef V_SET_THRESH

/* ---------------- float (SRC/psgstrf.c: thresh is float) ---------------- */
#define VT float
#define LUS sLUstruct_t
#define OR_NAME(x) s_##x
#define V_ZERO 0.0f
#define V_ADD(a, b) ((a) + (b))
#define V_SUB(a, b) ((a) - (b))
#define V_MUL(a, b) ((a) * (b))
#define V_DIV(a, b) ((a) / (b))
#define V_ABS(a) fabsf(a)
#define V_ISZERO(a) ((a) == 0.0f)
#define V_RECIP(a) (1.0f / (a))
#define V_SET_THRESH(a, t) ((a) = ((a) < 0 ? -(float)(t) : (float)(t)))
#include "oracle_impl.h"
#undef VT
#undef LUS
#undef OR_NAME
#undef V_ZERO
#undef V_ADD
#undef V_SUB
#undef V_MUL
#undef V_DIV
#undef V_ABS
#undef V_ISZERO
#undef V_RECIP
#undef V_SET_THRESH

/* ---------------- doublecomplex (SRC/dcomplex.h, SRC/dcomplex_dist.c) ---- */
static inline doublecomplex zc_add(doublecomplex a, doublecomplex b) {
    doublecomplex c = {a.r + b.r, a.i + b.i}; return c; }
static inline doublecomplex zc_sub(doublecomplex a, doublecomplex b) {
    doublecomplex c = {a.r - b.r, a.i - b.i}; return c; }
static inline doublecomplex zc_mul(doublecomplex a, doublecomplex b) {
    doublecomplex c = {a.r * b.r - a.i * b.i, a.i * b.r + a.r * b.i}; return c; }
/* slud_z_div, SRC/dcomplex_dist.c: Smith's scaled division */
static inline doublecomplex zc_div(doublecomplex a, doublecomplex b) {
    double ratio, den, abr = fabs(b.r), abi = fabs(b.i);
    doublecomplex c;
    if (abr <= abi) {
        ratio = b.r / b.i; den = b.i * (1 + ratio * ratio);
        c.r = (a.r * ratio + a.i) / den; c.i = (a.i * ratio - a.r) / den;
    } else {
        ratio = b.i / b.r; den = b.r * (1 + ratio * ratio);
        c.r = (a.r + a.i * ratio) / den; c.i = (a.i - a.r * ratio) / den;
    }
    return c;
}
static inline doublecomplex zc_recip(doublecomplex b) {
    doublecomplex one = {1.0, 0.0}; return zc_div(one, b); }
static inline double zc_abs1(doublecomplex a) { return fabs(a.r) + fabs(a.i); }
static const doublecomplex zc_zero = {0.0, 0.0};
#undef F_SCALE
#undef F_RANK1
#undef F_TRSM
#undef F_SCHUR
#define F_SCALE(x) (6.0 * (x) + 10.0)
#define F_RANK1 8.0
#define F_TRSM 4.0
#define F_SCHUR 8.0
#define VT doublecomplex
#define LUS zLUstruct_t
#define OR_NAME(x) z_##x
#define V_ZERO zc_zero
#define V_ADD(a, b) zc_add(a, b)
#define V_SUB(a, b) zc_sub(a, b)
#define V_MUL(a, b) zc_mul(a, b)
#define V_DIV(a, b) zc_div(a, b)
#define V_ABS(a) zc_abs1(a)
#define V_ISZERO(a) ((a).r == 0.0 && (a).i == 0.0)
#define V_RECIP(a) zc_recip(a)
#define V_SET_THRESH(a, t) ((a).r = ((a).r < 0 ? -(t) : (t)), (a).i = 0.0)
#include "oracle_impl.h"

int oracle_dfactor(int Pr, int Pc, void **LUs, int n, int rt, double anorm,
                   int *info, int *tiny, double *flops) {
    return d_factor(Pr, Pc, LUs, n, rt, anorm, info, tiny, flops);
}
int oracle_sfactor(int Pr, int Pc, void **LUs, int n, int rt, double anorm,
                   int *info, int *tiny, double *flops) {
    return s_factor(Pr, Pc, LUs, n, rt, (double)(float)anorm, info, tiny, flops);
}
int oracle_zfactor(int Pr, int Pc, void **LUs, int n, int rt, double anorm,
                   int *info, int *tiny, double *flops) {
    return z_factor(Pr, Pc, LUs, n, rt, anorm, info, tiny, flops);
}

/* Per-block fingerprints of one rank's factors (blocksum.h; the checker of
 * the full-size headline parity in bench.py's cpu_baseline leg).  Returns the
 * record count; out == NULL counts only. */
#include "blocksum.h"
int64_t oracle_blocksums(int dtype, int64_t nsupers, const int64_t *xsup, const int64_t *Lidx,
                         const long *Loff, const void *Lval, const long *Lvoff,
                         const int64_t *Uidx, const long *Uoff, const void *Uval,
                         const long *Uvoff, int nprow, int npcol, int myrow, int mycol,
                         blocksum_rec *out) {
    return blocksum_compute(dtype, nsupers, xsup, Lidx, Loff, Lval, Lvoff, Uidx, Uoff, Uval,
                            Uvoff, nprow, npcol, myrow, mycol, out);
}

// CDNA4 (gfx950) kernels of the numeric factorization.  Included by engine.hip.
//
// Every kernel is batched over the supernodes of one elimination level
// (a set of supernodes with no dependency between them) and reads its work
// items from a device array built once by the plan, so a factorization is a
// short, fixed sequence of launches per level.
//
//   k_diag_lu    diagonal-block LU without pivoting      SRC/pdgstrf2.c:213-269
//   k_trsm_l     L(:,k) := L(:,k) U_kk^{-1}              SRC/pdgstrf2.c:302-355
//   k_trsm_u     U(k,:) segments := L_kk^{-1} segments    SRC/pdgstrf2.c:843-887
//   k_schur      A(i,j) -= L(i,k) U(k,j): LDS-staged gather of the L rows and
//                zero-padded U segments, MFMA GEMM, fused indexed scatter
//                (dscatter_l / dscatter_u)               SRC/dSchCompUdt-2Ddynamic.c,
//                                                        SRC/dscatter.c:110-277
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "slu_abi.h"

namespace slu {

// ---------------------------------------------------------------- scalars
struct zc {
    double r, i;
};

template <typename T> struct S;
template <> struct S<double> {
    using T = double;
    __device__ static T zero() { return 0.0; }
    __device__ static T mul(T a, T b) { return a * b; }
    __device__ static T fms(T c, T a, T b) { return c - a * b; } // c - a*b
    __device__ static T div(T a, T b) { return a / b; }
    __device__ static T recip(T a) { return 1.0 / a; }
    __device__ static double abs1(T a) { return fabs(a); }
    __device__ static bool iszero(T a) { return a == 0.0; }
    __device__ static T thresh(T a, double t) { return a < 0 ? -t : t; }
    __device__ static void sub_to(T *p, T v) { *p -= v; }
    __device__ static void atomic_sub(T *p, T v) { unsafeAtomicAdd(p, -v); }
};
template <> struct S<float> {
    using T = float;
    __device__ static T zero() { return 0.0f; }
    __device__ static T mul(T a, T b) { return a * b; }
    __device__ static T fms(T c, T a, T b) { return c - a * b; }
    __device__ static T div(T a, T b) { return a / b; }
    __device__ static T recip(T a) { return 1.0f / a; }
    __device__ static double abs1(T a) { return fabsf(a); }
    __device__ static bool iszero(T a) { return a == 0.0f; }
    __device__ static T thresh(T a, double t) { return a < 0 ? -(float)t : (float)t; }
    __device__ static void sub_to(T *p, T v) { *p -= v; }
    __device__ static void atomic_sub(T *p, T v) { unsafeAtomicAdd(p, -v); }
};
template <> struct S<zc> {
    using T = zc;
    __device__ static T zero() { return {0.0, 0.0}; }
    __device__ static T mul(T a, T b) { return {a.r * b.r - a.i * b.i, a.i * b.r + a.r * b.i}; }
    __device__ static T fms(T c, T a, T b) {
        return {c.r - (a.r * b.r - a.i * b.i), c.i - (a.i * b.r + a.r * b.i)};
    }
    // slud_z_div (SRC/dcomplex_dist.c): Smith's scaled division
    __device__ static T div(T a, T b) {
        double ratio, den, abr = fabs(b.r), abi = fabs(b.i);
        T c;
        if (abr <= abi) {
            ratio = b.r / b.i; den = b.i * (1 + ratio * ratio);
            c.r = (a.r * ratio + a.i) / den; c.i = (a.i * ratio - a.r) / den;
        } else {
            ratio = b.i / b.r; den = b.r * (1 + ratio * ratio);
            c.r = (a.r + a.i * ratio) / den; c.i = (a.i - a.r * ratio) / den;
        }
        return c;
    }
    __device__ static T recip(T a) { return div({1.0, 0.0}, a); }
    __device__ static double abs1(T a) { return fabs(a.r) + fabs(a.i); } // slud_z_abs1
    __device__ static bool iszero(T a) { return a.r == 0.0 && a.i == 0.0; }
    __device__ static T thresh(T a, double t) { return {a.r < 0 ? -t : t, 0.0}; }
    __device__ static void sub_to(T *p, T v) { p->r -= v.r; p->i -= v.i; }
    __device__ static void atomic_sub(T *p, T v) {
        unsafeAtomicAdd(&p->r, -v.r);
        unsafeAtomicAdd(&p->i, -v.i);
    }
};

// ------------------------------------------------------------ work items
template <typename T> struct DiagItem {
    T *a;       // diagonal block (top of lusup)
    int ld;     // nsupr
    int w;      // nsupc
    int k;      // supernode
    int fcol;   // xsup[k]
};

template <typename T> struct TrsmLItem {
    T *x;        // first row of this chunk, column-major, ld = ldx
    const T *u;  // diagonal block (upper triangle used)
    int ldx, ldu, w, nrows;
};

template <typename T> struct TrsmUItem {
    const T *l;          // diagonal block (unit lower triangle used), ld = ldl
    T *ubase;            // base of the U values the offsets refer to
    const int64_t *voff; // per column: value offset of the segment
    const int *t0;       // per column: first row of the segment relative to xsup[k]
    int ldl, w, ncols, kmin;
};

// per supernode k of a level, everything the Schur tiles of k need
template <typename T> struct KInfo {
    const T *a;          // first L row below the diagonal block, column-major
    const T *ubase;      // base of U values (segments)
    const int64_t *cvoff; // per U column: segment value offset
    const int *ct0;      // per U column: segment start (relative to xsup[k])
    const int *rg;       // per L row: global row index
    const int *ra;       // per L row: index of its L block in the panel
    const int *cg;       // per U column: global column index
    const int *cb;       // per U column: index of its U block in the panel
    const int *pair;     // nLb x nUb destination handles
    int lda, m, n, kmin, kw, nub, atomic, pad;
};

struct TileItem {
    int kslot; // index into the level's KInfo array
    int tm, tn;
};

// destination tables
struct LBlk {          // one local L block (ib, jb)
    int64_t colvoff;   // offset of lusup of column jb in Lval
    int64_t mapoff;    // offset of its row map in Lmap (nsupc(ib) entries)
    int ld;            // nsupr of column jb
    int fcol;          // xsup[jb]
    int frow;          // xsup[ib]
    int pad;
};
struct UBlk {          // one local U block (ib, jb)
    int64_t coloff;    // offset of its per-column entries in ucol_voff/ucol_fst
    int fcol;          // xsup[jb]
    int pad;
};

// ------------------------------------------------------------- diag LU
// One workgroup per diagonal block; blocked right-looking LU (panels of NB
// columns) in place, thread-per-row.  Tiny-pivot replacement and the zero
// pivot test follow SRC/pdgstrf2.c:217-252 (reciprocal scaling).
constexpr int DIAG_NB = 16;
constexpr int DIAG_THREADS = 256;

template <typename T>
__global__ void __launch_bounds__(DIAG_THREADS)
k_diag_lu(const DiagItem<T> *items, double thresh, int replace_tiny,
          int *tiny_count, int *zpiv) {
    using Sx = S<T>;
    const DiagItem<T> it = items[blockIdx.x];
    T *A = it.a;
    const int ld = it.ld, w = it.w, tid = threadIdx.x;
    __shared__ T s_piv[DIAG_NB];        // reciprocal pivots of the panel
    __shared__ T s_l11[DIAG_NB][DIAG_NB];
    __shared__ T s_u12[DIAG_NB][512 + 1];
    __shared__ int s_zero;
    if (tid == 0) s_zero = 0;
    for (int j0 = 0; j0 < w; j0 += DIAG_NB) {
        const int jb = min(DIAG_NB, w - j0);
        // ---- panel factorization: columns j0..j0+jb-1, rows j0..w-1
        for (int j = j0; j < j0 + jb; ++j) {
            __syncthreads();
            if (tid == 0) {
                T p = A[j + (int64_t)j * ld];
                if (replace_tiny && Sx::abs1(p) < thresh) {
                    p = Sx::thresh(p, thresh);
                    A[j + (int64_t)j * ld] = p;
                    atomicAdd(tiny_count, 1);
                }
                if (Sx::iszero(p)) {
                    s_zero = 1;
                    atomicMax(&zpiv[it.k], it.fcol + j + 1);
                } else {
                    s_zero = 0;
                    s_piv[j - j0] = Sx::recip(p);
                }
            }
            __syncthreads();
            const bool z = s_zero;
            const T rp = s_piv[j - j0];
            for (int i = j + 1 + tid; i < w; i += DIAG_THREADS) {
                T lij = A[i + (int64_t)j * ld];
                if (!z) lij = Sx::mul(lij, rp);
                A[i + (int64_t)j * ld] = lij;
                for (int l = j + 1; l < j0 + jb; ++l)
                    A[i + (int64_t)l * ld] = Sx::fms(A[i + (int64_t)l * ld], lij, A[j + (int64_t)l * ld]);
            }
        }
        __syncthreads();
        const int c0 = j0 + jb;
        if (c0 >= w) break;
        // ---- U12 = L11^{-1} A12 (rows j0..j0+jb-1, columns c0..w-1)
        for (int e = tid; e < jb * jb; e += DIAG_THREADS) {
            int r = e % jb, c = e / jb;
            s_l11[r][c] = A[(j0 + r) + (int64_t)(j0 + c) * ld];
        }
        __syncthreads();
        for (int c = c0 + tid; c < w; c += DIAG_THREADS) {
            T x[DIAG_NB];
#pragma unroll
            for (int t = 0; t < DIAG_NB; ++t)
                if (t < jb) x[t] = A[(j0 + t) + (int64_t)c * ld];
#pragma unroll
            for (int t = 0; t < DIAG_NB; ++t) {
#pragma unroll
                for (int s = 0; s < DIAG_NB; ++s)
                    if (s < t && t < jb) x[t] = Sx::fms(x[t], s_l11[t][s], x[s]);
            }
#pragma unroll
            for (int t = 0; t < DIAG_NB; ++t)
                if (t < jb) {
                    A[(j0 + t) + (int64_t)c * ld] = x[t];
                    s_u12[t][c - c0] = x[t];
                }
        }
        __syncthreads();
        // ---- A22 -= L21 U12 (thread per row)
        for (int i = c0 + tid; i < w; i += DIAG_THREADS) {
            T l21[DIAG_NB];
#pragma unroll
            for (int t = 0; t < DIAG_NB; ++t)
                if (t < jb) l21[t] = A[i + (int64_t)(j0 + t) * ld];
            for (int c = c0; c < w; ++c) {
                T acc = A[i + (int64_t)c * ld];
#pragma unroll
                for (int t = 0; t < DIAG_NB; ++t)
                    if (t < jb) acc = Sx::fms(acc, l21[t], s_u12[t][c - c0]);
                A[i + (int64_t)c * ld] = acc;
            }
        }
    }
}

// ------------------------------------------------------------- TRSM (L)
// X := X U^{-1} for a chunk of <= 256 rows, thread per row, column blocks
// of TRSM_NB staged through LDS.
constexpr int TRSM_NB = 16;
constexpr int TRSM_THREADS = 256;

template <typename T>
__global__ void __launch_bounds__(TRSM_THREADS)
k_trsm_l(const TrsmLItem<T> *items) {
    using Sx = S<T>;
    const TrsmLItem<T> it = items[blockIdx.x];
    const int tid = threadIdx.x, w = it.w;
    __shared__ T sU[512][TRSM_NB + 1]; // U[0..j0+jb, j0..j0+jb]
    const bool active = tid < it.nrows;
    T *x = it.x + tid;
    for (int j0 = 0; j0 < w; j0 += TRSM_NB) {
        const int jb = min(TRSM_NB, w - j0);
        __syncthreads();
        for (int e = tid; e < (j0 + jb) * jb; e += TRSM_THREADS) {
            int l = e % (j0 + jb), t = e / (j0 + jb);
            sU[l][t] = it.u[l + (int64_t)(j0 + t) * it.ldu];
        }
        __syncthreads();
        if (!active) continue;
        T acc[TRSM_NB];
#pragma unroll
        for (int t = 0; t < TRSM_NB; ++t)
            if (t < jb) acc[t] = x[(int64_t)(j0 + t) * it.ldx];
        for (int l = 0; l < j0; ++l) {
            T xl = x[(int64_t)l * it.ldx];
#pragma unroll
            for (int t = 0; t < TRSM_NB; ++t)
                if (t < jb) acc[t] = Sx::fms(acc[t], xl, sU[l][t]);
        }
#pragma unroll
        for (int t = 0; t < TRSM_NB; ++t) {
#pragma unroll
            for (int s = 0; s < TRSM_NB; ++s)
                if (s < t && t < jb) acc[t] = Sx::fms(acc[t], acc[s], sU[j0 + s][t]);
            if (t < jb) acc[t] = Sx::div(acc[t], sU[j0 + t][t]);
        }
#pragma unroll
        for (int t = 0; t < TRSM_NB; ++t)
            if (t < jb) x[(int64_t)(j0 + t) * it.ldx] = acc[t];
    }
}

// ------------------------------------------------------------- TRSM (U)
// Each U column segment [t0, w) := L_kk(t0:w, t0:w)^{-1} segment (unit lower),
// thread per column, row blocks of TRSM_NB; rows above t0 act as zeros.
template <typename T>
__global__ void __launch_bounds__(TRSM_THREADS)
k_trsm_u(const TrsmUItem<T> *items) {
    using Sx = S<T>;
    const TrsmUItem<T> it = items[blockIdx.x];
    const int tid = threadIdx.x, w = it.w, kmin = it.kmin;
    __shared__ T sL[TRSM_NB][512 + 1]; // L[i0..i0+ib, kmin..i0+ib]
    const bool active = tid < it.ncols;
    int t0 = w;
    T *x = nullptr;
    if (active) {
        t0 = it.t0[tid];
        x = it.ubase + it.voff[tid] - t0; // x[t] valid for t >= t0
    }
    for (int i0 = kmin; i0 < w; i0 += TRSM_NB) {
        const int ib = min(TRSM_NB, w - i0);
        const int nc = i0 + ib - kmin;
        __syncthreads();
        for (int e = tid; e < ib * nc; e += TRSM_THREADS) {
            int t = e % ib, j = e / ib;
            sL[t][j] = it.l[(i0 + t) + (int64_t)(kmin + j) * it.ldl];
        }
        __syncthreads();
        if (!active || i0 + ib <= t0) continue;
        T acc[TRSM_NB];
#pragma unroll
        for (int t = 0; t < TRSM_NB; ++t)
            acc[t] = (t < ib && i0 + t >= t0) ? x[i0 + t] : Sx::zero();
        for (int j = max(t0, kmin); j < i0; ++j) {
            T xj = x[j];
#pragma unroll
            for (int t = 0; t < TRSM_NB; ++t)
                if (t < ib) acc[t] = Sx::fms(acc[t], sL[t][j - kmin], xj);
        }
#pragma unroll
        for (int t = 0; t < TRSM_NB; ++t) {
#pragma unroll
            for (int s = 0; s < TRSM_NB; ++s)
                if (s < t && t < ib && i0 + s >= t0)
                    acc[t] = Sx::fms(acc[t], sL[t][i0 + s - kmin], acc[s]);
        }
#pragma unroll
        for (int t = 0; t < TRSM_NB; ++t)
            if (t < ib && i0 + t >= t0) x[i0 + t] = acc[t];
    }
}

// ------------------------------------------------------------- Schur
// 64x64 output tile per 256-thread workgroup (2x2 waves of 32x32), K staged
// through LDS 16 deep.  A = L rows (column-major, straight from lusup),
// B = U segments gathered with zero padding above each segment's first row.
constexpr int SC_BM = 64, SC_BN = 64, SC_BK = 16, SC_THREADS = 256;

template <typename T> struct Mma;

// fp64: v_mfma_f64_16x16x4_f64.  A/B: lane l holds A[l&15][l>>4], B[l>>4][l&15];
// C/D: col = l&15, row = (l>>4) + 4*i  (cdna_hip_programming.md §3).
template <> struct Mma<double> {
    using acc_t = __attribute__((ext_vector_type(4))) double;
    static constexpr int KSTEP = 4;
    __device__ static acc_t zero() { return acc_t{0, 0, 0, 0}; }
    __device__ static void step(acc_t &c, double a, double b) {
        c = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c, 0, 0, 0);
    }
    __device__ static int row(int lane, int i) { return (lane >> 4) + 4 * i; }
    __device__ static double get(const acc_t &c, int i) { return c[i]; }
};
// fp32: v_mfma_f32_16x16x4_f32; C/D: col = l&15, row = 4*(l>>4) + i.
template <> struct Mma<float> {
    using acc_t = __attribute__((ext_vector_type(4))) float;
    static constexpr int KSTEP = 4;
    __device__ static acc_t zero() { return acc_t{0, 0, 0, 0}; }
    __device__ static void step(acc_t &c, float a, float b) {
        c = __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0);
    }
    __device__ static int row(int lane, int i) { return 4 * (lane >> 4) + i; }
    __device__ static float get(const acc_t &c, int i) { return c[i]; }
};
// complex fp64 on four real fp64 MFMAs: Cr += Ar Br - Ai Bi, Ci += Ar Bi + Ai Br.
struct zacc {
    Mma<double>::acc_t r, i;
};
template <> struct Mma<zc> {
    using acc_t = zacc;
    static constexpr int KSTEP = 4;
    __device__ static acc_t zero() { return {Mma<double>::zero(), Mma<double>::zero()}; }
    __device__ static void step(acc_t &c, zc a, zc b) {
        c.r = __builtin_amdgcn_mfma_f64_16x16x4f64(a.r, b.r, c.r, 0, 0, 0);
        c.r = __builtin_amdgcn_mfma_f64_16x16x4f64(-a.i, b.i, c.r, 0, 0, 0);
        c.i = __builtin_amdgcn_mfma_f64_16x16x4f64(a.r, b.i, c.i, 0, 0, 0);
        c.i = __builtin_amdgcn_mfma_f64_16x16x4f64(a.i, b.r, c.i, 0, 0, 0);
    }
    __device__ static int row(int lane, int i) { return (lane >> 4) + 4 * i; }
    __device__ static zc get(const acc_t &c, int i) { return {c.r[i], c.i[i]}; }
};

template <typename T>
__global__ void __launch_bounds__(SC_THREADS)
k_schur(const TileItem *tiles, const KInfo<T> *kinfo, T *Lval, T *Uval,
        const LBlk *lblk, const int *lmap, const UBlk *ublk,
        const int64_t *ucol_voff, const int *ucol_fst) {
    using Sx = S<T>;
    using M = Mma<T>;
    const TileItem ti = tiles[blockIdx.x];
    const KInfo<T> ki = kinfo[ti.kslot];
    const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
    const int wr = wid >> 1, wc = wid & 1;
    const int row0 = ti.tm * SC_BM, col0 = ti.tn * SC_BN;
    const int mrows = min(SC_BM, ki.m - row0), ncols = min(SC_BN, ki.n - col0);

    // LDS: staging for A (k-major) and B (k-major); reused for the C tile.
    constexpr int ALD = SC_BM + 1, BLD = SC_BN + 1, CLD = SC_BM + 1;
    constexpr int STAGE = SC_BK * ALD + SC_BK * BLD;
    constexpr int CSIZE = SC_BN * CLD;
    __shared__ T smem[STAGE > CSIZE ? STAGE : CSIZE];
    __shared__ int s_rg[SC_BM], s_ra[SC_BM], s_cg[SC_BN], s_cb[SC_BN];
    T *sA = smem, *sB = smem + SC_BK * ALD;

    if (tid < SC_BM) {
        int r = row0 + tid;
        s_rg[tid] = tid < mrows ? ki.rg[r] : 0;
        s_ra[tid] = tid < mrows ? ki.ra[r] : 0;
    } else if (tid < SC_BM + SC_BN) {
        int c = tid - SC_BM;
        s_cg[c] = c < ncols ? ki.cg[col0 + c] : 0;
        s_cb[c] = c < ncols ? ki.cb[col0 + c] : 0;
    }
    // B gather: thread owns column bc = tid>>2 and 4 consecutive k of the stage
    const int bc = tid >> 2, bk = (tid & 3) * 4;
    const bool bvalid = bc < ncols;
    int64_t bvoff = 0;
    int bt0 = 0;
    if (bvalid) {
        bvoff = ki.cvoff[col0 + bc];
        bt0 = ki.ct0[col0 + bc];
    }
    const T *ub = ki.ubase + bvoff - bt0; // ub[t] valid for t >= bt0
    // A gather: thread owns row ar = tid & 63, k = (tid>>6) + 4*s
    const int ar = tid & 63, ak = tid >> 6;
    const bool avalid = ar < mrows;
    const T *ap = ki.a + row0 + ar;

    typename M::acc_t acc[2][2];
#pragma unroll
    for (int a = 0; a < 2; ++a)
#pragma unroll
        for (int b = 0; b < 2; ++b) acc[a][b] = M::zero();

    for (int k0 = 0; k0 < ki.kw; k0 += SC_BK) {
        __syncthreads();
#pragma unroll
        for (int s = 0; s < SC_BK / 4; ++s) {
            int kk = ak + 4 * s;
            int t = ki.kmin + k0 + kk;
            T v = Sx::zero();
            if (avalid && k0 + kk < ki.kw) v = ap[(int64_t)t * ki.lda];
            sA[kk * ALD + ar] = v;
        }
#pragma unroll
        for (int s = 0; s < 4; ++s) {
            int kk = bk + s;
            int t = ki.kmin + k0 + kk;
            T v = Sx::zero();
            if (bvalid && k0 + kk < ki.kw && t >= bt0) v = ub[t];
            sB[kk * BLD + bc] = v;
        }
        __syncthreads();
#pragma unroll
        for (int ks = 0; ks < SC_BK; ks += M::KSTEP) {
            const int kl = ks + (lane >> 4);
            T a0 = sA[kl * ALD + wr * 32 + (lane & 15)];
            T a1 = sA[kl * ALD + wr * 32 + 16 + (lane & 15)];
            T b0 = sB[kl * BLD + wc * 32 + (lane & 15)];
            T b1 = sB[kl * BLD + wc * 32 + 16 + (lane & 15)];
            M::step(acc[0][0], a0, b0);
            M::step(acc[0][1], a0, b1);
            M::step(acc[1][0], a1, b0);
            M::step(acc[1][1], a1, b1);
        }
    }
    // ---- C tile through LDS, then column-contiguous scatter-subtract
    __syncthreads();
    T *sC = smem; // [col][row], ld CLD
#pragma unroll
    for (int fm = 0; fm < 2; ++fm)
#pragma unroll
        for (int fn = 0; fn < 2; ++fn)
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                int r = wr * 32 + fm * 16 + M::row(lane, i);
                int c = wc * 32 + fn * 16 + (lane & 15);
                sC[c * CLD + r] = M::get(acc[fm][fn], i);
            }
    __syncthreads();
    const int r = tid & 63;
    if (r >= mrows) return;
    const int gr = s_rg[r], a = s_ra[r];
    const int *prow = ki.pair + (int64_t)a * ki.nub;
    int lastb = -1, h = 0;
    int64_t rbase = 0; // L dest: colvoff + pos ; U dest: unused
    for (int c = tid >> 6; c < ncols; c += 4) {
        const T v = sC[c * CLD + r];
        const int b = s_cb[c], gc = s_cg[c];
        if (b != lastb) {
            lastb = b;
            h = prow[b];
            if (h >= 0) {
                const LBlk L = lblk[h];
                rbase = L.colvoff + lmap[L.mapoff + gr - L.frow] - (int64_t)L.fcol * L.ld;
            }
        }
        T *dst;
        if (h >= 0) {
            const int ld = lblk[h].ld;
            dst = Lval + rbase + (int64_t)gc * ld;
        } else {
            const UBlk U = ublk[~h];
            const int64_t e = U.coloff + gc - U.fcol;
            dst = Uval + ucol_voff[e] + gr - ucol_fst[e];
        }
        if (ki.atomic) Sx::atomic_sub(dst, v);
        else Sx::sub_to(dst, v);
    }
}

} // namespace slu

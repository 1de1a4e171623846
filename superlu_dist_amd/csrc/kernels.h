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

#include <type_traits>

#include "slu_abi.h"

namespace slu {

// ---------------------------------------------------------------- scalars
struct zc {
    double r, i;
};

// Fire-and-forget atomic add through a GLOBAL pointer (global_atomic_add_*):
// through a generic pointer the compiler emits flat_atomic_add_*, which
// also counts in lgkmcnt, so the s_waitcnt lgkmcnt(0) before each of the
// Schur epilogue's barriers also waited for the wave's atomics.  (Measured
// neutral at 100^3: 0.597-0.599 either way, profiles/r06atom/.)  Callers
// pass global memory only.
template <typename X> __device__ __forceinline__ void global_atomic_add(X *p, X v) {
    __hip_atomic_fetch_add((__attribute__((address_space(1))) X *)p, v, __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_AGENT);
}

template <typename T> struct S;
template <> struct S<double> {
    using T = double;
    __device__ static T zero() { return 0.0; }
    __device__ static T neg(T a) { return -a; }
    __device__ static T mul(T a, T b) { return a * b; }
    __device__ static T fms(T c, T a, T b) { return c - a * b; } // c - a*b
    __device__ static T div(T a, T b) { return a / b; }
    __device__ static T recip(T a) { return 1.0 / a; }
    __device__ static double abs1(T a) { return fabs(a); }
    __device__ static bool iszero(T a) { return a == 0.0; }
    __device__ static T thresh(T a, double t) { return a < 0 ? -t : t; }
    __device__ static void sub_to(T *p, T v) { *p -= v; }
    __device__ static T sub(T a, T b) { return a - b; }
    __device__ static void atomic_sub(T *p, T v) { global_atomic_add(p, -v); }
};
template <> struct S<float> {
    using T = float;
    __device__ static T zero() { return 0.0f; }
    __device__ static T neg(T a) { return -a; }
    __device__ static T mul(T a, T b) { return a * b; }
    __device__ static T fms(T c, T a, T b) { return c - a * b; }
    __device__ static T div(T a, T b) { return a / b; }
    __device__ static T recip(T a) { return 1.0f / a; }
    __device__ static double abs1(T a) { return fabsf(a); }
    __device__ static bool iszero(T a) { return a == 0.0f; }
    __device__ static T thresh(T a, double t) { return a < 0 ? -(float)t : (float)t; }
    __device__ static void sub_to(T *p, T v) { *p -= v; }
    __device__ static T sub(T a, T b) { return a - b; }
    __device__ static void atomic_sub(T *p, T v) { global_atomic_add(p, -v); }
};
template <> struct S<zc> {
    using T = zc;
    __device__ static T zero() { return {0.0, 0.0}; }
    __device__ static T neg(T a) { return {-a.r, -a.i}; }
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
    __device__ static T sub(T a, T b) { return {a.r - b.r, a.i - b.i}; }
    __device__ static void atomic_sub(T *p, T v) {
        global_atomic_add(&p->r, -v.r);
        global_atomic_add(&p->i, -v.i);
    }
};

// v if c else 0 without control flow.  In k_schur_big a short-circuit
// (c1 && c2) ? v : 0 at the LDS store let the compiler sink the global load
// feeding v into a branch behind the stage's MFMAs, exposing its latency.
__device__ __forceinline__ double keep_if(bool c, double v) {
    return __longlong_as_double(__double_as_longlong(v) & -(long long)c);
}
__device__ __forceinline__ float keep_if(bool c, float v) {
    return __int_as_float(__float_as_int(v) & -(int)c);
}
__device__ __forceinline__ zc keep_if(bool c, zc v) { return {keep_if(c, v.r), keep_if(c, v.i)}; }

// Staging loop "for (e = tid; e < n; e += NT) st(e, ld(e))" with the loads of
// U consecutive iterations issued before their stores: ld(e, ok) must read a
// valid address for every e < n + NT*U (callers clamp it) and return the
// value masked by ok (keep_if).  A plain loop compiles to load -> wait ->
// LDS store per iteration, a full global-memory round trip each (the
// diagonal LU and TRSM kernels spent most of their time in such loops).
template <int NT, int U, typename T, typename LD, typename ST>
__device__ __forceinline__ void stage_loop(int tid, int n, LD ld, ST st) {
    for (int e0 = tid; e0 < n; e0 += NT * U) {
        T v[U];
#pragma unroll
        for (int u = 0; u < U; ++u) v[u] = ld(e0 + u * NT, e0 + u * NT < n);
#pragma unroll
        for (int u = 0; u < U; ++u)
            if (e0 + u * NT < n) st(e0 + u * NT, v[u]);
    }
}

__device__ inline double one_of(double) { return 1.0; }
__device__ inline float one_of(float) { return 1.0f; }
__device__ inline zc one_of(zc) { return {1.0, 0.0}; }

// Loads through the global address space.  Pointers that come out of the
// work-item structs are generic; dereferencing them emits flat_load, which
// also counts against lgkmcnt, so every s_waitcnt lgkmcnt(0) for an LDS read
// would wait for the in-flight global prefetch too.
template <typename T> __device__ __forceinline__ T gld(const T *p) {
    return *(const __attribute__((address_space(1))) T *)p;
}
template <> __device__ __forceinline__ zc gld<zc>(const zc *p) {
    typedef double d2 __attribute__((ext_vector_type(2)));
    const d2 v = *(const __attribute__((address_space(1))) d2 *)p; // one 16-byte load
    return {v.x, v.y};
}
// Four consecutive elements through 16-byte global loads from an address
// that is only element-aligned (gfx950 global loads need dword alignment).
typedef double d2u8 __attribute__((ext_vector_type(2), aligned(8)));
__device__ __forceinline__ void gld2(const double *p, double &x, double &y) {
    const d2u8 a = *(const __attribute__((address_space(1))) d2u8 *)p;
    x = a.x;
    y = a.y;
}
__device__ __forceinline__ void gld2(const float *, float &, float &) {}
__device__ __forceinline__ void gld2(const zc *, zc &, zc &) {}
__device__ __forceinline__ void gld4(const double *p, double (&r)[4]) {
    const auto *q = (const __attribute__((address_space(1))) d2u8 *)p;
    const d2u8 a = q[0], b = q[1];
    r[0] = a.x; r[1] = a.y; r[2] = b.x; r[3] = b.y;
}

// ------------------------------------------------------------ MFMA
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
    const struct DRec *prec; // nLb x nUb destinations resolved at plan time
    int lda, m, n, kmin, kw, nub, atomic, pad;
};

// One (L block ib, U block jb) destination of a panel, resolved by the plan
// from LBlk / UBlk so the Schur epilogue needs no chained table walk:
//   L(ib,jb): element (gr, gc) at Lval[base + gc*ld + lmap[mb + gr]]
//   U(ib,jb): element (gr, gc) at Uval[ucol_voff[e] - ucol_fst[e] + gr], e = base + gc
struct DRec {
    int64_t base; // L: colvoff - fcol*ld; U: coloff - fcol
    int64_t mb;   // L: mapoff - frow
    int ld;       // L: nsupr of block column jb; U: -1
    int pad;
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

// ------------------------------------------------------------- pack
// Column-major 2D copies dst[r + c*ldd] = src[r + c*lds] that stage a rank's
// own diagonal blocks and panels into the contiguous per-level sections the
// 2D-grid broadcasts send (the reference sends lusup / uval straight from
// Llu, SRC/pdgstrf.c:1039-1044,1330-1335).  Items are pre-chunked by the plan
// to <= COPY_CHUNK elements.  HBM-bound.
constexpr int COPY_CHUNK = 1 << 16;
template <typename T> struct CopyItem {
    const T *src;
    T *dst;
    int64_t lds, ldd;
    int rows, cols;
};

template <typename T>
__global__ void __launch_bounds__(256) k_copy(const CopyItem<T> *items) {
    const CopyItem<T> it = items[blockIdx.x];
    const int tot = it.rows * it.cols;
    if (it.cols == 1) {
        for (int e = threadIdx.x; e < tot; e += 256) it.dst[e] = it.src[e];
    } else {
        for (int e = threadIdx.x; e < tot; e += 256) {
            const int r = e % it.rows, c = e / it.rows;
            it.dst[r + c * it.ldd] = it.src[r + c * it.lds];
        }
    }
}

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
constexpr int SB_TB = 4; // epilogue tables: row blocks x column blocks per tile
constexpr int SB_AEB = 4; // atomic scatters formed per batch (8: slower)

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
    __shared__ T smem[2 * STAGE > CSIZE ? 2 * STAGE : CSIZE];
    __shared__ int s_rg[SC_BM], s_ra[SC_BM], s_cg[SC_BN], s_cb[SC_BN];
    if (tid < SC_BM) {
        int r = row0 + tid;
        s_rg[tid] = tid < mrows ? ki.rg[r] : 0;
        s_ra[tid] = tid < mrows ? ki.ra[r] : 0;
    } else if (tid < SC_BM + SC_BN) {
        int c = tid - SC_BM;
        s_cg[c] = c < ncols ? ki.cg[col0 + c] : 0;
        s_cb[c] = c < ncols ? ki.cb[col0 + c] : 0;
    }
    // destination tables (k_schur_big's fast path): the tile's rows lie in
    // NA consecutive L blocks of the panel, its columns in NB consecutive U
    // blocks; with NA, NB <= SB_TB every address is a column part plus a row
    // part, resolved once per tile (the records come in with the first stage)
    const int a0 = ki.ra[row0], b0 = ki.cb[col0];
    const int NA = ki.ra[row0 + mrows - 1] - a0 + 1, NB = ki.cb[col0 + ncols - 1] - b0 + 1;
    const bool tbl = NA <= SB_TB && NB <= SB_TB;
    __shared__ int64_t s_db[SB_TB * SB_TB], s_dmb[SB_TB * SB_TB];
    __shared__ int s_dld[SB_TB * SB_TB];
    __shared__ int64_t s_cp[SB_TB * SC_BN]; // [row block][column] column parts
    __shared__ int s_rl[SB_TB * SC_BM];     // [column block][row] lmap positions
    if (tbl && tid >= SC_BM + SC_BN && tid < SC_BM + SC_BN + SB_TB * SB_TB) {
        const int e = tid - SC_BM - SC_BN, al = e / SB_TB, bl = e % SB_TB;
        DRec d{0, 0, -1, 0};
        if (al < NA && bl < NB) d = ki.prec[(int64_t)(a0 + al) * ki.nub + b0 + bl];
        s_db[e] = d.base;
        s_dmb[e] = d.mb;
        s_dld[e] = d.ld;
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
    const int tlast = ki.kmin + ki.kw - 1;
    // A gather: thread owns row ar = tid & 63, k = (tid>>6) + 4*s
    const int ar = tid & 63, ak = tid >> 6;
    const bool avalid = ar < mrows;
    const T *ap = ki.a + row0 + (avalid ? ar : 0);

    typename M::acc_t acc[2][2];
#pragma unroll
    for (int a = 0; a < 2; ++a)
#pragma unroll
        for (int b = 0; b < 2; ++b) acc[a][b] = M::zero();

    // K staged SC_BK deep through two LDS buffers, the next stage's global
    // loads (clamped in-bounds addresses, masked values) in flight during the
    // current stage's MFMAs
    T ra[SC_BK / 4], rb[4];
    auto gload = [&](int k0) {
#pragma unroll
        for (int s = 0; s < SC_BK / 4; ++s) {
            const int kk = k0 + ak + 4 * s;
            ra[s] = keep_if(avalid & (kk < ki.kw), gld(ap + (int64_t)(ki.kmin + min(kk, ki.kw - 1)) * ki.lda));
        }
#pragma unroll
        for (int s = 0; s < 4; ++s) {
            const int t = ki.kmin + k0 + bk + s;
            rb[s] = keep_if(bvalid & (t <= tlast) & (t >= bt0), gld(ub + max(min(t, tlast), bt0)));
        }
    };
    auto lstore = [&](int buf) {
        T *a = smem + buf * STAGE, *b = a + SC_BK * ALD;
#pragma unroll
        for (int s = 0; s < SC_BK / 4; ++s) a[(ak + 4 * s) * ALD + ar] = ra[s];
#pragma unroll
        for (int s = 0; s < 4; ++s) b[(bk + s) * BLD + bc] = rb[s];
    };
    const int nst = (ki.kw + SC_BK - 1) / SC_BK;
    gload(0);
    __syncthreads(); // (the tables above)
    lstore(0);
    __syncthreads();
    static_assert(SB_TB * SC_BN == SC_THREADS && SB_TB * SC_BM == SC_THREADS, "one table entry per thread");
    int64_t t_code = 0, t_uv = 0;
    int t_fst = 0, t_rl = 0;
    for (int st = 0; st < nst; ++st) {
        const bool more = st + 1 < nst;
        if (more) gload((st + 1) * SC_BK);
        if (!more && tbl) { // the destination tables' loads, beside the last stage's MFMAs
            {
                const int al = tid / SC_BN, c = tid % SC_BN;
                if (al < NA && c < ncols) {
                    const int bl = s_cb[c] - b0, rec = al * SB_TB + bl, ld = s_dld[rec];
                    if (ld >= 0) {
                        t_code = (s_db[rec] + (int64_t)s_cg[c] * ld) * 8 + 1 + bl;
                    } else {
                        const int64_t x = s_db[rec] + s_cg[c];
                        t_uv = ucol_voff[x];
                        t_fst = ucol_fst[x];
                    }
                }
            }
            {
                const int bl = tid / SC_BM, rr = tid % SC_BM;
                if (bl < NB && rr < mrows) {
                    const int rec = (s_ra[rr] - a0) * SB_TB + bl;
                    if (s_dld[rec] >= 0) t_rl = lmap[s_dmb[rec] + s_rg[rr]];
                }
            }
        }
        const T *a = smem + (st & 1) * STAGE, *b = a + SC_BK * ALD;
#pragma unroll
        for (int ks = 0; ks < SC_BK; ks += M::KSTEP) {
            const int kl = ks + (lane >> 4);
            T a0 = a[kl * ALD + wr * 32 + (lane & 15)];
            T a1 = a[kl * ALD + wr * 32 + 16 + (lane & 15)];
            T b0 = b[kl * BLD + wc * 32 + (lane & 15)];
            T b1 = b[kl * BLD + wc * 32 + 16 + (lane & 15)];
            M::step(acc[0][0], a0, b0);
            M::step(acc[0][1], a0, b1);
            M::step(acc[1][0], a1, b0);
            M::step(acc[1][1], a1, b1);
        }
        if (more) lstore((st + 1) & 1);
        __syncthreads();
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
    if (tbl) {
        s_cp[tid] = t_code ? t_code : (t_uv - t_fst) * 8;
        s_rl[tid] = t_rl;
    }
    __syncthreads();
    const int r = tid & 63;
    if (r >= mrows) return;
    const int gr = s_rg[r], a = s_ra[r];
    if (tbl) { // one LDS word per element besides the destination (k_schur_big)
        int rl[SB_TB];
#pragma unroll
        for (int bl = 0; bl < SB_TB; ++bl) rl[bl] = s_rl[bl * SC_BM + r];
        const int al = a - a0;
        for (int c0 = tid >> 6; c0 < ncols; c0 += 4 * SB_AEB) {
            T *dp[SB_AEB];
            T v[SB_AEB];
#pragma unroll
            for (int j = 0; j < SB_AEB; ++j) {
                const int c = c0 + 4 * j;
                dp[j] = nullptr;
                v[j] = Sx::zero();
                if (c < ncols) {
                    v[j] = sC[c * CLD + r];
                    const int64_t code = s_cp[al * SC_BN + c];
                    const int tag = (int)(code & 7);
                    int rp = gr;
                    rp = tag == 1 ? rl[0] : rp;
                    rp = tag == 2 ? rl[1] : rp;
                    rp = tag == 3 ? rl[2] : rp;
                    rp = tag == 4 ? rl[3] : rp;
                    dp[j] = (tag ? Lval : Uval) + ((code >> 3) + rp);
                }
            }
#pragma unroll
            for (int j = 0; j < SB_AEB; ++j)
                if (dp[j]) {
                    if (ki.atomic) Sx::atomic_sub(dp[j], v[j]);
                    else Sx::sub_to(dp[j], v[j]);
                }
        }
        return;
    }
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


// ===================================================================== fast
// panel path (supernodes of width <= 256): blocked, MFMA-based.
//
// PW = panel width = size of the inverted diagonal blocks (Dinv).
template <typename T> struct PWOf { static constexpr int v = 32; };
template <> struct PWOf<zc> { static constexpr int v = 16; };
constexpr int FAST_MAXW = 256;

template <typename T> struct DiagItemF {
    T *a;     // diagonal block, ld
    T *dinv;  // out: [nb][PW][PW] U11^{-1} blocks, then [nb][PW][PW] (L11^{-1})^T blocks
    int ld, w, k, fcol;
};

// Wave-uniform read of lane l's value (v_readlane; l must be uniform).
__device__ inline double rlane(double v, int l) {
    const long long x = __double_as_longlong(v);
    const int lo = __builtin_amdgcn_readlane((int)x, l);
    const int hi = __builtin_amdgcn_readlane((int)(x >> 32), l);
    return __longlong_as_double(((long long)hi << 32) | (unsigned)lo);
}
__device__ inline float rlane(float v, int l) {
    return __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), l));
}
__device__ inline zc rlane(zc v, int l) { return {rlane(v.r, l), rlane(v.i, l)}; }

// Blocked right-looking LU of one <= 256 x 256 diagonal block per 512-thread
// workgroup, built for latency (the top-of-tree levels hold one supernode
// each, so this kernel sits on the critical path).  Per panel of PW columns:
//   0. the panel (rows p0.., PW columns) and the U12 row block (PW rows,
//      columns right of the panel) are staged into LDS, coalesced;
//   1. waves 0 and 1 both factor the PW x PW block A11 in registers (lane =
//      row, the pivot row read with v_readlane: no LDS, no barrier per
//      column; SRC/pdgstrf2.c:213-269 semantics: tiny-pivot replacement,
//      reciprocal scaling, a zero pivot sets info and leaves its column
//      unscaled), then wave 0 forms U11^{-1} and wave 1 L11^{-1} (lane =
//      column), written to LDS and to dinv for the MFMA TRSMs;
//   2. L21 = A21 U11^{-1} and U12 = L11^{-1} A12 on MFMA (a panel with a zero
//      pivot takes the substitution path instead, to keep the unscaled-column
//      semantics);
//   3. the panel and U12 go back to global memory and A22 -= L21 U12 runs on
//      MFMA with both operands in LDS, the next batch's loads in flight.
constexpr int DF_THREADS = 512;
#ifdef SLU_DIAG_PROBE
// Diagnostics build only (tools/micro/diag_micro.hip): cycles per phase of
// k_diag_lu_f summed over panels and blocks (thread 0's view).
__device__ long long slu_diag_tp[8];
#define DF_PROBE_START() long long df_t0 = clock64()
#define DF_PROBE(i)                                                                          \
    do {                                                                                     \
        if (threadIdx.x == 0) {                                                              \
            const long long t = clock64();                                                   \
            atomicAdd((unsigned long long *)&slu_diag_tp[i], (unsigned long long)(t - df_t0)); \
            df_t0 = t;                                                                       \
        }                                                                                    \
    } while (0)
#else
#define DF_PROBE_START()
#define DF_PROBE(i)
#endif
// MAXW / NTHR: the widest block a launch holds and its workgroup size.  The
// levels near the leaves hold thousands of narrow (relaxed) supernodes: a
// <= 64-wide variant on 256 threads takes 50 KB of LDS instead of 150 KB,
// so three workgroups share a CU instead of one.
constexpr int DF_SMALLW = 64, DF_SMALL_THREADS = 256;
template <typename T, int MAXW = FAST_MAXW, int NTHR = DF_THREADS>
__global__ void __launch_bounds__(NTHR, NTHR == DF_SMALL_THREADS ? 2 : 1)
k_diag_lu_f(const DiagItemF<T> *items, double thresh, int replace_tiny, int *tiny_count,
            int *zpiv) {
    constexpr int DF_THREADS = NTHR; // (shadows the default for the loops below)
    constexpr int FAST_MAXW = MAXW;
    constexpr int PW = PWOf<T>::v;
    constexpr int NW = DF_THREADS / 64;
    static_assert(NW >= 2 && MAXW >= PW, "waves 0 and 1 form the inverses");
    using Sx = S<T>;
    using M = Mma<T>;
    const DiagItemF<T> it = items[blockIdx.x];
    T *A = it.a;
    const int ld = it.ld, w = it.w, tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
    const int nb = (w + PW - 1) / PW;
    T *dinvU = it.dinv, *dinvLT = it.dinv + (int64_t)nb * PW * PW;
    __shared__ T sP[FAST_MAXW][PW + 1];   // panel rows (row 0 = row p0), PW columns
    __shared__ T sU[PW][FAST_MAXW + 1];   // U12: PW rows x columns right of the panel
    __shared__ T sUi[PW][PW + 1], sLi[PW][PW + 1]; // U11^{-1}, L11^{-1}
    __shared__ T s_rp[PW];
    __shared__ int s_z[PW];
    __shared__ int s_anyz;
    DF_PROBE_START();
    for (int p = 0; p < nb; ++p) {
        const int p0 = p * PW, pw = min(PW, w - p0), nrow = w - p0, nbl = nrow - pw;
        const int c0 = p0 + pw;
        T *A11 = A + p0 + (int64_t)p0 * ld;

        // ---- 0. stage the panel and U12 (zero outside pw; a last panel with
        // nrow < PW zero-fills rows nrow..PW-1, which the inverse sweeps in
        // 1b multiply by zero: stale LDS there could be NaN, and 0 * NaN
        // would reach the stored U11^{-1})
        const int nrs = max(nrow, PW);
        stage_loop<DF_THREADS, 4, T>(
            tid, nrs * PW,
            [&](int e, bool ok) {
                const int r = e % nrs, c = min(e / nrs, PW - 1);
                return keep_if(ok & (c < pw) & (r < nrow),
                               gld(A11 + min(r, nrow - 1) + (int64_t)min(c, pw - 1) * ld));
            },
            [&](int e, T v) { sP[e % nrs][e / nrs] = v; });
        if (nbl > 0)
            stage_loop<DF_THREADS, 4, T>(
                tid, nbl * PW,
                [&](int e, bool ok) {
                    const int i = e % PW, c = min(e / PW, nbl - 1);
                    return keep_if(ok & (i < pw), gld(A11 + min(i, pw - 1) + (int64_t)(pw + c) * ld));
                },
                [&](int e, T v) { sU[e % PW][e / PW] = v; });
        __syncthreads();
        DF_PROBE(0);
        // ---- 1. A11 = L11 U11 in registers (wave 0); meanwhile, on the first
        // panel, the other waves pull the trailing block into L2 (every
        // panel's update re-reads it)
        if (p == 0 && wid >= 1 && nbl > 0) {
            T sink = Sx::zero();
            for (int e = tid - 64; e < nbl * nbl; e += DF_THREADS - 64)
                sink = Sx::sub(sink, A11[pw + e % nbl + (int64_t)(pw + e / nbl) * ld]);
            if (Sx::abs1(sink) == -1.0) s_anyz = 0; // keeps the loads; never true
        }
        if (wid == 0) {
            const int row = lane & (PW - 1);
            T xr[PW];
#pragma unroll
            for (int c = 0; c < PW; ++c) xr[c] = (row < pw) ? sP[row][c] : Sx::zero();
            int anyz = 0;
#pragma unroll
            for (int j = 0; j < PW; ++j) {
                if (j < pw) { // uniform
                    T piv = rlane(xr[j], j);
                    if (replace_tiny && Sx::abs1(piv) < thresh) {
                        piv = Sx::thresh(piv, thresh);
                        if (lane == 0) atomicAdd(tiny_count, 1);
                    }
                    const int z = Sx::iszero(piv);
                    if (z) {
                        anyz = 1;
                        if (lane == 0) atomicMax(&zpiv[it.k], it.fcol + p0 + j + 1);
                    }
                    const T rp = z ? Sx::zero() : Sx::recip(piv);
                    // branch-free: rows below j eliminate, row j keeps the pivot
                    const bool below = row > j;
                    const T l = below ? (z ? xr[j] : Sx::mul(xr[j], rp)) : Sx::zero();
                    xr[j] = below ? l : (row == j ? piv : xr[j]);
                    __builtin_amdgcn_sched_barrier(0); // keep the readlanes next to their FMAs
#pragma unroll
                    for (int c = j + 1; c < PW; ++c) {
                        xr[c] = Sx::fms(xr[c], l, rlane(xr[c], j));
                        if ((c & 3) == 3) __builtin_amdgcn_sched_barrier(0);
                    }
                    __builtin_amdgcn_sched_barrier(0);
                    if (lane == 0) {
                        s_rp[j] = rp;
                        s_z[j] = z;
                    }
                }
            }
            if (lane < pw) {
#pragma unroll
                for (int c = 0; c < PW; ++c) sP[lane][c] = xr[c];
            }
            if (lane == 0) s_anyz = anyz;
            if (lane >= pw && lane < PW) {
                s_rp[lane] = Sx::zero();
                s_z[lane] = 0;
            }
        }
        __syncthreads();
        DF_PROBE(1);
        // ---- 1b. inverses from the factored A11 in LDS, lane = column j
        // (wave 0 U11^{-1}, wave 1 L11^{-1}), column-sweep (axpy) order so the
        // dependent chain is one multiply per row
        if (wid < 2 && lane < PW) {
            const int j = lane;
            T x[PW];
#pragma unroll
            for (int i = 0; i < PW; ++i) x[i] = (i == j) ? one_of(Sx::zero()) : Sx::zero();
            if (wid == 0) { // U11 x = e_j
#pragma unroll
                for (int i = PW - 1; i >= 0; --i) {
                    x[i] = Sx::mul(x[i], s_rp[i]);
#pragma unroll
                    for (int k = 0; k < i; ++k) x[k] = Sx::fms(x[k], sP[k][i], x[i]);
                }
#pragma unroll
                for (int i = 0; i < PW; ++i) sUi[i][j] = (i <= j && j < pw) ? x[i] : Sx::zero();
            } else { // L11 x = e_j (unit lower)
#pragma unroll
                for (int i = 0; i < PW; ++i)
#pragma unroll
                    for (int k = i + 1; k < PW; ++k) x[k] = Sx::fms(x[k], sP[k][i], x[i]);
#pragma unroll
                for (int i = 0; i < PW; ++i) sLi[i][j] = (i >= j && i < pw && j < pw) ? x[i] : Sx::zero();
            }
        }
        __syncthreads();
        DF_PROBE(2);
        // ---- 2. L21 = A21 U11^{-1}, U12 = L11^{-1} A12
        if (!s_anyz) {
            const int nfr = (nbl + 15) / 16; // L21 row fragments; U12 column fragments
            for (int f = wid; f < 2 * nfr; f += NW) {
                typename M::acc_t acc0 = M::zero(), acc1 = M::zero();
                if (f < nfr) { // rows 16f.. of L21, both 16-column halves
                    const int r = f * 16 + (lane & 15);
#pragma unroll
                    for (int ks = 0; ks < PW; ks += M::KSTEP) {
                        const int k = ks + (lane >> 4);
                        const T av = r < nbl ? sP[pw + r][k] : Sx::zero();
                        M::step(acc0, av, sUi[k][lane & 15]);
                        if (PW > 16) M::step(acc1, av, sUi[k][16 + (lane & 15)]);
                    }
#pragma unroll
                    for (int i = 0; i < 4; ++i) {
                        const int rr = f * 16 + M::row(lane, i), cc = lane & 15;
                        if (rr < nbl) {
                            sP[pw + rr][cc] = cc < pw ? M::get(acc0, i) : Sx::zero();
                            if (PW > 16)
                                sP[pw + rr][16 + cc] = 16 + cc < pw ? M::get(acc1, i) : Sx::zero();
                        }
                    }
                } else { // columns 16g.. of U12, both 16-row halves
                    const int g = f - nfr, c = g * 16 + (lane & 15);
#pragma unroll
                    for (int ks = 0; ks < PW; ks += M::KSTEP) {
                        const int k = ks + (lane >> 4);
                        const T bv = c < nbl ? sU[k][c] : Sx::zero();
                        M::step(acc0, sLi[lane & 15][k], bv);
                        if (PW > 16) M::step(acc1, sLi[16 + (lane & 15)][k], bv);
                    }
                    // all waves have read their U12 columns before any is overwritten
                    // (each fragment's columns belong to this wave only)
#pragma unroll
                    for (int i = 0; i < 4; ++i) {
                        const int ii = M::row(lane, i), cc = g * 16 + (lane & 15);
                        if (cc < nbl) {
                            sU[ii][cc] = ii < pw ? M::get(acc0, i) : Sx::zero();
                            if (PW > 16) sU[16 + ii][cc] = 16 + ii < pw ? M::get(acc1, i) : Sx::zero();
                        }
                    }
                }
            }
        } else {
            for (int t = tid; t < 2 * nbl; t += DF_THREADS) {
                if (t < nbl) { // row t of L21: x U11 = a, column by column
                    for (int c = 0; c < PW; ++c) {
                        T v = sP[pw + t][c];
                        for (int i = 0; i < c; ++i) v = Sx::fms(v, sP[pw + t][i], sP[i][c]);
                        sP[pw + t][c] = c >= pw ? Sx::zero() : s_z[c] ? v : Sx::mul(v, s_rp[c]);
                    }
                } else { // column cc of U12: L11 y = a
                    const int cc = t - nbl;
                    for (int i = 0; i < PW; ++i) {
                        T v = sU[i][cc];
                        for (int k = 0; k < i; ++k) v = Sx::fms(v, sP[i][k], sU[k][cc]);
                        sU[i][cc] = i < pw ? v : Sx::zero();
                    }
                }
            }
        }
        __syncthreads();
        DF_PROBE(3);
        // ---- 3. panel, U12 and the dinv blocks back to global (written here
        // so that no barrier before the trailing update waits for them);
        // A22 -= L21 U12 on MFMA
        for (int e = tid; e < PW * PW; e += DF_THREADS) {
            const int i = e / PW, jj = e % PW;
            dinvU[(int64_t)p * PW * PW + e] = sUi[i][jj];  // row-major U11^{-1}
            dinvLT[(int64_t)p * PW * PW + e] = sLi[jj][i]; // row-major (L11^{-1})^T
        }
        for (int e = tid; e < nrow * pw; e += DF_THREADS) {
            const int r = e % nrow, c = e / nrow;
            A11[r + (int64_t)c * ld] = sP[r][c];
        }
        for (int e = tid; e < nbl * pw; e += DF_THREADS) {
            const int i = e % pw, c = e / pw;
            A11[i + (int64_t)(pw + c) * ld] = sU[i][c];
        }
        if (nbl > 0) {
            // wave wid takes fragment batches f0 = (wid + NW i) FB; the next
            // batch's C loads are issued before this batch's MFMAs
            const int nf = (nbl + 15) / 16, nff = nf * nf;
            T *A22 = A + c0 + (int64_t)c0 * ld;
            constexpr int FB = sizeof(T) == 16 ? 2 : 4; // complex: fewer live accumulators
            T cv[FB][4], cn[FB][4];
            auto cload = [&](T (&dst)[FB][4], int f0) {
#pragma unroll
                for (int q = 0; q < FB; ++q) {
                    const int f = f0 + q, fr = f % nf, fc = f / nf;
#pragma unroll
                    for (int i = 0; i < 4; ++i) {
                        // transposed fragment (operands swapped below): lane
                        // l&15 holds row fr*16 + (l&15) -- 16 consecutive rows
                        // of 4 columns per load, 4 cache lines instead of 16
                        const int r = fr * 16 + (lane & 15), c = fc * 16 + M::row(lane, i);
                        // unconditional load from a clamped address + branch-free
                        // mask: the next batch's loads stay ahead of the MFMAs
                        const bool ok = (f < nff) & (r < nbl) & (c < nbl);
                        dst[q][i] = keep_if(ok, A22[min(r, nbl - 1) + (int64_t)min(c, nbl - 1) * ld]);
                    }
                }
            };
            int f0 = wid * FB;
            if (f0 < nff) cload(cv, f0);
            for (; f0 < nff; f0 += NW * FB) {
                const int f1 = f0 + NW * FB;
                if (f1 < nff) cload(cn, f1);
                // the FB fragments' accumulation chains interleaved (one
                // dependent MFMA chain per fragment would wait out the MFMA
                // and LDS latencies at every k step)
                typename M::acc_t acc[FB];
#pragma unroll
                for (int q = 0; q < FB; ++q) acc[q] = M::zero();
#pragma unroll
                for (int ks = 0; ks < PW; ks += M::KSTEP) {
                    const int k = ks + (lane >> 4);
                    T av[FB], bv[FB];
#pragma unroll
                    for (int q = 0; q < FB; ++q) {
                        const int f = f0 + q, fr = f % nf, fc = f / nf;
                        const int r = fr * 16 + (lane & 15), c = fc * 16 + (lane & 15);
                        av[q] = keep_if(r < nbl, sP[pw + min(r, nbl - 1)][k]);
                        bv[q] = keep_if(c < nbl, sU[k][min(c, nbl - 1)]);
                    }
#pragma unroll
                    for (int q = 0; q < FB; ++q) M::step(acc[q], bv[q], av[q]); // C^T = U12^T L21^T
                }
#pragma unroll
                for (int q = 0; q < FB; ++q) {
                    const int f = f0 + q, fr = f % nf, fc = f / nf;
#pragma unroll
                    for (int i = 0; i < 4; ++i) {
                        const int rr = fr * 16 + (lane & 15), cc = fc * 16 + M::row(lane, i);
                        if (f < nff && rr < nbl && cc < nbl)
                            A22[rr + (int64_t)cc * ld] =
                                Sx::fms(cv[q][i], M::get(acc[q], i), one_of(cv[q][i]));
                    }
                }
#pragma unroll
                for (int q = 0; q < FB; ++q)
#pragma unroll
                    for (int i = 0; i < 4; ++i) cv[q][i] = cn[q][i];
            }
        }
        __syncthreads();
        DF_PROBE(4);
    }
}

template <typename T> struct TrsmItemF {
    T *x;                // MODE 0: first row, column-major ld ldx; MODE 1: U value base
    const int64_t *voff; // MODE 1: per row (U column) segment offset
    const int *t0;       // MODE 1: per row first row of the segment (rel. to xsup[k])
    const T *t;          // diagonal block, ld ldt
    const T *dinv;       // [nb][PW][PW] (MODE 0: U^{-1} blocks; MODE 1: (L^{-1})^T blocks)
    int ldx, ldt, nrows, w;
};
template <typename T> struct RBOf { static constexpr int v = 32; };
template <> struct RBOf<zc> { static constexpr int v = 16; };

template <typename T, int MODE>
__global__ void __launch_bounds__(256)
k_trsm_blk(const TrsmItemF<T> *items) {
    constexpr int PW = PWOf<T>::v, RB = RBOf<T>::v;
    constexpr int NFC = PW / 16, NFR = RB / 16, NFRAG = NFC * NFR;
    using Sx = S<T>;
    using M = Mma<T>;
    const TrsmItemF<T> it = items[blockIdx.x];
    const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
    const int w = it.w, nb = (w + PW - 1) / PW, NBW = nb * PW;
    __shared__ T sX[RB][FAST_MAXW + 1];
    __shared__ T sT[FAST_MAXW][PW + 1]; // T[0 : b*PW, b-block]
    __shared__ T sD[PW][PW + 1];
    __shared__ T sZ[RB][PW + 1];
    // ---- load the RB rows
    if (MODE == 0) {
        for (int e = tid; e < RB * NBW; e += 256) {
            int r = e % RB, c = e / RB;
            sX[r][c] = (r < it.nrows && c < w) ? it.x[r + (int64_t)c * it.ldx] : Sx::zero();
        }
    } else {
        for (int e = tid; e < RB * NBW; e += 256) {
            int r = e / NBW, c = e % NBW;
            T v = Sx::zero();
            if (r < it.nrows && c < w) {
                int t0 = it.t0[r];
                if (c >= t0) v = it.x[it.voff[r] + c - t0];
            }
            sX[r][c] = v;
        }
    }
    const int fr = (wid % NFRAG) / NFC, fc = (wid % NFRAG) % NFC;
    const bool mfma_wave = wid < NFRAG;
    for (int b = 0; b < nb; ++b) {
        // stage Dinv_b and the whole column block T[0:b*PW, b*PW:(b+1)*PW]
        for (int e = tid; e < PW * PW; e += 256) {
            int i = e / PW, j = e % PW;
            sD[i][j] = it.dinv[(int64_t)b * PW * PW + e];
        }
        const int kr = b * PW;
        for (int e = tid; e < kr * PW; e += 256) {
            int i, j;
            T v;
            if (MODE == 0) {
                i = e % kr; j = e / kr;
                v = (b * PW + j < w) ? it.t[i + (int64_t)(b * PW + j) * it.ldt] : Sx::zero();
            } else {
                j = e % PW; i = e / PW;
                v = (b * PW + j < w) ? it.t[(b * PW + j) + (int64_t)i * it.ldt] : Sx::zero();
            }
            sT[i][j] = v;
        }
        __syncthreads();
        typename M::acc_t acc = M::zero();
        if (mfma_wave) {
            for (int k0 = 0; k0 < kr; k0 += 4) {
                T av = sX[fr * 16 + (lane & 15)][k0 + (lane >> 4)];
                T bv = sT[k0 + (lane >> 4)][fc * 16 + (lane & 15)];
                M::step(acc, av, bv);
            }
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                const int r = fr * 16 + M::row(lane, i), c = fc * 16 + (lane & 15);
                T v = sX[r][b * PW + c];
                T a = M::get(acc, i);
                sZ[r][c] = Sx::fms(v, a, one_of(a));
            }
        }
        __syncthreads();
        if (mfma_wave) {
            typename M::acc_t acc2 = M::zero();
#pragma unroll
            for (int ks = 0; ks < PW; ks += 4) {
                T av = sZ[fr * 16 + (lane & 15)][ks + (lane >> 4)];
                T bv = sD[ks + (lane >> 4)][fc * 16 + (lane & 15)];
                M::step(acc2, av, bv);
            }
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                const int r = fr * 16 + M::row(lane, i), c = fc * 16 + (lane & 15);
                sX[r][b * PW + c] = M::get(acc2, i);
            }
        }
        __syncthreads();
    }
    // ---- store
    if (MODE == 0) {
        for (int e = tid; e < RB * w; e += 256) {
            int r = e % RB, c = e / RB;
            if (r < it.nrows) it.x[r + (int64_t)c * it.ldx] = sX[r][c];
        }
    } else {
        for (int e = tid; e < RB * NBW; e += 256) {
            int r = e / NBW, c = e % NBW;
            if (r < it.nrows && c < w) {
                int t0 = it.t0[r];
                if (c >= t0) it.x[it.voff[r] + c - t0] = sX[r][c];
            }
        }
    }
}


// ------------------------------------------------------------- Schur (big)
// 128x128 output tile per 512-thread workgroup: 4x2 waves, each 32x64 = 2x4
// v_mfma_f64_16x16x4 fragments (64 accumulator VGPRs, so 4 waves per SIMD fit
// beside the 2 workgroups per CU the 66 KB of LDS allow -- measured: more
// resident waves, not more ILP per wave, is what feeds the fp64 MFMA pipe,
// tools/micro/gemm_exp.hip).  K is staged 16 deep through double-buffered LDS
// with the next stage's global loads in flight during the current stage's
// MFMAs.  Epilogue: the C tile goes through LDS in two 64-column passes and
// is scatter-subtracted column-contiguously into the destination blocks
// (dscatter_l / dscatter_u, SRC/dscatter.c:175-187,240-272).
//
// Complex (pzgstrf): 128x64 tiles, each wave 32x32 = 2x2 fragments of four
// real MFMAs each (Mma<zc>), K staged 8 deep -- the same accumulator VGPRs,
// MFMAs per stage and LDS per workgroup as the real tile, at twice the
// MFMAs per LDS operand; the epilogue stages 16 columns per pass.
constexpr int SB_BM = 128;
// Elements allocated on either side of the U value and panel buffers
// (DevBuf::alloc_guarded; the L values too): k_schur_big's B loads read a
// column's 4 consecutive k without clamping them to its segment (the mask
// drops what lies outside), i.e. up to the panel width before a segment and
// 15 past it; the A loads read up to 127 rows past a column.
constexpr size_t SB_UGUARD = 1024;
// THREADS / WN: workgroup size and waves along N; MINW: waves per SIMD the
// register budget must allow (workgroups per CU x waves per workgroup / 4).
template <typename T> struct BigCfg {
    static constexpr int THREADS = 512, WN = 2, MINW = 4, BN = 128, BK = 16, FN = 4, PASSW = 64;
};
template <> struct BigCfg<zc> {
    static constexpr int THREADS = 512, WN = 2, MINW = 4, BN = 64, BK = 8, FN = 2, PASSW = 16;
};
// fp32: three workgroups per CU (6 waves per SIMD, <= 80 VGPRs; 42 KB LDS each)
// (SLU_F32_BK / SLU_F32_MINW: A/B builds, tools/ab_build.sh)
#ifndef SLU_F32_BK
#define SLU_F32_BK 16
#endif
#ifndef SLU_F32_MINW
#define SLU_F32_MINW 6
#endif
template <> struct BigCfg<float> {
    static constexpr int THREADS = 512, WN = 2, MINW = SLU_F32_MINW, BN = 128, BK = SLU_F32_BK, FN = 4, PASSW = 64;
};
constexpr int SB_BN = BigCfg<double>::BN;
constexpr int SB_THREADS = 512; // the 512-thread configurations (k_schur_big<float>, <zc>)

#ifdef SLU_SB_STAMP
// Diagnostics build only (tools/ab_build.sh NAME "-DSLU_SB_STAMP"): per-tile
// phase timestamps of k_schur_big, read back by the engine after a factor()
// (SLU_STAMP_OUT) and summarised by tools/stamp_analyze.py.  Four u64 per
// tile: realtime start (40 b) + duration (24 b, 100 MHz) | prologue, K-loop
// cycles | epilogue cycles, HW_ID | XCC_ID, tile shape, workgroup id.
constexpr unsigned SLU_STAMP_MAX = 1u << 21;
__device__ uint64_t slu_stamp[SLU_STAMP_MAX * 4];
__device__ unsigned slu_stamp_n;
#define SB_STAMP(v) if (threadIdx.x == 0) s_stamp_[v] = __builtin_readcyclecounter()
#else
#define SB_STAMP(v)
#endif

// 2 workgroups (16 waves) per CU need <= 128 VGPRs: ask for 4 waves per SIMD
template <typename T>
__global__ void __launch_bounds__(BigCfg<T>::THREADS, BigCfg<T>::MINW)
k_schur_big(const TileItem *tiles, const KInfo<T> *kinfo, T *Lval, T *Uval,
            const LBlk *lblk, const int *lmap, const UBlk *ublk,
            const int64_t *ucol_voff, const int *ucol_fst) {
    using Sx = S<T>;
    using M = Mma<T>;
    constexpr int SB_BN = BigCfg<T>::BN, SB_BK = BigCfg<T>::BK;
    constexpr int SB_THREADS = BigCfg<T>::THREADS;
    constexpr int WN = BigCfg<T>::WN;       // waves along N
    constexpr int FM = 2, FN = BigCfg<T>::FN; // fragments per wave (32 x 16*FN)
    constexpr int PASSW = BigCfg<T>::PASSW; // epilogue columns per pass
    constexpr int LDS_A = SB_BM + 4, LDS_B = SB_BN + 4; // padded stages
    constexpr int STAGE = SB_BK * LDS_A + SB_BK * LDS_B;
    constexpr int CLD = SB_BM + 1; // C staging: [PASSW cols][CLD]
    constexpr int AE = SB_BM * SB_BK / SB_THREADS, BE = SB_BN * SB_BK / SB_THREADS;
    static_assert(WN * 16 * FN == SB_BN && AE >= 1 && BE >= 1, "tile shape");
    static_assert((SB_THREADS / 64 / WN) * 16 * FM == SB_BM, "waves along M");
    constexpr int CPN = SB_TB * SB_BN, RLN = SB_TB * SB_BM;
    static_assert(CPN <= SB_THREADS && RLN % SB_THREADS == 0, "table entries per thread");
    // the epilogue tables go in the stage buffers' tail past the C staging
    // where it is large enough, else in arrays of their own
    // one LDS buffer: the two stages, then (epilogue) the C staging and,
    // where it leaves room for them, the destination tables
    constexpr int SMEM = 2 * STAGE;
    static_assert(PASSW * CLD <= SMEM, "C staging must fit in the stage buffers");
    constexpr bool TAIL = (SMEM - PASSW * CLD) * (int)sizeof(T) >= CPN * 8 + RLN * 4;
    __shared__ __attribute__((aligned(16))) T smem[SMEM];
    __shared__ int s_rg[SB_BM], s_ra[SB_BM], s_cg[SB_BN], s_cb[SB_BN];
    __shared__ int64_t s_db[SB_TB * SB_TB], s_dmb[SB_TB * SB_TB]; // destination records
    __shared__ int s_dld[SB_TB * SB_TB];                          // ld (L) or -1 (U)
    __shared__ int64_t s_cpx[TAIL ? 1 : CPN];                     // [row block][column] column parts
    __shared__ int s_rlx[TAIL ? 1 : RLN];                         // [column block][row] lmap positions
    int64_t *const s_cp = TAIL ? (int64_t *)(smem + PASSW * CLD) : s_cpx;
    int *const s_rl = TAIL ? (int *)(s_cp + CPN) : s_rlx;

#ifdef SLU_SB_STAMP
    __shared__ uint64_t s_stamp_[5]; // in LDS: the stamps must not add VGPRs (occupancy)
    enum { c0_, c1_, c2_, c3_, rt_ };
    if (threadIdx.x == 0) s_stamp_[rt_] = wall_clock64();
#endif
    SB_STAMP(c0_);
    const TileItem ti = tiles[blockIdx.x];
    const KInfo<T> ki = kinfo[ti.kslot];
    const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
    const int wr = wid / WN, wc = wid % WN;
    const int row0 = ti.tm * SB_BM, col0 = ti.tn * SB_BN;
    const int mrows = min(SB_BM, ki.m - row0), ncols = min(SB_BN, ki.n - col0);
    // destination tables (epilogue fast path, below): the tile's rows lie in
    // NA consecutive L blocks of the panel, its columns in NB consecutive U
    // blocks; their NA x NB destination records come in with the first stage
    const int a0 = ki.ra[row0], b0 = ki.cb[col0];
    const int NA = ki.ra[row0 + mrows - 1] - a0 + 1, NB = ki.cb[col0 + ncols - 1] - b0 + 1;
    const bool tbl = NA <= SB_TB && NB <= SB_TB;
    if (tbl && tid < SB_TB * SB_TB) {
        const int al = tid / SB_TB, bl = tid % SB_TB;
        DRec d{0, 0, -1, 0};
        if (al < NA && bl < NB) d = ki.prec[(int64_t)(a0 + al) * ki.nub + b0 + bl];
        s_db[tid] = d.base;
        s_dmb[tid] = d.mb;
        s_dld[tid] = d.ld;
    }
    if (tid < SB_BM) {
        s_rg[tid] = tid < mrows ? ki.rg[row0 + tid] : 0;
        s_ra[tid] = tid < mrows ? ki.ra[row0 + tid] : 0;
    } else if (tid < SB_BM + SB_BN) {
        const int c = tid - SB_BM;
        s_cg[c] = c < ncols ? ki.cg[col0 + c] : 0;
        s_cb[c] = c < ncols ? ki.cb[col0 + c] : 0;
    }
    // A: thread owns row ar and k = ak + 4s (s < 4); B: column bc, k = bk..bk+3.
    // Loads are unconditional from clamped in-bounds addresses; out-of-range
    // elements are zeroed afterwards (no per-element branches).
    // fp64: thread owns rows ar, ar + 1 and k = ak + 8s (s < 2): one 16-byte
    // load per k along the column, unclamped rows (guarded L / panel
    // buffers), one 16-byte LDS store (312.4 -> 307.1 ms at 100^3, Schur
    // 56.1 -> 57.3 %, profiles/r03x_ab)
    constexpr bool A16 = AE == 4 && std::is_same<T, double>::value;
    const int ar = A16 ? 2 * (tid & 63) : tid & (SB_BM - 1), ak = A16 ? tid >> 6 : tid / SB_BM;
    const bool avalid = ar < mrows;
    const T *ap = ki.a + row0 + (A16 || avalid ? ar : 0);
    const int bc = tid / (SB_BK / BE), bk = (tid % (SB_BK / BE)) * BE;
    const bool bvalid = bc < ncols;
    const int bcc = col0 + (bvalid ? bc : 0);
    const int bt0 = ki.ct0[bcc];
    const T *ub = ki.ubase + ki.cvoff[bcc] - bt0; // ub[t] valid for bt0 <= t < kmin + kw
    const int tlast = ki.kmin + ki.kw - 1;
    // The zeroing of out-of-range elements happens at the LDS store, after
    // the current stage's MFMAs, so the prefetch's latency is not waited on
    // before them.
    T ra[AE], rb[BE];
    auto gload = [&](int k0) {
        if constexpr (A16) {
#pragma unroll
            for (int s = 0; s < 2; ++s) {
                const int kk = k0 + ak + 8 * s;
                gld2(ap + (int64_t)(ki.kmin + min(kk, ki.kw - 1)) * ki.lda, ra[2 * s], ra[2 * s + 1]);
            }
        } else
#pragma unroll
        for (int s = 0; s < AE; ++s) {
            const int kk = k0 + ak + (SB_THREADS / SB_BM) * s;
            ra[s] = gld(ap + (int64_t)(ki.kmin + min(kk, ki.kw - 1)) * ki.lda);
        }
        // a column's 4 consecutive k through 16-byte loads, unclamped (the
        // buffers carry SB_UGUARD guards; 315.2 -> 310.7 ms at 100^3, Schur
        // 56.3 -> 57.0 %, and no spilled VGPRs, profiles/r03w_ab)
        if constexpr (BE == 4 && std::is_same<T, double>::value) { // (fp32: more spills)
            gld4(ub + ki.kmin + k0 + bk, rb);
            return;
        }
#pragma unroll
        for (int s = 0; s < BE; ++s) {
            const int t = ki.kmin + k0 + bk + s;
            rb[s] = gld(ub + max(min(t, tlast), bt0));
        }
    };
    auto lstore = [&](int buf, int k0) {
        T *sA = smem + buf * STAGE, *sB = sA + SB_BK * LDS_A;
        if constexpr (A16) {
#pragma unroll
            for (int s = 0; s < 2; ++s) {
                const bool okk = k0 + ak + 8 * s < ki.kw;
                typedef double d2 __attribute__((ext_vector_type(2)));
                *(d2 *)&sA[(ak + 8 * s) * LDS_A + ar] =
                    d2{keep_if(okk & (ar < mrows), ra[2 * s]), keep_if(okk & (ar + 1 < mrows), ra[2 * s + 1])};
            }
        } else
#pragma unroll
        for (int s = 0; s < AE; ++s) {
            const int kk = k0 + ak + (SB_THREADS / SB_BM) * s;
            sA[(ak + (SB_THREADS / SB_BM) * s) * LDS_A + ar] =
                keep_if(avalid & (kk < ki.kw), ra[s]);
        }
#pragma unroll
        for (int s = 0; s < BE; ++s) {
            const int t = ki.kmin + k0 + bk + s;
            sB[(bk + s) * LDS_B + bc] =
                keep_if(bvalid & (t <= tlast) & (t >= bt0), rb[s]);
        }
    };

    typename M::acc_t acc[FM][FN];
#pragma unroll
    for (int a = 0; a < FM; ++a)
#pragma unroll
        for (int b = 0; b < FN; ++b) acc[a][b] = M::zero();

    const int nst = (ki.kw + SB_BK - 1) / SB_BK;
    gload(0);
    lstore(0, 0);
    __syncthreads();
    SB_STAMP(c1_);
    auto mfma_stage = [&](int st) {
        const T *sA = smem + (st & 1) * STAGE, *sB = sA + SB_BK * LDS_A;
#pragma unroll
        for (int ks = 0; ks < SB_BK; ks += M::KSTEP) {
            const int kl = ks + (lane >> 4);
            T av[FM], bv[FN];
#pragma unroll
            for (int f = 0; f < FM; ++f)
                av[f] = sA[kl * LDS_A + wr * (16 * FM) + f * 16 + (lane & 15)];
#pragma unroll
            for (int f = 0; f < FN; ++f)
                bv[f] = sB[kl * LDS_B + wc * (16 * FN) + f * 16 + (lane & 15)];
#pragma unroll
            for (int fm = 0; fm < FM; ++fm)
#pragma unroll
                for (int fn = 0; fn < FN; ++fn) M::step(acc[fm][fn], av[fm], bv[fn]);
        }
    };
    for (int st = 0; st + 1 < nst; ++st) {
        gload((st + 1) * SB_BK);
        mfma_stage(st);
        lstore((st + 1) & 1, (st + 1) * SB_BK);
        __syncthreads();
    }
    // last stage (peeled: no prefetch, so its registers carry the second
    // half of the destination tables instead): per (row block, column) the
    // column part of the address, tagged with the column block (1 + bl) or
    // 0 for a U destination; per (column block, row) the lmap position.
    constexpr int RLT = RLN / SB_THREADS; // lmap positions per thread
    int64_t t_code = 0, t_uv = 0;
    int t_fst = 0, t_rl[RLT];
#pragma unroll
    for (int u = 0; u < RLT; ++u) t_rl[u] = 0;
    if (tbl) {
        if (tid < CPN) {
            const int al = tid / SB_BN, c = tid % SB_BN;
            if (al < NA && c < ncols) {
                const int bl = s_cb[c] - b0, rec = al * SB_TB + bl, ld = s_dld[rec];
                const int64_t x = s_db[rec] + s_cg[c];
                if (ld >= 0) {
                    t_code = (s_db[rec] + (int64_t)s_cg[c] * ld) * 8 + 1 + bl;
                } else {
                    t_uv = ucol_voff[x];
                    t_fst = ucol_fst[x];
                }
            }
        }
#pragma unroll
        for (int u = 0; u < RLT; ++u) {
            const int e = tid + u * SB_THREADS, bl = e / SB_BM, rr = e % SB_BM;
            if (bl < NB && rr < mrows) {
                const int rec = (s_ra[rr] - a0) * SB_TB + bl;
                if (s_dld[rec] >= 0) t_rl[u] = lmap[s_dmb[rec] + s_rg[rr]];
            }
        }
    }
    mfma_stage(nst - 1);
    __syncthreads();
    if (tbl) {
        if (tid < CPN) s_cp[tid] = t_code ? t_code : (t_uv - t_fst) * 8;
#pragma unroll
        for (int u = 0; u < RLT; ++u) s_rl[tid + u * SB_THREADS] = t_rl[u];
    }

    // ---- epilogue: passes of PASSW columns through LDS, column-contiguous.
    // Thread (r, q) owns row r and columns q, q+4, ...  (a wave = 64 rows of
    // one column, so column data is wave-uniform).
    SB_STAMP(c2_);
    T *sC = smem; // [c][r], ld CLD
    constexpr int TPR = SB_THREADS / SB_BM, CPT = PASSW / TPR;
    const int r = tid & (SB_BM - 1), q = tid / SB_BM;
    const int gr = s_rg[r], a = s_ra[r];
    // C tile columns [pass*PASSW, (pass+1)*PASSW) from the accumulators into LDS
    auto stage_c = [&](int pass) {
#pragma unroll
        for (int fn = 0; fn < FN; ++fn) {
            const int c0 = wc * 16 * FN + fn * 16; // first tile column of fragment column fn
            if (c0 / PASSW != pass) continue;
#pragma unroll
            for (int fm = 0; fm < FM; ++fm)
#pragma unroll
                for (int i = 0; i < 4; ++i) {
                    const int rr = wr * (16 * FM) + fm * 16 + M::row(lane, i);
                    const int cc = c0 - pass * PASSW + (lane & 15);
                    sC[cc * CLD + rr] = M::get(acc[fm][fn], i);
                }
        }
    };
    // Fast path (tbl): a tile's rows lie in NA consecutive L blocks of the
    // panel and its columns in NB consecutive U blocks; with NA, NB <= TB
    // (99.6 % of the 100^3 flops) every destination address splits into a
    // column part and a row part,
    //   L(ib,jb): Lval + [colvoff + (gc - fcol)*ld] + [lmap position of gr]
    //   U(ib,jb): Uval + [ucol_voff - ucol_fst](ib, gc) + [gr]
    // resolved once per tile above: the column parts per (row block, column)
    // in LDS (tagged with the column block, 0 = U destination), the lmap
    // positions per column block in the row's registers.  The scatter then
    // reads one LDS word per element besides the destination itself
    // (dscatter_l / dscatter_u, SRC/dscatter.c:137-142,229-235 search per
    // element).  The stores are fire-and-forget atomic adds: no load round
    // trip per element; where a tile is the only writer of its destinations
    // the sums are the plain subtraction's, bit for bit.
    if (tbl) {
        int rl[SB_TB];
        const int al = a - a0;
        for (int pass = 0; pass < SB_BN / PASSW; ++pass) {
            stage_c(pass);
            __syncthreads();
            if (pass == 0) {
#pragma unroll
                for (int bl = 0; bl < SB_TB; ++bl) rl[bl] = s_rl[bl * SB_BM + r];
            }
            if (r < mrows) {
                constexpr int EB = CPT < SB_AEB ? CPT : SB_AEB;
#pragma unroll
                for (int j0 = 0; j0 < CPT; j0 += EB) {
                    T *dp[EB];
                    T v[EB];
#pragma unroll
                    for (int j = 0; j < EB; ++j) {
                        const int cl = q + TPR * (j0 + j), c = pass * PASSW + cl;
                        dp[j] = nullptr;
                        v[j] = Sx::zero();
                        if (c < ncols) {
                            v[j] = sC[cl * CLD + r];
                            const int64_t code = s_cp[al * SB_BN + c];
                            const int tag = (int)(code & 7);
                            int rp = gr; // branch-free: U row part, or the column block's lmap position
                            rp = tag == 1 ? rl[0] : rp;
                            rp = tag == 2 ? rl[1] : rp;
                            rp = tag == 3 ? rl[2] : rp;
                            rp = tag == 4 ? rl[3] : rp;
                            T *const base = tag ? Lval : Uval;
                            dp[j] = base + ((code >> 3) + rp);
                        }
                    }
#pragma unroll
                    for (int j = 0; j < EB; ++j)
                        if (dp[j]) Sx::atomic_sub(dp[j], v[j]);
                }
            }
            __syncthreads();
        }
    } else {
        // slow path (tiles over more blocks): per-element table walk, EB
        // read-modify-writes in flight per thread
        constexpr int EB = CPT < 4 ? CPT : 4; // (8 in flight: slower)
        static_assert(CPT % EB == 0, "epilogue batches");
        const int *prow = ki.pair + (int64_t)a * ki.nub;
        int lastb = -1, h = 0, ldh = 0;
        int64_t rbase = 0;
        for (int pass = 0; pass < SB_BN / PASSW; ++pass) {
            stage_c(pass);
            __syncthreads();
            if (r < mrows) {
#pragma unroll
                for (int j0 = 0; j0 < CPT; j0 += EB) {
                    T *dp[EB];
                    T v[EB];
#pragma unroll
                    for (int j = 0; j < EB; ++j) {
                        const int cl = q + TPR * (j0 + j), c = pass * PASSW + cl;
                        dp[j] = nullptr;
                        v[j] = Sx::zero();
                        if (c < ncols) {
                            v[j] = sC[cl * CLD + r];
                            const int b = s_cb[c], gc = s_cg[c];
                            if (b != lastb) {
                                lastb = b;
                                h = prow[b];
                                if (h >= 0) {
                                    const LBlk L = lblk[h];
                                    ldh = L.ld;
                                    rbase = L.colvoff + lmap[L.mapoff + gr - L.frow] -
                                            (int64_t)L.fcol * L.ld;
                                }
                            }
                            if (h >= 0) {
                                dp[j] = Lval + rbase + (int64_t)gc * ldh;
                            } else {
                                const UBlk U = ublk[~h];
                                const int64_t e = U.coloff + gc - U.fcol;
                                dp[j] = Uval + ucol_voff[e] + gr - ucol_fst[e];
                            }
                        }
                    }
                    if (ki.atomic) {
#pragma unroll
                        for (int j = 0; j < EB; ++j)
                            if (dp[j]) Sx::atomic_sub(dp[j], v[j]);
                    } else {
                        T o[EB];
#pragma unroll
                        for (int j = 0; j < EB; ++j) o[j] = dp[j] ? *dp[j] : Sx::zero();
#pragma unroll
                        for (int j = 0; j < EB; ++j)
                            if (dp[j]) *dp[j] = Sx::sub(o[j], v[j]);
                    }
                }
            }
            __syncthreads();
        }
    }
#ifdef SLU_SB_STAMP
    SB_STAMP(c3_);
    if (tid == 0) {
        const unsigned s = atomicAdd(&slu_stamp_n, 1u);
        if (s < SLU_STAMP_MAX) {
            const unsigned hw = __builtin_amdgcn_s_getreg((31 << 11) | 4);   // HW_ID
            const unsigned xcc = __builtin_amdgcn_s_getreg((31 << 11) | 20); // XCC_ID
            uint64_t *o = slu_stamp + (size_t)s * 4;
            const uint64_t *t = s_stamp_;
            o[0] = (t[rt_] & ((1ull << 40) - 1)) | (((wall_clock64() - t[rt_]) & 0xFFFFFFull) << 40);
            o[1] = (uint64_t)(t[c1_] - t[c0_]) | ((uint64_t)(t[c2_] - t[c1_]) << 32);
            o[2] = (uint64_t)(t[c3_] - t[c2_]) | ((uint64_t)hw << 32);
            o[3] = (uint64_t)(xcc & 15) | ((uint64_t)ki.kw << 4) | ((uint64_t)mrows << 14) |
                   ((uint64_t)ncols << 22) | ((uint64_t)ki.atomic << 30) | ((uint64_t)blockIdx.x << 32);
        }
    }
#endif
}


// TRSM with the RB x w row slab of X held in MFMA A-operand registers
// (fp64 / fp32): wave q owns rows 16q..16q+15; lane keeps X[row lane&15]
// [4s + lane>>4] for k-step s.  Column block b: acc = X_{<b} T_{<b,b} (B from
// LDS), Z = X_b - acc, X_b = Z Dinv_b; results return to A layout through a
// per-wave LDS tile.  Same MODE convention as k_trsm_blk.
constexpr int TR_WAVES = 4;
// T staged 8 elements per thread in flight (16: slower, profiles/r05tu/) --
// the non-PF form.  Round 6's phase probes (profiles/r06j/trsm_micro.txt) put
// 40% of a lone 256-wide slab's 59 us in that staging (one global round trip
// per 8 elements, 1 wave per SIMD, nothing to hide it) and 13% in the final
// store; the PF form below (next block's T / Dinv in registers, loads that
// land untouched until used, stores per block) takes it to 39 us, and
// serialized 100^3 TRSM from 29.0 to 23.1 ms with the pipelined factor
// unchanged (profiles/r06j/).  (Round 5's register prefetch masked the
// loaded values, which made the compiler wait for each load at once.)
constexpr int TR_TU = 8;
// B operands read from LDS this many k-steps ahead of their MFMAs (k_trsm_reg)
#ifndef TR_PFD
#define TR_PFD 4
#endif
// LDS written by a wave, then read by other lanes of the same wave
__device__ __forceinline__ void wave_lds_sync() {
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_s_waitcnt(0xc07f); // lgkmcnt(0)
    __builtin_amdgcn_wave_barrier();
}
#ifdef SLU_TR_PROBE
// Diagnostics build only (tools/micro/trsm_micro.hip): k_trsm_reg cycles per
// phase summed over workgroups (thread 0's view): 0 X load, 1 Dinv/T staging,
// 2 X_{<b} T_{<b,b} MFMAs, 3 Z Dinv_b with its layout changes, 4 X store.
__device__ long long slu_tr_tp[8];
#define TR_PROBE_START() long long tr_t0 = clock64()
#define TR_PROBE(i)                                                                          \
    do {                                                                                     \
        if (threadIdx.x == 0) {                                                              \
            const long long t = clock64();                                                   \
            atomicAdd((unsigned long long *)&slu_tr_tp[i], (unsigned long long)(t - tr_t0)); \
            tr_t0 = t;                                                                       \
        }                                                                                    \
    } while (0)
#else
#define TR_PROBE_START()
#define TR_PROBE(i)
#endif
// MAXW: the widest supernode of the launch's items.  The narrow levels
// (MAXW 64: 16 row registers, 17 KB of LDS) run several workgroups per CU
// where the 256-wide form (64 registers, 68 KB) runs one.
// PF (the latency form, for launches of few slabs, where each workgroup's
// chain of global round trips is the launch time): Dinv_{b+1} and
// T_{<b+1,b+1} are loaded into registers while block b computes, and the
// columns of block b are stored as soon as they are final.
template <typename T, int MODE, int MAXW = FAST_MAXW, bool PF = false>
__global__ void __launch_bounds__(64 * TR_WAVES, MAXW <= 64 ? 4 : MAXW <= 128 ? 2 : 1)
__attribute__((amdgpu_waves_per_eu(MAXW <= 64 ? 4 : MAXW <= 128 ? 2 : 1, MAXW <= 64 ? 4 : MAXW <= 128 ? 2 : 1)))
k_trsm_reg(const TrsmItemF<T> *items) {
    constexpr int PW = 32, NKS = MAXW / 4, NBMAX = MAXW / PW;
    constexpr int TROWS = MAXW - PW > TR_WAVES * 16 ? MAXW - PW : TR_WAVES * 16; // sT rows
    using Sx = S<T>;
    using M = Mma<T>;
    TR_PROBE_START();
    const TrsmItemF<T> it = items[blockIdx.x];
    const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
    const int w = it.w, nb = (w + PW - 1) / PW;
    // sW (each wave's 16 x PW layout-change tile) lives in the first rows of
    // sT, which the block's MFMAs have read by then (a barrier separates
    // them): 68 KB of LDS instead of 85, so the kernel fits beside a Schur
    // workgroup (engine.hip, rest_split)
    __shared__ T sT[TROWS][PW + 1];
    static_assert(TR_WAVES * 16 <= TROWS, "sW inside sT");
    T (*W)[PW + 1] = sT + wid * 16;
    __shared__ T sD[PW][PW + 1];
    const int rl = lane & 15, kq = lane >> 4;
    const int myr = wid * 16 + rl;
    // fp64: the block products computed transposed (their C layout is then
    // the A layout X lives in); fp32's C layout differs, so it goes through
    // the per-wave LDS tile
    constexpr bool TRANSPOSED = std::is_same<T, double>::value;
    const bool rv = myr < it.nrows;
    int64_t rbase = 0;
    int t0 = 0;
    if (MODE == 1 && rv) {
        t0 = it.t0[myr];
        rbase = it.voff[myr] - t0;
    }
    constexpr int NT = 64 * TR_WAVES, DPT = PW * PW / NT; // Dinv elements per thread
    static_assert(PW * PW % NT == 0, "TR_WAVES");
    T pd[DPT], pt[PF ? DPT * (NBMAX - 1) : 1]; // PF: the next block's Dinv / T
    // T_{<b,b} element e (b * PW * PW of them, DPT * b per thread); the
    // columns past w are masked when stored, not when loaded, so that the
    // loads can land in registers untouched until then
    auto t_src = [&](int b, int e) {
        const int kr = b * PW;
        const int i = MODE == 0 ? e % kr : e / PW, j = MODE == 0 ? e / kr : e % PW;
        const int col = min(b * PW + j, w - 1);
        return gld(MODE == 0 ? it.t + i + (int64_t)col * it.ldt : it.t + col + (int64_t)i * it.ldt);
    };
    auto t_put = [&](int b, int e, T v) {
        const int kr = b * PW;
        const int j = MODE == 0 ? e / kr : e % PW;
        v = keep_if(b * PW + j < w, v);
        if (MODE == 0) sT[e % kr][e / kr] = v;
        else sT[e / PW][e % PW] = v;
    };
    // (PF: Dinv_0, Dinv_1 and T_{<1,1} requested ahead of X, so that their
    // round trip overlaps X's)
    T pd0[DPT];
    if (PF) {
#pragma unroll
        for (int u = 0; u < DPT; ++u) pd0[u] = gld(it.dinv + tid + u * NT);
        if (nb > 1) {
#pragma unroll
            for (int u = 0; u < DPT; ++u) pd[u] = gld(it.dinv + PW * PW + tid + u * NT);
#pragma unroll
            for (int u = 0; u < DPT; ++u) pt[u] = t_src(1, tid + u * NT);
        }
    }
    T xa[NKS];
#pragma unroll
    for (int s = 0; s < NKS; ++s) {
        const int k = 4 * s + kq;
        T v = Sx::zero();
        if (rv && k < w) {
            if (MODE == 0) v = it.x[myr + (int64_t)k * it.ldx];
            else if (k >= t0) v = it.x[rbase + k];
        }
        xa[s] = v;
    }
#ifdef SLU_TR_PROBE
    if (tid == 0) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
#endif
    TR_PROBE(0);
#pragma unroll
    for (int b = 0; b < NBMAX; ++b) {
        if (b >= nb) break;
        __syncthreads();
        const int kr = b * PW;
        if (PF) {
#pragma unroll
            for (int u = 0; u < DPT; ++u) sD[(tid + u * NT) / PW][(tid + u * NT) % PW] = b == 0 ? pd0[u] : pd[u];
#pragma unroll
            for (int u = 0; u < DPT * b; ++u) t_put(b, tid + u * NT, pt[u]);
        } else {
            stage_loop<64 * TR_WAVES, 4, T>(
                tid, PW * PW,
                [&](int e, bool ok) { return keep_if(ok, gld(it.dinv + (int64_t)b * PW * PW + min(e, PW * PW - 1))); },
                [&](int e, T v) { sD[e / PW][e % PW] = v; });
        }
        if (!PF && kr > 0)
            stage_loop<64 * TR_WAVES, TR_TU, T>(
                tid, kr * PW,
                [&](int e, bool ok) {
                    const int ee = min(e, kr * PW - 1);
                    const int i = MODE == 0 ? ee % kr : ee / PW, j = MODE == 0 ? ee / kr : ee % PW;
                    const int col = min(b * PW + j, w - 1);
                    const T *src = MODE == 0 ? it.t + i + (int64_t)col * it.ldt : it.t + col + (int64_t)i * it.ldt;
                    return keep_if(ok & (b * PW + j < w), gld(src));
                },
                [&](int e, T v) {
                    if (MODE == 0) sT[e % kr][e / kr] = v;
                    else sT[e / PW][e % PW] = v;
                });
        __syncthreads();
        if (PF && b > 0 && b + 1 < nb) {
#pragma unroll
            for (int u = 0; u < DPT; ++u) pd[u] = gld(it.dinv + (int64_t)(b + 1) * PW * PW + tid + u * NT);
#pragma unroll
            for (int u = 0; u < DPT * (b + 1); ++u) pt[u] = t_src(b + 1, tid + u * NT);
        }
        TR_PROBE(1);
        typename M::acc_t a0 = M::zero(), a1 = M::zero();
        {
            // the B operands read from LDS TR_PFD k-steps ahead of their
            // MFMAs: one wave per SIMD has no other wave to hide an LDS read
            // behind, and with the read right before its MFMA every pair of
            // MFMAs waited for one (lgkmcnt(0)) -- the compiler, short of
            // registers, did not pipeline them itself
            T q0[TR_PFD], q1[TR_PFD];
            const int ns = 8 * b;
#pragma unroll
            for (int s = 0; s < TR_PFD; ++s)
                if (s < ns) {
                    q0[s] = sT[4 * s + kq][rl];
                    q1[s] = sT[4 * s + kq][16 + rl];
                }
#pragma unroll
            for (int s = 0; s < 8 * b; ++s) {
                const T b0 = q0[s % TR_PFD], b1 = q1[s % TR_PFD];
                if (s + TR_PFD < ns) {
                    q0[s % TR_PFD] = sT[4 * (s + TR_PFD) + kq][rl];
                    q1[s % TR_PFD] = sT[4 * (s + TR_PFD) + kq][16 + rl];
                }
                // (the scheduler would sink the reads back to their uses)
                __builtin_amdgcn_sched_barrier(0);
                if constexpr (TRANSPOSED) { // (X T)^T = T^T X^T
                    M::step(a0, b0, xa[s]);
                    M::step(a1, b1, xa[s]);
                } else {
                    M::step(a0, xa[s], b0);
                    M::step(a1, xa[s], b1);
                }
                __builtin_amdgcn_sched_barrier(0);
            }
        }
        if constexpr (TRANSPOSED) {
            // the products' transposes in C layout are X_b's own A layout
            // (fp64: lane l holds rows l & 15, columns (l >> 4) + 4 i): Z and
            // Z Dinv_b need no trip through LDS
            TR_PROBE(2);
            T za[8];
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                za[i] = Sx::sub(xa[8 * b + i], M::get(a0, i));
                za[4 + i] = Sx::sub(xa[8 * b + 4 + i], M::get(a1, i));
            }
            typename M::acc_t c0 = M::zero(), c1 = M::zero();
#pragma unroll
            for (int s = 0; s < 8; ++s) {
                M::step(c0, sD[4 * s + kq][rl], za[s]);
                M::step(c1, sD[4 * s + kq][16 + rl], za[s]);
            }
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                xa[8 * b + i] = M::get(c0, i);
                xa[8 * b + 4 + i] = M::get(c1, i);
            }
        } else {
        __syncthreads(); // every wave is done with sT before W (= its first rows) is written
        TR_PROBE(2);
        // Z = X_b - acc: acc (C layout) -> LDS, read back in A layout
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            W[M::row(lane, i)][rl] = M::get(a0, i);
            W[M::row(lane, i)][16 + rl] = M::get(a1, i);
        }
        // W is the wave's own: its layout changes need the wave's LDS writes
        // done, not the workgroup (the first __syncthreads above covers sT)
        wave_lds_sync();
        T za[8], d0[8], d1[8];
#pragma unroll
        for (int s = 0; s < 8; ++s) { // (Dinv_b's B operands read with Z: one wait for both)
            d0[s] = sD[4 * s + kq][rl];
            d1[s] = sD[4 * s + kq][16 + rl];
        }
#pragma unroll
        for (int s = 0; s < 8; ++s) za[s] = Sx::fms(xa[8 * b + s], W[rl][4 * s + kq], one_of(xa[0]));
        typename M::acc_t c0 = M::zero(), c1 = M::zero();
#pragma unroll
        for (int s = 0; s < 8; ++s) {
            M::step(c0, za[s], d0[s]);
            M::step(c1, za[s], d1[s]);
        }
        wave_lds_sync();
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            W[M::row(lane, i)][rl] = M::get(c0, i);
            W[M::row(lane, i)][16 + rl] = M::get(c1, i);
        }
        wave_lds_sync();
#pragma unroll
        for (int s = 0; s < 8; ++s) xa[8 * b + s] = W[rl][4 * s + kq];
        }
        if (PF) {
#pragma unroll
            for (int s = 8 * b; s < 8 * b + 8; ++s) {
                const int k = 4 * s + kq;
                if (rv && k < w) {
                    if (MODE == 0) it.x[myr + (int64_t)k * it.ldx] = xa[s];
                    else if (k >= t0) it.x[rbase + k] = xa[s];
                }
            }
        }
        TR_PROBE(3);
    }
#pragma unroll
    for (int s = 0; s < (PF ? 0 : NKS); ++s) {
        const int k = 4 * s + kq;
        if (rv && k < w) {
            if (MODE == 0) it.x[myr + (int64_t)k * it.ldx] = xa[s];
            else if (k >= t0) it.x[rbase + k] = xa[s];
        }
    }
#ifdef SLU_TR_PROBE
    if (tid == 0) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
#endif
    TR_PROBE(4);
}

} // namespace slu

// Device-resident triangular solves with the factored supernodal L and U
// (1x1 grid), level-scheduled like the factorization: SURVEY §8(f) row 2,
// the first step of pdgstrs (SRC/pdgstrs.c, SRC/pdgstrs_lsum.c) on the
// factors the engine leaves in HBM.  Included by engine.hip.
//
// Forward  L y = b : per level, (1) unit-lower solve with each supernode's
//                    diagonal block, (2) y_rows_below -= L_panel * y_k
//                    (chunks of 256 panel rows, atomics across supernodes).
// Backward U x = y : per level in reverse, (1) y_k -= U(k,:) x over the
//                    supernode's U row segments (chunks of 256 columns,
//                    atomics), (2) upper solve with the diagonal block.
// The diagonal block holds L\U in the first w rows of the supernode's L
// column block (SRC/pdgstrf2.c:213-269 stores U11 there); the arithmetic per
// element is the reference's dtrsv/dgemv on those blocks (SRC/pdgstrs.c
// dlsum_fmod / dlsum_bmod).
#pragma once
#include "kernels.h"

namespace slu {

struct SvDiag {     // one supernode's diagonal block
    int64_t voff;   // offset of its L column block in Lval
    int ld, w, fst; // nsupr, width, first global row/column
    int pad;
};
struct SvChunk {    // 256 panel rows (forward) or 256 U columns (backward)
    int sn;         // index into the SvDiag / per-supernode tables
    int c0;         // first row below the diagonal block / first U column
};

constexpr int SV_THREADS = 256;  // panel chunks
constexpr int SVD_THREADS = 512; // diagonal solves: one thread per row, w <= MAX_SUPER_SIZE

// value of lane `src` (wavefront-uniform) for every lane: v_readlane into a
// scalar register, no LDS round trip (tools/micro/lat_micro.hip: readlane +
// FMA 56 cycles against 92 for an LDS load)
__device__ inline float sv_shfl(float v, int src) {
    return __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), src));
}
__device__ inline double sv_shfl(double v, int src) {
    const long long b = __double_as_longlong(v);
    const int lo = __builtin_amdgcn_readlane((int)b, src);
    const int hi = __builtin_amdgcn_readlane((int)(b >> 32), src);
    return __longlong_as_double(((long long)hi << 32) | (unsigned)lo);
}
__device__ inline zc sv_shfl(zc v, int src) { return {sv_shfl(v.r, src), sv_shfl(v.i, src)}; }

// columns per panel of the diagonal solves: 32 (16 complex, to keep the
// thread's panel row in registers); divides the 64-wide wavefront, so a
// panel's rows always sit in one wavefront
template <typename T> struct SvPanel { static constexpr int v = sizeof(T) == 16 ? 16 : 32; };

// Right-hand sides: NR (compile-time, 1 or SV_NR) columns of x with leading
// dimension ldx, of which the first nr (<= NR, uniform) are live; every
// factor element is read once per sweep for all of them.  Dead columns are
// carried as zeros through the arithmetic (never loaded or stored), so the
// NR independent chains stay branch-free and interleave.
constexpr int SV_NR = 8;
template <typename T> struct SvNr { static constexpr int v = sizeof(T) == 16 ? 2 : SV_NR; }; // no spills

// L_kk y_k = b_k, unit lower, blocked by SVP-column panels.  Thread t owns
// row t and holds its SVP panel entries in registers (one coalesced batch of
// loads per panel).  The panel's own rows are solved inside their wavefront
// (y_j passed by lane shuffle, no barrier per column); one barrier publishes
// the panel's y through LDS, then every row below subtracts L(t, panel) y.
template <typename T, int NR>
__global__ void __launch_bounds__(SVD_THREADS)
k_sv_ldiag(const SvDiag *items, const T *Lval, T *x, int64_t ldx, int nr) {
    using Sx = S<T>;
    constexpr int SVP = SvPanel<T>::v;
    const SvDiag it = items[blockIdx.x];
    const T *L = Lval + it.voff;
    const int t = threadIdx.x, w = it.w, ld = it.ld;
    __shared__ T s_y[2][NR][SVP];
    T yi[NR];
#pragma unroll
    for (int q = 0; q < NR; ++q) yi[q] = (q < nr && t < w) ? x[it.fst + t + q * ldx] : Sx::zero();
    for (int j0 = 0, buf = 0; j0 < w; j0 += SVP, buf ^= 1) {
        const int nj = min(SVP, w - j0);
        T l[SVP];
#pragma unroll
        for (int j = 0; j < SVP; ++j)
            l[j] = (j < nj && t > j0 + j && t < w) ? L[t + (int64_t)(j0 + j) * ld] : Sx::zero();
        if ((t >> 6) == (j0 >> 6)) {
            const int base = j0 & 63;
#pragma unroll
            for (int j = 0; j < SVP; ++j) {
                const bool upd = t > j0 + j && t < j0 + nj;
#pragma unroll
                for (int q = 0; q < NR; ++q) {
                    const T yj = sv_shfl(yi[q], base + j);
                    if (upd) yi[q] = Sx::fms(yi[q], l[j], yj);
                }
            }
            if (t >= j0 && t < j0 + nj)
#pragma unroll
                for (int q = 0; q < NR; ++q) s_y[buf][q][t - j0] = yi[q];
        }
        __syncthreads();
        if (t >= j0 + nj && t < w) { // only for full panels (a partial one is the last)
#pragma unroll
            for (int q = 0; q < NR; ++q) {
#pragma unroll
                for (int j = 0; j < SVP; ++j) yi[q] = Sx::fms(yi[q], l[j], s_y[buf][q][j]);
            }
        }
    }
#pragma unroll
    for (int q = 0; q < NR; ++q)
        if (q < nr && t < w) x[it.fst + t + q * ldx] = yi[q];
}

// U_kk x_k = y_k (upper, non-unit), blocked like k_sv_ldiag from the last
// panel up: in-panel back substitution by lane shuffles, then every row above
// the panel subtracts U(t, panel) x_panel.
template <typename T, int NR>
__global__ void __launch_bounds__(SVD_THREADS)
k_sv_udiag(const SvDiag *items, const T *Lval, T *x, int64_t ldx, int nr) {
    using Sx = S<T>;
    constexpr int SVP = SvPanel<T>::v;
    const SvDiag it = items[blockIdx.x];
    const T *L = Lval + it.voff;
    const int t = threadIdx.x, w = it.w, ld = it.ld;
    __shared__ T s_x[2][NR][SVP];
    T yi[NR];
#pragma unroll
    for (int q = 0; q < NR; ++q) yi[q] = (q < nr && t < w) ? x[it.fst + t + q * ldx] : Sx::zero();
    for (int j0 = ((w - 1) / SVP) * SVP, buf = 0; j0 >= 0; j0 -= SVP, buf ^= 1) {
        const int nj = min(SVP, w - j0);
        T u[SVP];
#pragma unroll
        for (int j = 0; j < SVP; ++j)
            u[j] = (j < nj && t < j0 + j) ? L[t + (int64_t)(j0 + j) * ld] : Sx::zero();
        const bool mine = t >= j0 && t < j0 + nj;
        const T d = mine ? L[t + (int64_t)t * ld] : Sx::zero();
        if ((t >> 6) == (j0 >> 6)) {
            const int base = j0 & 63;
#pragma unroll
            for (int j = SVP - 1; j >= 0; --j) {
                if (j < nj) {
                    const bool upd = t >= j0 && t < j0 + j;
#pragma unroll
                    for (int q = 0; q < NR; ++q) {
                        if (t == j0 + j) yi[q] = Sx::div(yi[q], d);
                        const T xj = sv_shfl(yi[q], base + j);
                        if (upd) yi[q] = Sx::fms(yi[q], u[j], xj);
                    }
                }
            }
            if (mine)
#pragma unroll
                for (int q = 0; q < NR; ++q) s_x[buf][q][t - j0] = yi[q];
        }
        __syncthreads();
        if (t < j0) { // the first (last-column) panel may be partial: no stale LDS
#pragma unroll
            for (int q = 0; q < NR; ++q) {
#pragma unroll
                for (int j = 0; j < SVP; ++j)
                    if (j < nj) yi[q] = Sx::fms(yi[q], u[j], s_x[buf][q][j]);
            }
        }
    }
#pragma unroll
    for (int q = 0; q < NR; ++q)
        if (q < nr && t < w) x[it.fst + t + q * ldx] = yi[q];
}

// x[rows below] -= L_panel(256-row chunk) * y_k.  The panel descriptor
// (SvDiag fields) points at the first row below the diagonal block: voff =
// its offset in Lval, ld = nsupr, pad = number of rows below (on a 2D grid
// the rank's rows of L(:,k) on its process row; on the diagonal owner they
// follow the diagonal block, elsewhere the column block has none).
template <typename T, int NR>
__global__ void __launch_bounds__(SV_THREADS)
k_sv_lpanel(const SvChunk *chunks, const SvDiag *pan, const int64_t *roff, const int *rows,
            const T *Lval, T *x, int64_t ldx, int nr) {
    using Sx = S<T>;
    const SvChunk ch = chunks[blockIdx.x];
    const SvDiag it = pan[ch.sn];
    const int t = threadIdx.x, w = it.w, nb = it.pad;
    __shared__ T s_y[NR][FAST_MAXW * 2];
    for (int q = 0; q < nr; ++q)
        for (int j = t; j < w; j += SV_THREADS) s_y[q][j] = x[it.fst + j + q * ldx];
    __syncthreads();
    const int r = ch.c0 + t;
    if (r >= nb) return;
    const T *L = Lval + it.voff + r;
    T acc[NR];
#pragma unroll
    for (int q = 0; q < NR; ++q) acc[q] = Sx::zero();
    constexpr int UN = 16; // columns of loads in flight per thread
    for (int j0 = 0; j0 < w; j0 += UN) {
        T v[UN];
#pragma unroll
        for (int u = 0; u < UN; ++u) v[u] = j0 + u < w ? L[(int64_t)(j0 + u) * it.ld] : Sx::zero();
#pragma unroll
        for (int q = 0; q < NR; ++q) {
#pragma unroll
            for (int u = 0; u < UN; ++u)
                if (j0 + u < w) acc[q] = Sx::fms(acc[q], v[u], s_y[q][j0 + u]);
        }
    }
    // acc = -(L_r . y)
    const int64_t gr = rows[roff[ch.sn] + r];
#pragma unroll
    for (int q = 0; q < NR; ++q)
        if (q < nr) Sx::atomic_sub(x + gr + q * ldx, Sx::neg(acc[q]));
}

// y_k -= U(k, chunk of SVU_COLS columns) x: thread t owns rows t, t + 256 of
// the supernode; each U column is a segment of rows fst..w-1 stored
// contiguously (coalesced along t).  Short chunks (many workgroups per
// supernode at the chain-bound top of the tree) and 16 columns of loads in
// flight per thread; partial sums meet in x through atomics.
constexpr int SVU_COLS = 64;
template <typename T, int NR>
__global__ void __launch_bounds__(SV_THREADS)
k_sv_upanel(const SvChunk *chunks, const SvDiag *diag, const int64_t *coff, const int *ncol,
            const int64_t *ucol_voff, const int *ucol_fst, const int *ucol_gc, const T *Uval,
            T *x, int64_t ldx, int nr) {
    using Sx = S<T>;
    constexpr int UN = 16;
    const SvChunk ch = chunks[blockIdx.x];
    const SvDiag it = diag[ch.sn];
    const int t = threadIdx.x, w = it.w;
    const int nc = min(SVU_COLS, ncol[ch.sn] - ch.c0);
    __shared__ int64_t s_v[SVU_COLS];
    __shared__ int s_f[SVU_COLS];
    __shared__ T s_x[NR][SVU_COLS];
    if (t < SVU_COLS) {
        const int64_t e = coff[ch.sn] + ch.c0 + t;
        s_v[t] = t < nc ? ucol_voff[e] : 0;
        s_f[t] = t < nc ? ucol_fst[e] - it.fst : w; // first row of the segment, relative
        const int64_t gc = t < nc ? ucol_gc[e] : 0;
#pragma unroll
        for (int q = 0; q < NR; ++q) s_x[q][t] = (t < nc && q < nr) ? x[gc + q * ldx] : Sx::zero();
    }
    __syncthreads();
    for (int i = t; i < w; i += SV_THREADS) { // w <= MAX_SUPER_SIZE = 2 x SV_THREADS
        T acc[NR];
#pragma unroll
        for (int q = 0; q < NR; ++q) acc[q] = Sx::zero();
        for (int c0 = 0; c0 < nc; c0 += UN) {
            T v[UN];
#pragma unroll
            for (int u = 0; u < UN; ++u) {
                const int rf = s_f[c0 + u]; // w (no load) past the chunk's last column
                v[u] = i >= rf ? Uval[s_v[c0 + u] + i - rf] : Sx::zero();
            }
#pragma unroll
            for (int q = 0; q < NR; ++q) {
#pragma unroll
                for (int u = 0; u < UN; ++u) acc[q] = Sx::fms(acc[q], v[u], s_x[q][c0 + u]);
            }
        }
#pragma unroll
        for (int q = 0; q < NR; ++q)
            if (q < nr) Sx::atomic_sub(x + it.fst + i + q * ldx, Sx::neg(acc[q]));
    }
}

// 2D-grid solve helpers (pdgstrs's lsum reduction, SRC/pdgstrs_lsum.c): the
// diagonal owner of a block row adds the nslot partial sums its process row
// sent, stored one after another (x[dst + i] += sum_s slot[src + s*len + i]);
// one item per block row, so no two workgroups update the same x.  Rows this
// rank does not own start a sweep at zero (x[dst + i] = 0 for src < 0).
struct SvAdd {
    int64_t dst, src;
    int len, nslot;
};
template <typename T>
__global__ void __launch_bounds__(256) k_sv_add(const SvAdd *items, T *x, const T *slot) {
    const SvAdd it = items[blockIdx.x];
    for (int i = threadIdx.x; i < it.len; i += 256) {
        if (it.src < 0) {
            x[it.dst + i] = S<T>::zero();
            continue;
        }
        T v = x[it.dst + i];
        for (int q = 0; q < it.nslot; ++q) v = S<T>::sub(v, S<T>::neg(slot[it.src + (int64_t)q * it.len + i]));
        x[it.dst + i] = v;
    }
}

// 2D-grid refinement (pdgsrfs with pdgsmv's distributed product,
// SRC/pdgsrfs.c:197-253, SRC/pdgsmv.c): every entry of A lives on the rank
// of its block, so a rank forms partial rows r_p = -A_p x and s_p = |A_p||x|
// from its own entries (rows in CSR over this rank's nonzeros, x replicated).
template <typename T>
__global__ void __launch_bounds__(256)
k_resid_part(const int64_t *rp, const int *rc, const int64_t *re, const T *a, const T *x, T *r,
             double *s, int n) {
    using Sx = S<T>;
    const int i = blockIdx.x * 256 + threadIdx.x;
    if (i >= n) return;
    T acc = Sx::zero();
    double tmp = 0.0;
    for (int64_t e = rp[i]; e < rp[i + 1]; ++e) {
        const T av = a[re[e]], xv = x[rc[e]];
        acc = Sx::fms(acc, av, xv);
        tmp += Sx::abs1(av) * Sx::abs1(xv);
    }
    r[i] = acc;
    s[i] = tmp;
}
// The partial rows of a block row go to its diagonal owner along the
// process row (nslot consecutive slots each), and the owner finishes them:
// r = b + sum r_p, s = |b| + sum s_p, berr = max |r_i| / s_i with the
// SAFE1 / SAFE2 guards, NaN winning the max as in k_resid.
struct RfRow {
    int64_t fst, src; // first row; first slot (elements) of the block row
    int len, nslot;
};
template <typename T>
__global__ void __launch_bounds__(256)
k_resid_fin(const RfRow *items, const T *b, T *r, const double *s, const T *slot_r,
            const double *slot_s, double safe1, double safe2, unsigned long long *berr) {
    using Sx = S<T>;
    const RfRow it = items[blockIdx.x];
    double mx = 0.0;
    for (int i = threadIdx.x; i < it.len; i += 256) {
        const int64_t row = it.fst + i;
        T rv = Sx::sub(r[row], Sx::neg(b[row]));
        double sv = s[row] + Sx::abs1(b[row]);
        for (int q = 0; q < it.nslot; ++q) {
            rv = Sx::sub(rv, Sx::neg(slot_r[it.src + (int64_t)q * it.len + i]));
            sv += slot_s[it.src + (int64_t)q * it.len + i];
        }
        r[row] = rv;
        const double ra = Sx::abs1(rv);
        double e = 0.0;
        if (sv > safe2) e = ra / sv;
        else if (sv != 0.0) e = (safe1 + ra) / sv;
        mx = (mx != mx || e != e) ? __builtin_nan("") : fmax(mx, e);
    }
    for (int off = 32; off > 0; off >>= 1) {
        const double o = __shfl_xor(mx, off, 64);
        mx = (mx != mx || o != o) ? __builtin_nan("") : fmax(mx, o);
    }
    if ((threadIdx.x & 63) == 0 && !(mx <= 0.0))
        atomicMax(berr, (unsigned long long)__double_as_longlong(mx));
}

// Residual of the iterative refinement (SRC/pdgsrfs.c:209-230) by rows of A
// (CSR index over the CSC values): r = b - A x, s = |A||x| + |b| (abs1 for
// complex, as pzgsrfs), berr = max_i |r_i| / s_i with the SAFE1 / SAFE2
// guards; the max over rows goes through the bit pattern of non-negative
// doubles (monotone as unsigned integers).
template <typename T>
__global__ void __launch_bounds__(256)
k_resid(const int64_t *rp, const int *rc, const int64_t *re, const T *a, const T *x, const T *b,
        T *r, int n, double safe1, double safe2, unsigned long long *berr) {
    using Sx = S<T>;
    const int i = blockIdx.x * 256 + threadIdx.x;
    double s = 0.0;
    if (i < n) {
        T acc = b[i];
        double tmp = Sx::abs1(b[i]);
        for (int64_t e = rp[i]; e < rp[i + 1]; ++e) {
            const T av = a[re[e]], xv = x[rc[e]];
            acc = Sx::fms(acc, av, xv);
            tmp += Sx::abs1(av) * Sx::abs1(xv);
        }
        r[i] = acc;
        const double ra = Sx::abs1(acc);
        if (tmp > safe2) s = ra / tmp;
        else if (tmp != 0.0) s = (safe1 + ra) / tmp;
    }
    // NaN must win the max, as SUPERLU_MAX lets it through to berr
    // (SRC/pdgsrfs.c:222-226): fmax alone would drop it.  A NaN's bit
    // pattern is above +Inf's as an unsigned integer, so atomicMax keeps it.
    for (int off = 32; off > 0; off >>= 1) {
        const double o = __shfl_xor(s, off, 64);
        s = (s != s || o != o) ? __builtin_nan("") : fmax(s, o);
    }
    if ((threadIdx.x & 63) == 0 && !(s <= 0.0))
        atomicMax(berr, (unsigned long long)__double_as_longlong(s));
}

template <typename T> __global__ void __launch_bounds__(256) k_axpy1(T *x, const T *dx, int n) {
    const int i = blockIdx.x * 256 + threadIdx.x;
    if (i < n) x[i] = S<T>::sub(x[i], S<T>::neg(dx[i]));
}

} // namespace slu

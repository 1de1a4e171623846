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

// L_kk y_k = b_k, unit lower; thread t owns row t, column j is read one step
// ahead (coalesced along the column), y_j is broadcast through LDS.
template <typename T>
__global__ void __launch_bounds__(SVD_THREADS) k_sv_ldiag(const SvDiag *items, const T *Lval, T *x) {
    using Sx = S<T>;
    const SvDiag it = items[blockIdx.x];
    const T *L = Lval + it.voff;
    const int t = threadIdx.x, w = it.w, ld = it.ld;
    __shared__ T s_y[2];
    T yi = t < w ? x[it.fst + t] : Sx::zero();
    T lc = (t < w && t > 0) ? L[t] : Sx::zero();
    for (int j = 0; j < w; ++j) {
        if (t == j) s_y[j & 1] = yi;
        __syncthreads();
        const T yj = s_y[j & 1];
        const T ln = (t < w && t > j + 1) ? L[t + (int64_t)(j + 1) * ld] : Sx::zero();
        if (t > j && t < w) yi = Sx::fms(yi, lc, yj);
        lc = ln;
    }
    if (t < w) x[it.fst + t] = yi;
}

// U_kk x_k = y_k (upper, non-unit), column sweep from the last column.
template <typename T>
__global__ void __launch_bounds__(SVD_THREADS) k_sv_udiag(const SvDiag *items, const T *Lval, T *x) {
    using Sx = S<T>;
    const SvDiag it = items[blockIdx.x];
    const T *L = Lval + it.voff;
    const int t = threadIdx.x, w = it.w, ld = it.ld;
    __shared__ T s_x[2];
    T yi = t < w ? x[it.fst + t] : Sx::zero();
    T uc = (t < w - 1) ? L[t + (int64_t)(w - 1) * ld] : Sx::zero(); // column w-1, rows < w-1
    for (int j = w - 1; j >= 0; --j) {
        if (t == j) {
            yi = Sx::div(yi, L[j + (int64_t)j * ld]);
            s_x[j & 1] = yi;
        }
        __syncthreads();
        const T xj = s_x[j & 1];
        const T un = (j > 0 && t < j - 1) ? L[t + (int64_t)(j - 1) * ld] : Sx::zero();
        if (t < j) yi = Sx::fms(yi, uc, xj);
        uc = un;
    }
    if (t < w) x[it.fst + t] = yi;
}

// x[rows below] -= L_panel(256-row chunk) * y_k.
template <typename T>
__global__ void __launch_bounds__(SV_THREADS)
k_sv_lpanel(const SvChunk *chunks, const SvDiag *diag, const int64_t *roff, const int *rows,
            const T *Lval, T *x) {
    using Sx = S<T>;
    const SvChunk ch = chunks[blockIdx.x];
    const SvDiag it = diag[ch.sn];
    const int t = threadIdx.x, w = it.w, nb = it.ld - it.w;
    __shared__ T s_y[FAST_MAXW * 2];
    for (int j = t; j < w; j += SV_THREADS) s_y[j] = x[it.fst + j];
    __syncthreads();
    const int r = ch.c0 + t;
    if (r >= nb) return;
    const T *L = Lval + it.voff + w + r;
    T acc = Sx::zero();
    for (int j = 0; j < w; ++j) acc = Sx::fms(acc, L[(int64_t)j * it.ld], s_y[j]);
    // acc = -(L_r . y)
    Sx::atomic_sub(x + rows[roff[ch.sn] + r], Sx::neg(acc));
}

// y_k -= U(k, chunk of 256 columns) x: thread t owns rows t, t + 256 of the supernode;
// each U column is a segment of rows fst..w-1 stored contiguously.
template <typename T>
__global__ void __launch_bounds__(SV_THREADS)
k_sv_upanel(const SvChunk *chunks, const SvDiag *diag, const int64_t *coff, const int *ncol,
            const int64_t *ucol_voff, const int *ucol_fst, const int *ucol_gc, const T *Uval,
            T *x) {
    using Sx = S<T>;
    const SvChunk ch = chunks[blockIdx.x];
    const SvDiag it = diag[ch.sn];
    const int t = threadIdx.x, w = it.w;
    const int nc = min(SV_THREADS, ncol[ch.sn] - ch.c0);
    __shared__ int64_t s_v[SV_THREADS];
    __shared__ int s_f[SV_THREADS];
    __shared__ T s_x[SV_THREADS];
    if (t < nc) {
        const int64_t e = coff[ch.sn] + ch.c0 + t;
        s_v[t] = ucol_voff[e];
        s_f[t] = ucol_fst[e] - it.fst; // first row of the segment, relative
        s_x[t] = x[ucol_gc[e]];
    }
    __syncthreads();
    for (int i = t; i < w; i += SV_THREADS) { // w <= MAX_SUPER_SIZE = 2 x SV_THREADS
        T acc = Sx::zero();
        for (int c = 0; c < nc; ++c) {
            const int rf = s_f[c];
            if (i >= rf) acc = Sx::fms(acc, Uval[s_v[c] + i - rf], s_x[c]);
        }
        Sx::atomic_sub(x + it.fst + i, Sx::neg(acc));
    }
}

} // namespace slu

// Diagonal-block LU of narrow supernodes (w <= 64), one WAVE per block:
// the levels near the leaves hold thousands of them (100^3: 11 082 at level
// 0; 2D 1000^2: 16 383), where k_diag_lu_f spent one 256-thread workgroup
// and a dozen barriers per 32-column panel on each (lap2d level 0: 1.6 ms
// for 16 383 blocks).  Included by engine.hip after kernels.h.
//
// Lane r holds row r of the block in registers (WMAX values) and the wave
// eliminates column by column -- the unblocked right-looking order of the
// reference's panel factorization (SRC/pdgstrf2.c:213-269: tiny-pivot
// replacement, reciprocal scaling of the column below the pivot, a zero
// pivot leaves its column unscaled and is reported through zpiv), the pivot
// row broadcast by v_readlane; no barrier at all.  The factored block goes
// back in place; then the TRSM kernels' dinv blocks of every 32-column panel
// p (row-major U_pp^{-1} and (L_pp^{-1})^T, DiagItemF) come from the
// factored 32 x 32 diagonal sub-blocks: lanes 0-31 form U_pp^{-1} by
// columns, lanes 32-63 L_pp^{-1}, through a per-wave LDS copy of the
// sub-block.
#pragma once
#include <hip/hip_runtime.h>

#include "kernels.h"

namespace slu {

constexpr int DW_WAVES = 4; // blocks per workgroup

template <typename T, int WMAX>
__global__ void __launch_bounds__(64 * DW_WAVES, 2)
k_diag_lu_w(const DiagItemF<T> *items, int n, double thresh, int replace_tiny, int *tiny_count, int *zpiv) {
    static_assert(WMAX == 32 || WMAX == 64, "one or two 32-column panels");
    constexpr int PW = 32;
    static_assert(PWOf<T>::v == PW, "real types: 32-column panels");
    using Sx = S<T>;
    __shared__ T sS[DW_WAVES][2][PW][PW + 1]; // a factored 32 x 32 diagonal sub-block, and its transpose
    __shared__ T sR[DW_WAVES][WMAX];       // reciprocal pivots (0 for a zero pivot)
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    const int item = blockIdx.x * DW_WAVES + wid;
    if (item >= n) return; // (whole waves; no barrier below)
    const DiagItemF<T> it = items[item];
    T *A = it.a;
    const int ld = it.ld, w = it.w;
    const bool mine = lane < w;
    T xr[WMAX];
#pragma unroll
    for (int c = 0; c < WMAX; ++c) xr[c] = (mine && c < w) ? A[lane + (int64_t)c * ld] : Sx::zero();
#pragma unroll
    for (int j = 0; j < WMAX; ++j) {
        if (j < w) { // (uniform)
        T piv = rlane(xr[j], j);
        if (replace_tiny && Sx::abs1(piv) < thresh) {
            piv = Sx::thresh(piv, thresh);
            if (lane == 0) atomicAdd(tiny_count, 1);
        }
        const int z = Sx::iszero(piv);
        if (z && lane == 0) atomicMax(&zpiv[it.k], it.fcol + j + 1);
        const T rp = z ? Sx::zero() : Sx::recip(piv);
        // rows below j eliminate, row j keeps the (replaced) pivot
        const bool below = lane > j;
        const T l = below ? (z ? xr[j] : Sx::mul(xr[j], rp)) : Sx::zero();
        xr[j] = below ? l : (lane == j ? piv : xr[j]);
        if (lane == 0) sR[wid][j] = rp;
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int c = j + 1; c < WMAX; ++c) {
            xr[c] = Sx::fms(xr[c], l, rlane(xr[c], j));
            if ((c & 3) == 3) __builtin_amdgcn_sched_barrier(0);
        }
        __builtin_amdgcn_sched_barrier(0);
        }
    }
#pragma unroll
    for (int c = 0; c < WMAX; ++c)
        if (mine && c < w) A[lane + (int64_t)c * ld] = xr[c];
    // ---- the dinv blocks, panel by panel: the factored 32 x 32 diagonal
    // sub-block goes to LDS as S and as S^T, then every lane solves one unit-
    // or pivot-diagonal upper triangular system by columns, the same code on
    // both halves of the wave: lanes 0-31 U_pp x = e_j (S above the diagonal,
    // reciprocal pivots) -> column j of U_pp^{-1}; lanes 32-63 L_pp^T x = e_j
    // (S^T above the diagonal, unit) -> column j of (L_pp^T)^{-1} =
    // (L_pp^{-1})^T, stored row-major exactly like the first
    const int nb = (w + PW - 1) / PW;
    const bool up = lane < PW;
    const int j = lane & (PW - 1);
    T *const out = up ? it.dinv : it.dinv + (int64_t)nb * PW * PW;
#pragma unroll
    for (int p = 0; p < WMAX / PW; ++p) {
        if (p < nb) {
            const int p0 = p * PW, pw = min(PW, w - p0);
            if (lane >= p0 && lane < p0 + PW) {
                const int r = lane - p0;
#pragma unroll
                for (int c = 0; c < PW; ++c) {
                    const T v = (r < pw && c < pw) ? xr[p0 + c] : Sx::zero();
                    sS[wid][0][r][c] = v;
                    sS[wid][1][c][r] = v;
                }
            }
            __builtin_amdgcn_wave_barrier();
            __builtin_amdgcn_s_waitcnt(0xc07f); // lgkmcnt(0): the wave's LDS writes are visible
            const T(*M)[PW + 1] = sS[wid][up ? 0 : 1];
            T x[PW];
#pragma unroll
            for (int i = 0; i < PW; ++i) x[i] = (i == j) ? one_of(Sx::zero()) : Sx::zero();
#pragma unroll
            for (int i = PW - 1; i >= 0; --i) {
                // (bitwise masks, no select on `up`: a select let the compiler split
                // the whole unrolled sweep in two and spill)
                const T d = keep_if(up & (i < pw), sR[wid][p0 + i]) + keep_if(!up, one_of(Sx::zero()));
                x[i] = Sx::mul(x[i], d);
#pragma unroll
                for (int k = 0; k < i; ++k) x[k] = Sx::fms(x[k], M[k][i], x[i]);
            }
#pragma unroll
            for (int i = 0; i < PW; ++i)
                out[(int64_t)p * PW * PW + i * PW + j] = (i <= j && j < pw) ? x[i] : Sx::zero();
            __builtin_amdgcn_wave_barrier();
        }
    }
}

} // namespace slu

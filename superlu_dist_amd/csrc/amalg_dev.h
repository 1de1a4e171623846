// Device relayout between the caller's LUstruct layout and the coarse
// (amalgamated) one the plan factors (csrc/amalg.h).  Included by engine.hip.
// Both directions are HBM-bound copies: every original value is read once and
// written once (expand; the coarse arrays are zeroed first), or the reverse
// (compress: only the positions the caller stores are read back).
#pragma once
#include <hip/hip_runtime.h>

#include "amalg.h"

namespace slu {

// a column range [c0, c1) of one original L block column
struct LColX {
    int64_t src, dst, map;
    int32_t nsupr, c0, c1, ld2;
};

// dir 0: caller -> coarse, 1: coarse -> caller
template <typename T>
__global__ void __launch_bounds__(256) k_amalg_l(const LColX *items, const int32_t *lrow, T *oL,
                                                 T *mL, int dir) {
    const LColX x = items[blockIdx.x];
    for (int c = x.c0; c < x.c1; ++c) {
        T *o = oL + x.src + (int64_t)c * x.nsupr;
        T *m = mL + x.dst + (int64_t)c * x.ld2;
        for (int i = threadIdx.x; i < x.nsupr; i += 256) {
            const int32_t r = lrow[x.map + i];
            if (dir == 0) m[r] = o[i];
            else o[i] = m[r];
        }
    }
}

// One wave per original U block row, 64 columns at a time: the lanes fetch
// the columns' descriptors and coarse destinations in parallel and prefix-sum
// the segment lengths (into LDS), then sweep the chunk's values -- contiguous
// in the caller's layout -- one element per lane, each finding its column by
// a binary search over the 64 prefix sums.  No dependent global load per
// column (a column-at-a-time loop was 41 ms at 100^3, three load round trips
// per column of the wide rows).
template <typename T>
__global__ void __launch_bounds__(256) k_amalg_u(const Amalg::URowX *rows, int nrows,
                                                 const int32_t *ucol, const int64_t *D, int64_t DL0,
                                                 T *oU, T *mL, T *mU, int dir) {
    __shared__ int s_incl[4][64];
    __shared__ int64_t s_dst[4][64]; // coarse offset of the column's first value, kind in bit 62
    const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int r = blockIdx.x * 4 + w;
    if (r >= nrows) return; // (whole waves: no barrier below)
    const Amalg::URowX R = rows[r];
    int64_t src = R.src;
    const int2 *uc = (const int2 *)ucol + R.c0;
    for (int b = 0; b < R.nc; b += 64) {
        const int c = b + lane;
        int len = 0;
        int64_t dst = 0;
        if (c < R.nc) {
            const int2 e = uc[c];
            len = R.end - e.y;
            dst = D[e.x] + e.y;
            if (e.x >= DL0) dst |= (int64_t)1 << 62;
        }
        int incl = len;
#pragma unroll
        for (int d = 1; d < 64; d <<= 1) {
            const int v = __shfl_up(incl, d);
            if (lane >= d) incl += v;
        }
        s_incl[w][lane] = incl;
        s_dst[w][lane] = dst;
        const int total = __shfl(incl, 63);
        __builtin_amdgcn_wave_barrier();
        for (int t = lane; t < total; t += 64) {
            int lo = 0, hi = 63; // first column j with incl[j] > t
            while (lo < hi) {
                const int mid = (lo + hi) >> 1;
                if (s_incl[w][mid] > t) hi = mid;
                else lo = mid + 1;
            }
            const int start = lo ? s_incl[w][lo - 1] : 0;
            const int64_t d = s_dst[w][lo];
            T *m = ((d >> 62) & 1 ? mL : mU) + (d & (((int64_t)1 << 62) - 1)) + (t - start);
            if (dir == 0) *m = oU[src + t];
            else oU[src + t] = *m;
        }
        src += total;
        __builtin_amdgcn_wave_barrier();
    }
}

} // namespace slu

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

// one wave per original U block row: a wide row (w >= 16) column by column
// with the lanes over the segment; a narrow one (every segment shorter than
// 16) with the lanes over its columns, each lane's source offset from a wave
// prefix sum of the segment lengths
template <typename T>
__global__ void __launch_bounds__(256) k_amalg_u(const Amalg::URowX *rows, int nrows,
                                                 const int32_t *ucol, const int64_t *D, int64_t DL0,
                                                 T *oU, T *mL, T *mU, int dir) {
    const int r = blockIdx.x * 4 + (threadIdx.x >> 6), lane = threadIdx.x & 63;
    if (r >= nrows) return;
    const Amalg::URowX R = rows[r];
    int64_t src = R.src;
    const int2 *uc = (const int2 *)ucol + R.c0;
    if (R.w >= 16) {
        for (int c = 0; c < R.nc; ++c) {
            const int2 e = uc[c];
            const int len = R.end - e.y;
            T *m = (e.x >= DL0 ? mL : mU) + D[e.x] + e.y;
            for (int i = lane; i < len; i += 64) {
                if (dir == 0) m[i] = oU[src + i];
                else oU[src + i] = m[i];
            }
            src += len;
        }
        return;
    }
    for (int b = 0; b < R.nc; b += 64) {
        const int c = b + lane;
        int2 e = make_int2(0, R.end);
        if (c < R.nc) e = uc[c];
        const int len = R.end - e.y;
        int incl = len; // inclusive prefix sum over the wave
#pragma unroll
        for (int d = 1; d < 64; d <<= 1) {
            const int v = __shfl_up(incl, d);
            if (lane >= d) incl += v;
        }
        const int64_t o = src + incl - len;
        if (len > 0) {
            T *m = (e.x >= DL0 ? mL : mU) + D[e.x] + e.y;
            for (int i = 0; i < len; ++i) {
                if (dir == 0) m[i] = oU[o + i];
                else oU[o + i] = m[i];
            }
        }
        src += __shfl(incl, 63);
    }
}

} // namespace slu

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

// one thread per original U block (a, jb): its column segments, in order
template <typename T>
__global__ void __launch_bounds__(256) k_amalg_u(const Amalg::UBlkX *blks, int64_t nb,
                                                 const int32_t *ufst, const int64_t *D, T *oU,
                                                 T *mL, T *mU, int dir) {
    const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (i >= nb) return;
    const Amalg::UBlkX B = blks[i];
    T *M = B.kind ? mL : mU;
    int64_t src = B.src;
    for (int c = 0; c < B.w; ++c) {
        const int32_t f = ufst[B.f0 + c];
        const int len = B.end - f;
        T *m = M + D[B.d0 + c] + f;
        for (int k = 0; k < len; ++k) {
            if (dir == 0) m[k] = oU[src + k];
            else oU[src + k] = m[k];
        }
        src += len;
    }
}

} // namespace slu

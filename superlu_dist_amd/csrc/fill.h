// Device-side value fill of the factor storage from A.
//
// Replaces the numeric part of pddistribute for a repeated factorization with
// the same structure (options->Fact == SamePattern_SameRowPerm,
// SRC/pddistribute.c:545-672): U values are zeroed (:574-583), every L
// position is set from a dense SPA that holds A's column values or zero
// (:591-658).  Here the SPA walk is precomputed once per pattern into one
// destination per nonzero of A (Plan::set_a_pattern), so a refill is a memset
// of the rank's L/U values plus one coalesced pass over A's values -- an
// HBM-bound scatter of nnz(A) elements instead of a PCIe upload of all of
// L and U.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

namespace slu {

constexpr int FILL_THREADS = 256;

// amap[e] = 2*dst for L(:,·) storage, 2*dst + 1 for U storage, -1 when the
// nonzero is not stored on this rank (other process row / column) or is an
// earlier duplicate of the same position (the SPA keeps the last write,
// SRC/pddistribute.c:618,621).
template <typename T>
__global__ void __launch_bounds__(FILL_THREADS)
k_fill_a(const int64_t *__restrict__ amap, const T *__restrict__ a, int64_t nnz,
         T *__restrict__ L, T *__restrict__ U) {
    const int64_t stride = (int64_t)gridDim.x * FILL_THREADS;
    for (int64_t e = (int64_t)blockIdx.x * FILL_THREADS + threadIdx.x; e < nnz; e += stride) {
        const int64_t m = amap[e];
        if (m < 0) continue;
        const T v = a[e];
        if (m & 1) U[m >> 1] = v;
        else L[m >> 1] = v;
    }
}

} // namespace slu

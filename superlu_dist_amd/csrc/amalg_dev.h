// Device relayout between the caller's LUstruct layout and the coarse
// (amalgamated) one the plan factors (csrc/amalg.h).  Included by engine.hip.
// Both directions are HBM-bound copies: every original value is read once and
// written once (expand; the coarse arrays are zeroed first), or the reverse
// (compress: only the positions the caller stores are read back).
#pragma once
#include <hip/hip_runtime.h>

#include "amalg.h"

namespace slu {


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

// One wave per chunk of <= 64 non-empty columns of an original U block row (the
// engine splits the rows; the top separators' rows hold thousands of columns
// of segments up to 256 long).  The lanes fetch the chunk's column
// descriptors and coarse destinations at once and prefix-sum the segment
// lengths.  A chunk of short segments (<= 256 values) is then swept one value
// per lane, each lane finding its column by binary search over the prefix
// sums in LDS; a chunk of long segments goes column by column with the lanes
// over the segment (coalesced on both sides).

template <typename T>
__global__ void __launch_bounds__(256) k_amalg_u(const UChunk *chunks, int nchunks,
                                                 const int32_t *ucd, const uint16_t *ucl, const int64_t *D,
                                                 int64_t DL0, T *oU, T *mL, T *mU, int dir) {
    __shared__ int s_incl[4][64];
    __shared__ int64_t s_dst[4][64]; // coarse offset of the column's first value, kind in bit 62
    const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int r = blockIdx.x * 4 + w;
    if (r >= nchunks) return; // (whole waves: no barrier below)
    const UChunk C = chunks[r];
    constexpr int64_t KIND = (int64_t)1 << 62;
    int len = 0;
    int64_t dst = 0;
    if (lane < C.nc) {
        const int32_t d = ucd[C.c0 + lane];
        len = (int)ucl[C.c0 + lane] + 1;
        dst = D[d] + C.end - len;
        if (d >= DL0) dst |= KIND;
    }
    int incl = len;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
        const int v = __shfl_up(incl, d);
        if (lane >= d) incl += v;
    }
    const int total = __shfl(incl, 63);
    if (total <= 256) {
        s_incl[w][lane] = incl;
        s_dst[w][lane] = dst;
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
            T *m = (d & KIND ? mL : mU) + (d & (KIND - 1)) + (t - start);
            if (dir == 0) *m = oU[C.src + t];
            else oU[C.src + t] = *m;
        }
        return;
    }
    const int excl = incl - len;
    for (int j = 0; j < C.nc; ++j) {
        const int lj = __shfl(len, j);
        if (lj == 0) continue;
        const int64_t off = C.src + __shfl(excl, j), d = __shfl(dst, j);
        T *m = (d & KIND ? mL : mU) + (d & (KIND - 1));
        for (int i = lane; i < lj; i += 64) {
            if (dir == 0) m[i] = oU[off + i];
            else oU[off + i] = m[i];
        }
    }
}

} // namespace slu

namespace slu {

// Contiguous range copies (GaSpan), one wave per chunk of <= 64 ranges:
// dir 0 b[dst + i] = a[src + i], dir 1 the reverse.  Short chunks (<= 256
// values) go one value per lane (binary search over the prefix sums), long
// ones range by range with the lanes over the values.  The grid plan's
// pack of the caller's U blocks into the send buffer (and its reverse).
template <typename T>
__global__ void __launch_bounds__(256) k_ranges(const GaSpan *spans, int nspans, T *a, T *b, int dir) {
    __shared__ int64_t s_incl[4][64], s_src[4][64], s_dst[4][64];
    const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int64_t c0 = ((int64_t)blockIdx.x * 4 + w) * 64;
    if (c0 >= nspans) return; // (whole waves: no barrier below)
    const int nc = (int)min((int64_t)64, (int64_t)nspans - c0);
    GaSpan sp{0, 0, 0};
    if (lane < nc) sp = spans[c0 + lane];
    int64_t incl = sp.len;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
        const int64_t v = __shfl_up(incl, d);
        if (lane >= d) incl += v;
    }
    const int64_t total = __shfl(incl, 63);
    if (total <= 256) {
        s_incl[w][lane] = incl;
        s_src[w][lane] = sp.src;
        s_dst[w][lane] = sp.dst;
        __builtin_amdgcn_wave_barrier();
        for (int t = lane; t < total; t += 64) {
            int lo = 0, hi = 63;
            while (lo < hi) {
                const int mid = (lo + hi) >> 1;
                if (s_incl[w][mid] > t) hi = mid;
                else lo = mid + 1;
            }
            const int64_t o = t - (lo ? s_incl[w][lo - 1] : 0);
            const int64_t s = s_src[w][lo] + o, d = s_dst[w][lo] + o;
            if (dir == 0) b[d] = a[s];
            else a[s] = b[d];
        }
        return;
    }
    for (int j = 0; j < nc; ++j) {
        const int64_t s = __shfl(sp.src, j), d = __shfl(sp.dst, j), len = __shfl(sp.len, j);
        for (int64_t i = lane; i < len; i += 64) {
            if (dir == 0) b[d + i] = a[s + i];
            else a[s + i] = b[d + i];
        }
    }
}

} // namespace slu

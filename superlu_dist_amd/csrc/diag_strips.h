// Multi-workgroup diagonal-block LU for the levels near the root of the
// elimination tree, where a level holds one or a few wide supernodes and the
// diagonal LU -> TRSM -> Schur chain of every level is the critical path
// (DESIGN §5).  Included by engine.hip after kernels.h.
//
// k_diag_lu_f factors a <= 256 x 256 block on ONE workgroup: eight 32-column
// panels one after the other, each with a serial 32 x 32 register LU, two
// serial triangular inverses and a trailing update of the whole remaining
// block through that CU (365 us at w = 256, profiles/r03_diag_micro_phases.txt).
// Here the block is cut into column strips of 32 and strip q is owned by its
// own workgroup, which keeps the strip (all w rows) in LDS from start to end:
//
//   for p < q:  wait for strip p's flag; read its L part (rows 32p.., the
//               unit-lower L_pp and L21_p below it) and L_pp^{-1};
//               U_pq = L_pp^{-1} A_pq (MFMA), A(32p+32.., q) -= L21_p U_pq;
//   own panel:  unblocked right-looking LU of the strip's rows 32q.. (all
//               rows below the diagonal at once, one barrier per column,
//               SRC/pdgstrf2.c:213-269 semantics: tiny-pivot replacement,
//               reciprocal scaling, a zero pivot leaves its column unscaled
//               and sets info), then U_qq^{-1} and L_qq^{-1} by 8 x 8 blocks;
//   publish:    the strip and the two inverses (the TRSMs' dinv blocks) with
//               write-through stores, then the strip's flag.
//
// The critical path per panel is the next strip's update with this panel
// plus its own panel LU; the other strips apply earlier panels meanwhile.
// Hand-off protocol (MI355X_MICROARCH.md, inter-workgroup visibility, first
// row of the sc1 table): every payload byte is stored and loaded with sc1
// (agent-scope relaxed atomics, 8 / 4 bytes), every storing wave waits for
// its stores, a workgroup barrier, then one lane stores the flag (sc1); the
// consumer's lane 0 polls the flag with sc1 loads, a workgroup barrier
// releases the other waves.
//
// Placement: the strips of item i are blocks i % 8 + 8 s + 64 (i / 8), so
// under the observed round-robin dealing they share one XCD (its L2 then
// serves the hand-offs; placement is never needed for correctness).  A block
// only waits for lower-numbered blocks of its own item, dispatched before it.
// Every wait is bounded: after ~1 s the block records an error and returns,
// so the grid always drains (the engine then fails the factorization).
#pragma once
#include <hip/hip_runtime.h>

#include "kernels.h"

namespace slu {

constexpr int DS_THREADS = 256, DS_PW = 32, DS_MAXS = FAST_MAXW / DS_PW;
// a received panel staged 16 elements per thread in flight (32: no faster,
// profiles/r05ds/)
constexpr int DS_TU = 16;

#ifdef SLU_DS_PROBE
// Diagnostics build only (tools/micro/diag_strips_micro.hip): cycles per
// phase summed over all working blocks (thread 0's view): 0 flag wait, 1
// panel read, 2 panel update, 3 own panel LU, 4 inverses, 5 publish.
__device__ long long slu_ds_tp[8];
#define DS_PROBE_START() long long ds_t0 = clock64()
#define DS_PROBE(i)                                                                          \
    do {                                                                                     \
        if (threadIdx.x == 0) {                                                              \
            const long long t = clock64();                                                   \
            atomicAdd((unsigned long long *)&slu_ds_tp[i], (unsigned long long)(t - ds_t0)); \
            ds_t0 = t;                                                                       \
        }                                                                                    \
    } while (0)
#else
#define DS_PROBE_START()
#define DS_PROBE(i)
#endif

template <typename T> struct DsBits;
template <> struct DsBits<double> { using U = unsigned long long; };
template <> struct DsBits<float> { using U = unsigned int; };

// write-through (sc1) store / L1-bypassing (sc1) load of one element
// (global_, never flat_: the sc1 forms replace the acquire only as global /
// buffer instructions)
template <typename T> __device__ __forceinline__ void st_sc1(T *p, T v) {
    using U = typename DsBits<T>::U;
    U u;
    __builtin_memcpy(&u, &v, sizeof(T));
    __hip_atomic_store((__attribute__((address_space(1))) U *)p, u, __ATOMIC_RELAXED,
                       __HIP_MEMORY_SCOPE_AGENT);
}
template <typename T> __device__ __forceinline__ T ld_sc1(const T *p) {
    using U = typename DsBits<T>::U;
    const U u = __hip_atomic_load((__attribute__((address_space(1))) U *)p, __ATOMIC_RELAXED,
                                  __HIP_MEMORY_SCOPE_AGENT);
    T v;
    __builtin_memcpy(&v, &u, sizeof(T));
    return v;
}

// f(integral_constant<int, i>) for i = 0 .. N - 1, unrolled at compile time
template <int N, int I = 0, typename F> __device__ __forceinline__ void ds_unroll(F &&f) {
    if constexpr (I < N) {
        f(std::integral_constant<int, I>{});
        ds_unroll<N, I + 1>(f);
    }
}

// lane 0 of wave 0 waits for *f >= epoch; false (and *err set) on timeout
__device__ __forceinline__ bool ds_wait(const unsigned *f, unsigned epoch, int *err, int *s_ok) {
    if (threadIdx.x == 0) {
        int ok = 1;
        unsigned n = 0;
        while (__hip_atomic_load((const __attribute__((address_space(1))) unsigned *)f, __ATOMIC_RELAXED,
                                 __HIP_MEMORY_SCOPE_AGENT) < epoch) {
            __builtin_amdgcn_s_sleep(2);
            if (++n > (1u << 23)) { // ~1 s
                atomicExch(err, 1);
                ok = 0;
                break;
            }
        }
        *s_ok = ok;
    }
    __syncthreads();
    return *s_ok != 0;
}

// one wave waits for *f >= epoch (every lane loads the same word: a
// uniform loop); false (and *err set) on timeout
__device__ __forceinline__ bool ds_wait_wave(const unsigned *f, unsigned epoch, int *err) {
    unsigned n = 0;
    while (__hip_atomic_load((const __attribute__((address_space(1))) unsigned *)f, __ATOMIC_RELAXED,
                             __HIP_MEMORY_SCOPE_AGENT) < epoch) {
        __builtin_amdgcn_s_sleep(2);
        if (++n > (1u << 23)) { // ~1 s
            if ((threadIdx.x & 63) == 0) atomicExch(err, 1);
            return false;
        }
    }
    return true;
}

// publish: every wave's stores have completed, then one lane sets the flag
__device__ __forceinline__ void ds_publish(unsigned *f, unsigned epoch) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (threadIdx.x == 0)
        __hip_atomic_store((__attribute__((address_space(1))) unsigned *)f, epoch, __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_AGENT);
}

// Two flags per strip (the item's flags are 2 DS_MAXS words: A then B).
// A: the first 64 rows of L21_q and (L_qq^{-1})^T are published -- what the
// next strip's own LU needs; B: all of L21_q.  The strip right of q waits
// for A before its LU and its waves 1-3 for B beside the LU; the strips
// further right wait for B.
constexpr int DS_NFLAGS = 2 * DS_MAXS;

// Block -> (item, strip) of the XCD-grouped layout above; grid = 64 *
// ceil(nitems / 8).
__host__ __device__ inline int ds_grid(int nitems) { return 64 * ((nitems + 7) / 8); }

template <typename T>
__global__ void __launch_bounds__(DS_THREADS, 1) __attribute__((amdgpu_waves_per_eu(1, 1)))
k_diag_strips(const DiagItemF<T> *items, int nitems, unsigned *flags, unsigned epoch, int *err,
              double thresh, int replace_tiny, int *tiny_count, int *zpiv) {
    static_assert(std::is_same<T, double>::value || std::is_same<T, float>::value, "real types");
    constexpr int PW = DS_PW, MW = FAST_MAXW, LD = PW + 1;
    using Sx = S<T>;
    using M = Mma<T>;
    const int b = blockIdx.x, item = (b >> 6) * 8 + (b & 7), q = (b >> 3) & 7;
    if (item >= nitems) return;
    const DiagItemF<T> it = items[item];
    const int w = it.w, ns = (w + PW - 1) / PW;
    if (q >= ns) return;
    const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
    const int ld = it.ld, c0 = q * PW, pw = min(PW, w - c0);
    T *A = it.a;
    unsigned *fl = flags + (size_t)item * DS_NFLAGS, *flB = fl + DS_MAXS;
    const int nb = ns;
    T *dinvU = it.dinv, *dinvLT = it.dinv + (int64_t)nb * PW * PW;

    __shared__ T sS[MW][LD];  // my strip, all w rows
    __shared__ T sP[MW][LD];  // a received panel's L part (rows 32p..)
    __shared__ T sLi[PW][LD]; // L_pp^{-1}; later my L_qq^{-1}
    __shared__ T sTmp[2][16][17]; // the inverses' 16 x 16 products
    __shared__ T sUi[PW][LD]; // my U_qq^{-1}
    __shared__ int s_zp[PW];
    __shared__ T s_rp[PW];
    __shared__ int s_ok;
    DS_PROBE_START();

    // ---- my strip (values of earlier kernels: plain loads)
    stage_loop<DS_THREADS, 4, T>(
        tid, w * PW,
        [&](int e, bool ok) {
            const int r = e % w, c = min(e / w, pw - 1);
            return keep_if(ok & (e / w < pw), gld(A + min(r, w - 1) + (int64_t)(c0 + c) * ld));
        },
        [&](int e, T v) { sS[e % w][e / w] = v; });
    // rows w .. c0 + 32 (the last strip's diagonal block past pw) read as
    // zeros by the inverses below
    for (int e = tid; e < (c0 + PW - w) * PW; e += DS_THREADS) sS[w + e / PW][e % PW] = Sx::zero();
    __syncthreads();

    // A(r0 + 32 + [lo, hi), strip) -= L21 U_pq (sP rows 32 + .., U_pq in sS
    // rows r0..): 16 x 16 fragments (lo a multiple of 16), two chains per
    // wave, on waves w0, w0 + 1, .. (wn of them)
    auto trail = [&](int r0, int lo, int hi, int w0, int wn) {
        const int nfr = hi > lo ? (hi - lo + 15) / 16 : 0, nf = 2 * nfr;
        for (int f0 = 2 * (wv - w0); f0 < nf; f0 += 2 * wn) {
            typename M::acc_t acc[2] = {M::zero(), M::zero()};
#pragma unroll
            for (int ks = 0; ks < PW; ks += M::KSTEP) {
                const int k = ks + (lane >> 4);
#pragma unroll
                for (int u = 0; u < 2; ++u) {
                    const int f = min(f0 + u, nf - 1), fr = f >> 1, fc = f & 1;
                    const int r = lo + fr * 16 + (lane & 15);
                    M::step(acc[u], keep_if(r < hi, sP[PW + min(r, hi - 1)][k]),
                            sS[r0 + k][fc * 16 + (lane & 15)]);
                }
            }
#pragma unroll
            for (int u = 0; u < 2; ++u) {
                const int f = f0 + u, fr = f >> 1, fc = f & 1;
                if (f < nf)
#pragma unroll
                    for (int i = 0; i < 4; ++i) {
                        const int r = lo + fr * 16 + M::row(lane, i);
                        if (r < hi) {
                            T &d = sS[r0 + PW + r][fc * 16 + (lane & 15)];
                            d = Sx::sub(d, M::get(acc[u], i));
                        }
                    }
            }
        }
    };
    // trail() of rows [lo, hi) on waves w0.. (wn of them), each wave first
    // loading the rows of L21 (sP rows 32 + ..) its fragments read, from
    // the published strip r0 (wave-private rows: no barrier)
    auto trail_rest = [&](int r0, int lo, int hi, int w0, int wn) {
        const int nfr = hi > lo ? (hi - lo + 15) / 16 : 0;
        // (rows past the first 64 of L21: published with the strip's flag B;
        // on a timeout the error is set and the rows are garbage -- the
        // engine then fails the factorization)
        if (wv - w0 < nfr) (void)ds_wait_wave(flB + r0 / PW, epoch, err);
        for (int fr = wv - w0; fr < nfr; fr += wn) {
            T v[8];
#pragma unroll
            for (int u = 0; u < 8; ++u) {
                const int e = lane + 64 * u, r = lo + fr * 16 + (e & 15), k = e >> 4;
                v[u] = keep_if(r < hi, ld_sc1(A + r0 + PW + min(r, hi - 1) + (int64_t)(r0 + k) * ld));
            }
#pragma unroll
            for (int u = 0; u < 8; ++u) {
                const int e = lane + 64 * u, r = lo + fr * 16 + (e & 15), k = e >> 4;
                sP[PW + r][k] = v[u];
            }
        }
        asm volatile("" ::: "memory"); // (one wave: its LDS accesses complete in order)
        trail(r0, lo, hi, w0, wn);
    };
    // ---- apply the panels of the strips to my left, in order
    for (int p = 0; p < q; ++p) {
        if (!ds_wait((p + 1 == q ? fl : flB) + p, epoch, err, &s_ok)) return;
        const int r0 = p * PW, nr = w - r0;
        DS_PROBE(0);
        // only L21_p (rows r0 + 32 ..): L_pp enters through its inverse.  The
        // last panel before my own LU: only its first 64 rows now (the rows
        // my LU reads); waves 1-3 load the rest beside the LU, each the rows
        // it updates (trail_rest below)
        const int nb21 = nr - PW, rb = r0 + PW;
        const int nst = p + 1 == q ? min(64, nb21) : nb21;
        if (nst > 0)
            stage_loop<DS_THREADS, DS_TU, T>(
                tid, nst * PW,
                [&](int e, bool ok) {
                    const int ee = min(e, nst * PW - 1);
                    return keep_if(ok, ld_sc1(A + rb + ee % nst + (int64_t)(r0 + ee / nst) * ld));
                },
                [&](int e, T v) { sP[PW + e % nst][e / nst] = v; });
        stage_loop<DS_THREADS, 4, T>( // dinvLT: [b][a] = Linv[a][b]
            tid, PW * PW, [&](int e, bool ok) { return keep_if(ok, ld_sc1(dinvLT + (int64_t)p * PW * PW + min(e, PW * PW - 1))); },
            [&](int e, T v) { sLi[e % PW][e / PW] = v; });
        __syncthreads();
        DS_PROBE(1);
        // U_pq = L_pp^{-1} A(r0:r0+32, strip): 2 x 2 fragments, one per wave
        {
            const int fr = wv >> 1, fc = wv & 1;
            typename M::acc_t acc = M::zero();
#pragma unroll
            for (int ks = 0; ks < PW; ks += M::KSTEP) {
                const int k = ks + (lane >> 4);
                M::step(acc, sLi[fr * 16 + (lane & 15)][k], sS[r0 + k][fc * 16 + (lane & 15)]);
            }
            __syncthreads(); // all reads of rows r0.. before they are overwritten
#pragma unroll
            for (int i = 0; i < 4; ++i)
                sS[r0 + fr * 16 + M::row(lane, i)][fc * 16 + (lane & 15)] = M::get(acc, i);
        }
        __syncthreads();
        // A(r0+32.., strip) -= L21_p U_pq.  The last panel before my own LU
        // updates only the 64 rows the LU reads now; the rest is updated by
        // waves 1-3 beside the LU (below)
        trail(r0, 0, p + 1 == q ? min(64, nr - PW) : nr - PW, 0, 4);
        __syncthreads();
        DS_PROBE(2);
    }

    // ---- my panel: rows c0.. (nrow of them).  Wave 0 factors the top 64
    // (the 32 x 32 diagonal block and 32 rows below it; lane = row, the
    // pivot row through v_readlane: no barrier per column), then waves 1-3
    // eliminate rows 64.. one row per thread against the finished U_qq in
    // LDS (the same per-column semantics, no barrier at all) while wave 0
    // forms U_qq^{-1} / L_qq^{-1} (below).
    const int nrow = w - c0;
    if (wv == 0) {
        T x[PW];
        const bool mine = lane < nrow;
#pragma unroll
        for (int c = 0; c < PW; ++c) x[c] = mine ? sS[c0 + lane][c] : Sx::zero();
        // (tiny-pivot count and the last zero pivot in registers, one atomic
        // each after the loop: no control flow between the columns' steps)
        int ntiny = 0, zlast = 0;
        T rps[PW];
        int zps[PW];
#pragma unroll
        for (int j = 0; j < PW; ++j) {
            rps[j] = Sx::zero();
            zps[j] = 0;
        }
        // one column step (the same per-column semantics for every strip)
        auto lu_step = [&](auto jc) {
            constexpr int j = decltype(jc)::value;
            T piv = rlane(x[j], j);
            const bool tiny = replace_tiny && Sx::abs1(piv) < thresh;
            piv = tiny ? Sx::thresh(piv, thresh) : piv;
            ntiny += tiny;
            const int z = Sx::iszero(piv);
            zlast = z ? it.fcol + c0 + j + 1 : zlast;
            const T rp = z ? Sx::zero() : Sx::recip(piv);
            // a zero pivot leaves the column unscaled (SRC/pdgstrf2.c:246-252)
            const T l = lane > j ? (z ? x[j] : Sx::mul(x[j], rp)) : Sx::zero();
            x[j] = lane > j ? l : (lane == j ? piv : x[j]);
#pragma unroll
            for (int c = j + 1; c < PW; ++c) x[c] = Sx::fms(x[c], l, rlane(x[c], j));
            rps[j] = rp;
            zps[j] = z;
        };
        // full strips (pw = 32): the steps with no branch between them, so the
        // next column's pivot and reciprocal overlap this column's updates
        if (pw == PW)
            ds_unroll<PW>([&](auto jc) { lu_step(jc); });
        else
            ds_unroll<PW>([&](auto jc) {
                if (decltype(jc)::value < pw) lu_step(jc);
            });
        if (lane == 0) {
#pragma unroll
            for (int j = 0; j < PW; ++j) {
                s_rp[j] = rps[j];
                s_zp[j] = zps[j];
            }
        }
        if (lane == 0 && ntiny) atomicAdd(tiny_count, ntiny);
        if (lane == 0 && zlast) atomicMax(&zpiv[it.k], zlast);
        if (mine)
#pragma unroll
            for (int c = 0; c < PW; ++c) sS[c0 + lane][c] = x[c];
        if (lane >= pw && lane < PW) {
            s_rp[lane] = Sx::zero();
            s_zp[lane] = 0;
        }
    } else if (q > 0) {
        trail_rest(c0 - PW, 64, nrow, 1, 3); // the last panel's update of rows c0 + 64 ..
    }
    __syncthreads();
    DS_PROBE(3);
    // ---- the inverses, then the rows below the top 64.
    // (I) wave 0: the four 16 x 16 diagonal blocks of L_qq^{-1} (unit lower,
    // blocks A, C) and U_qq^{-1} (upper, blocks D, F), a quarter-wave each,
    // lane = column: w = e_j; for k: w[k] *= scale_k, w[t] -= M(t, k) w[k] for
    // t > k, with M = L and scale 1, or M(t, k) = U(15 - t, 15 - k) (the block
    // walked from its last row) and scale rp.  Columns >= pw of the strip are
    // zeros (loaded so, kept so by the LU), as are its rows past the block
    // (above); rows / columns >= pw of the inverses are set to zero.
    // (II) the off-diagonal blocks on MFMA: L21^{-1} = -C^{-1} (B A^{-1})
    // (wave 0), U12^{-1} = -D^{-1} (E F^{-1}) (wave 1).
    // (III) rows 64..: X = A U_qq^{-1} on MFMA (all waves).  A zero pivot
    // leaves its column unscaled (SRC/pdgstrf2.c:246-252), which no inverse
    // expresses: such a strip eliminates those rows one per thread instead.
    bool anyz = false;
#pragma unroll
    for (int c = 0; c < PW; ++c) anyz |= s_zp[c] != 0; // (uniform)
    const T *sflat = &sS[0][0];
    if (wv == 0) {
        const int qd = lane >> 4, jj = lane & 15, o = 16 * (qd & 1);
        const bool up = qd >= 2;
        // (an index into the __shared__ array, not a pointer: keeps ds_read)
        const int mb = up ? (c0 + o + 15) * LD + o + 15 : (c0 + o) * LD + o, sg = up ? -1 : 1;
        T v[16];
#pragma unroll
        for (int t = 0; t < 16; ++t) v[t] = (up ? 15 - t : t) == jj ? one_of(Sx::zero()) : Sx::zero();
#pragma unroll
        for (int k = 0; k < 16; ++k) {
            if (up) v[k] = Sx::mul(v[k], s_rp[o + 15 - k]);
#pragma unroll
            for (int t = k + 1; t < 16; ++t) v[t] = Sx::fms(v[t], sflat[mb + sg * (t * LD + k)], v[k]);
        }
        const bool cok = o + jj < pw;
#pragma unroll
        for (int t = 0; t < 16; ++t) {
            const int r = o + (up ? 15 - t : t);
            const T val = (cok & (r < pw)) ? v[t] : Sx::zero();
            if (up) sUi[r][o + jj] = val;
            else sLi[r][o + jj] = val;
        }
#pragma unroll
        for (int t = 0; t < 4; ++t) { // the structural zero blocks
            const int e = lane + 64 * t, r = e >> 4, c = e & 15;
            sLi[r][16 + c] = Sx::zero();
            sUi[16 + r][c] = Sx::zero();
        }
    }
    __syncthreads();
    if (wv < 2) {
        // wave 0: T = B A^{-1}, L21^{-1} = -C^{-1} T; wave 1: T = E F^{-1},
        // U12^{-1} = -D^{-1} T (one 16 x 16 x 16 product each, through sTmp)
        const bool ul = wv == 0;
        typename M::acc_t acc = M::zero();
#pragma unroll
        for (int ks = 0; ks < 16; ks += M::KSTEP) {
            const int k = ks + (lane >> 4), r = lane & 15;
            const T a = ul ? sS[c0 + 16 + r][k] : sS[c0 + r][16 + k];
            const T b = ul ? sLi[k][r] : sUi[16 + k][16 + r];
            M::step(acc, a, b);
        }
#pragma unroll
        for (int i = 0; i < 4; ++i) sTmp[wv][M::row(lane, i)][lane & 15] = M::get(acc, i);
        asm volatile("" ::: "memory"); // (one wave: its LDS accesses complete in order)
        acc = M::zero();
#pragma unroll
        for (int ks = 0; ks < 16; ks += M::KSTEP) {
            const int k = ks + (lane >> 4), r = lane & 15;
            const T a = ul ? sLi[16 + r][16 + k] : sUi[r][k];
            M::step(acc, a, sTmp[wv][k][r]);
        }
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const int r = M::row(lane, i), c = lane & 15;
            if (ul) sLi[16 + r][c] = Sx::neg(M::get(acc, i));
            else sUi[r][16 + c] = Sx::neg(M::get(acc, i));
        }
    }
    __syncthreads();
    // ---- (III) rows 64 .. nrow - 1 and the publication of L21_q: first
    // rows 64-95 (the first fragment of every wave) and L21_q's first 64 rows
    // with (L_qq^{-1})^T under flag A, then the rest under flag B.  (16 x 16
    // fragments, all reads of a part before a barrier, its writes after it:
    // a row block's two column halves are on two waves.)
    const int r1 = c0 + PW, n21 = w - r1;
    auto store21 = [&](int a, int b) { // L21_q rows [a, b) (rows of L21, from r1)
        const int nn = b - a;
        for (int e = tid; e < nn * pw; e += DS_THREADS) {
            const int r = r1 + a + e % nn, c = e / nn;
            st_sc1(A + r + (int64_t)(c0 + c) * ld, sS[r][c]);
        }
    };
    const int nA = min(64, max(n21, 0)); // L21 rows under flag A
    if (!anyz) {
        const int nb = nrow - 64, nfr = nb > 0 ? (nb + 15) / 16 : 0, nf = 2 * nfr;
        constexpr int FMAX = (MW - 64) / 16 * 2 / 4; // fragments per wave
        auto part = [&](int u0, int u1) {
            typename M::acc_t acc[FMAX];
#pragma unroll
            for (int u = 0; u < FMAX; ++u) {
                acc[u] = M::zero();
                const int f = wv + 4 * u;
                if (u >= u0 && u < u1 && f < nf) {
                    const int fr = f >> 1, fc = f & 1, r = fr * 16 + (lane & 15);
#pragma unroll
                    for (int ks = 0; ks < PW; ks += M::KSTEP) {
                        const int k = ks + (lane >> 4);
                        M::step(acc[u], keep_if(r < nb, sS[c0 + 64 + min(r, nb - 1)][k]),
                                sUi[k][fc * 16 + (lane & 15)]);
                    }
                }
            }
            __syncthreads();
#pragma unroll
            for (int u = 0; u < FMAX; ++u) {
                const int f = wv + 4 * u;
                if (u >= u0 && u < u1 && f < nf) {
                    const int fr = f >> 1, fc = f & 1;
#pragma unroll
                    for (int i = 0; i < 4; ++i) {
                        const int r = fr * 16 + M::row(lane, i);
                        if (r < nb) sS[c0 + 64 + r][fc * 16 + (lane & 15)] = M::get(acc[u], i);
                    }
                }
            }
            __syncthreads();
        };
        part(0, 1); // rows 64 .. 95
        DS_PROBE(4);
        store21(0, nA);
        for (int e = tid; e < PW * PW; e += DS_THREADS) {
            const int i = e / PW, jj = e % PW;
            st_sc1(dinvLT + (int64_t)q * PW * PW + e, sLi[jj][i]);
        }
        ds_publish(fl + q, epoch);
        part(1, FMAX); // rows 96 ..
        store21(nA, n21);
        ds_publish(flB + q, epoch);
    } else {
        if (wv > 0) { // rows 64.., thread per row
            const int i = tid;
            if (i < nrow) {
                T x[PW];
#pragma unroll
                for (int c = 0; c < PW; ++c) x[c] = sS[c0 + i][c];
#pragma unroll
                for (int j = 0; j < PW; ++j) {
                    if (j < pw) {
                        const T l = s_zp[j] ? x[j] : Sx::mul(x[j], s_rp[j]);
                        x[j] = l;
#pragma unroll
                        for (int c = j + 1; c < PW; ++c) x[c] = Sx::fms(x[c], l, sS[c0 + j][c]);
                    }
                }
#pragma unroll
                for (int c = 0; c < PW; ++c) sS[c0 + i][c] = x[c];
            }
        }
        __syncthreads();
        DS_PROBE(4);
        store21(0, max(n21, 0));
        for (int e = tid; e < PW * PW; e += DS_THREADS) {
            const int i = e / PW, jj = e % PW;
            st_sc1(dinvLT + (int64_t)q * PW * PW + e, sLi[jj][i]);
        }
        ds_publish(fl + q, epoch);
        ds_publish(flB + q, epoch);
    }
    DS_PROBE(5);
    // ---- then the rest of the strip (rows < c0 + 32) and U_qq^{-1}
    // (row-major), which only the TRSMs after this kernel read
    {
        const int r1c = min(r1, w);
        for (int e = tid; e < r1c * pw; e += DS_THREADS) {
            const int r = e % r1c, c = e / r1c;
            A[r + (int64_t)(c0 + c) * ld] = sS[r][c];
        }
        for (int e = tid; e < PW * PW; e += DS_THREADS) dinvU[(int64_t)q * PW * PW + e] = sUi[e / PW][e % PW];
    }
}

} // namespace slu

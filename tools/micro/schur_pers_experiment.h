// Persistent form of k_schur_big (fp64, SLU_SB_PERSIST=1): each workgroup
// takes tiles from a per-launch counter until the launch's tiles are gone,
// and fetches the next tile's descriptor and tables while it is still
// scattering the current one.
//
// Why: per-tile phase stamps put a full 128x128x256 tile at
// ~198 k cycles, 20 k of them in the prologue -- four dependent global rounds
// (tile item -> KInfo -> row / column tables, U segment offsets, destination
// records -> the first stage's operands) before the first MFMA.  A fresh
// workgroup per tile pays them all with the MFMA pipe fed only by the CU's
// other workgroup.  Here:
//   * the next tile index is claimed (one atomic) when the K loop starts and
//     read back after it;
//   * the next descriptor and KInfo come in as scalar loads at the start of
//     the epilogue (constant address space: SGPRs, no VGPRs);
//   * the next tile's row / column tables, U segment offsets and destination
//     records go straight from global memory into LDS (global_load_lds, no
//     VGPRs either) during the first epilogue pass, and are waited for at the
//     end of the second.
// So a tile after the first starts with one dependent round (its first K
// stage).  The arithmetic, the destination tables and the scatter are
// k_schur_big's: the factors are the same bit for bit.
#pragma once

namespace slu {

// dword loads through the constant address space (the kernel never writes
// the descriptors): scalar loads into SGPRs
__device__ __forceinline__ int sload(const int *p) { return *(const __attribute__((address_space(4))) int *)p; }
template <typename X> __device__ __forceinline__ X sload(const X *p) {
    static_assert(sizeof(X) % 4 == 0, "dword structs");
    X x;
    int *d = (int *)&x;
#pragma unroll
    for (int i = 0; i < (int)(sizeof(X) / 4); ++i) d[i] = __builtin_amdgcn_readfirstlane(sload((const int *)p + i));
    return x;
}
// one dword per lane, global -> LDS at the wave's base l + 4 * lane (l must
// be the same for every active lane)
__device__ __forceinline__ void lds_dma4(const void *g, void *l) {
    __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void *)g,
                                     (__attribute__((address_space(3))) void *)l, 4, 0, 0);
}

template <typename T>
__global__ void __launch_bounds__(BigCfg<T>::THREADS, BigCfg<T>::MINW)
k_schur_pers(const TileItem *tiles, const KInfo<T> *kinfo, T *Lval, T *Uval, const LBlk *lblk,
             const int *lmap, const UBlk *ublk, const int64_t *ucol_voff, const int *ucol_fst,
             int ntiles, unsigned *tctr, int prefetch) {
    static_assert(std::is_same<T, double>::value, "k_schur_pers: fp64 tiles only");
    using Sx = S<T>;
    using M = Mma<T>;
    constexpr int SB_BN = BigCfg<T>::BN, SB_BK = BigCfg<T>::BK;
    constexpr int SB_THREADS = BigCfg<T>::THREADS;
    constexpr int WN = BigCfg<T>::WN;
    constexpr int FM = 2, FN = BigCfg<T>::FN;
    constexpr int PASSW = BigCfg<T>::PASSW;
    constexpr int LDS_A = SB_BM + 4, LDS_B = SB_BN + 4;
    constexpr int STAGE = SB_BK * LDS_A + SB_BK * LDS_B;
    constexpr int CLD = SB_BM + 1;
    constexpr int AE = SB_BM * SB_BK / SB_THREADS, BE = SB_BN * SB_BK / SB_THREADS;
    static_assert(AE == 4 && BE == 4 && SB_BN == SB_BM && SB_BM == 128 && SB_THREADS == 512, "fp64 tile");
    static_assert(WN * 16 * FN == SB_BN && (SB_THREADS / 64 / WN) * 16 * FM == SB_BM, "waves");
    constexpr int CPN = SB_TB * SB_BN, RLN = SB_TB * SB_BM;
    constexpr int SMEM = 2 * STAGE;
    static_assert(PASSW * CLD <= SMEM, "C staging must fit in the stage buffers");
    static_assert(SB_TB * SB_TB == 16, "destination records: 16");
    __shared__ __attribute__((aligned(16))) T smem[SMEM];
    __shared__ int s_rg[SB_BM], s_ra[SB_BM], s_cg[SB_BN], s_cb[SB_BN];
    __shared__ int s_ct0[SB_BN];     // per U column: segment start
    __shared__ int64_t s_cvo[SB_BN]; // per U column: segment value offset
    __shared__ int64_t s_dbm[32];    // destination records: base [0, 16), mb [16, 32)
    __shared__ int s_dld[16];        //   and ld
    __shared__ int s_next;
    __shared__ int64_t s_cp[CPN]; // [row block][column] column parts
    __shared__ int s_rl[RLN];     // [column block][row] lmap positions
    int64_t *const s_db = s_dbm, *const s_dmb = s_dbm + 16;

    const int tid = threadIdx.x;
    if (tid == 0) s_next = (int)atomicAdd(tctr, 1u);
    __syncthreads();
    int t = __builtin_amdgcn_readfirstlane(s_next);
    if (t >= ntiles) return;
    TileItem ti = sload(tiles + t);
    KInfo<T> ki = sload(kinfo + ti.kslot);
    bool meta = false; // tables of tile t already in LDS (prefetched)

    for (;;) {
        // the thread's indices are derived anew in every tile (an opaque zero
        // keeps the compiler from hoisting them out of the tile loop, where
        // they would stay live through the epilogue)
        int oz;
        asm volatile("s_mov_b32 %0, 0" : "=s"(oz));
        const int tix = tid + oz, lane = tix & 63, wid = tix >> 6;
        const int wr = wid / WN, wc = wid % WN;
        // A: rows ar, ar + 1, k = ak + 8s (s < 2); B: column bc, k = bk..bk+3
        const int ar = 2 * (tix & 63), ak = tix >> 6;
        const int bc = tix / (SB_BK / BE), bk = (tix % (SB_BK / BE)) * BE;
        const int row0 = ti.tm * SB_BM, col0 = ti.tn * SB_BN;
        const int mrows = min(SB_BM, ki.m - row0), ncols = min(SB_BN, ki.n - col0);
        if (!meta) {
            if (tix < SB_BM) {
                s_rg[tix] = tix < mrows ? ki.rg[row0 + tix] : 0;
                s_ra[tix] = tix < mrows ? ki.ra[row0 + tix] : 0;
            } else if (tix < SB_BM + SB_BN) {
                const int c = tix - SB_BM;
                s_cg[c] = c < ncols ? ki.cg[col0 + c] : 0;
                s_cb[c] = c < ncols ? ki.cb[col0 + c] : 0;
            } else if (tix < SB_BM + 2 * SB_BN) {
                const int c = tix - SB_BM - SB_BN, cc = col0 + (c < ncols ? c : 0);
                s_ct0[c] = ki.ct0[cc];
                s_cvo[c] = ki.cvoff[cc];
            }
            __syncthreads();
        }
        // (wave-uniform: readfirstlane keeps them, and the branches on them, scalar)
        const int a0 = __builtin_amdgcn_readfirstlane(s_ra[0]), b0 = __builtin_amdgcn_readfirstlane(s_cb[0]);
        const int NA = __builtin_amdgcn_readfirstlane(s_ra[mrows - 1]) - a0 + 1;
        const int NB = __builtin_amdgcn_readfirstlane(s_cb[ncols - 1]) - b0 + 1;
        const bool tbl = NA <= SB_TB && NB <= SB_TB;
        if (!meta && tbl && tix < 16) {
            const int al = tix / SB_TB, bl = tix % SB_TB;
            DRec d{0, 0, -1, 0};
            if (al < NA && bl < NB) d = ki.prec[(int64_t)(a0 + al) * ki.nub + b0 + bl];
            s_db[tix] = d.base;
            s_dmb[tix] = d.mb;
            s_dld[tix] = d.ld;
        }
        const T *ap = ki.a + row0 + ar;
        const bool bvalid = bc < ncols;
        const int bt0 = s_ct0[bc];
        const T *ub = ki.ubase + s_cvo[bc] - bt0;
        const int tlast = ki.kmin + ki.kw - 1;
        T ra[AE], rb[BE];
        auto gload = [&](int k0) {
#pragma unroll
            for (int s = 0; s < 2; ++s) {
                const int kk = k0 + ak + 8 * s;
                gld2(ap + (int64_t)(ki.kmin + min(kk, ki.kw - 1)) * ki.lda, ra[2 * s], ra[2 * s + 1]);
            }
            gld4(ub + ki.kmin + k0 + bk, rb);
        };
        auto lstore = [&](int buf, int k0) {
            T *sA = smem + buf * STAGE, *sB = sA + SB_BK * LDS_A;
#pragma unroll
            for (int s = 0; s < 2; ++s) {
                const bool okk = k0 + ak + 8 * s < ki.kw;
                typedef double d2 __attribute__((ext_vector_type(2)));
                *(d2 *)&sA[(ak + 8 * s) * LDS_A + ar] =
                    d2{keep_if(okk & (ar < mrows), ra[2 * s]), keep_if(okk & (ar + 1 < mrows), ra[2 * s + 1])};
            }
#pragma unroll
            for (int s = 0; s < BE; ++s) {
                const int tt = ki.kmin + k0 + bk + s;
                sB[(bk + s) * LDS_B + bc] = keep_if(bvalid & (tt <= tlast) & (tt >= bt0), rb[s]);
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
        // claim the next tile now; its index is read after the K loop
        unsigned claim = 0;
        if (tix == 0) claim = atomicAdd(tctr, 1u);
        auto mfma_stage = [&](int st) {
            const T *sA = smem + (st & 1) * STAGE, *sB = sA + SB_BK * LDS_A;
#pragma unroll
            for (int ks = 0; ks < SB_BK; ks += M::KSTEP) {
                const int kl = ks + (lane >> 4);
                T av[FM], bv[FN];
#pragma unroll
                for (int f = 0; f < FM; ++f) av[f] = sA[kl * LDS_A + wr * (16 * FM) + f * 16 + (lane & 15)];
#pragma unroll
                for (int f = 0; f < FN; ++f) bv[f] = sB[kl * LDS_B + wc * (16 * FN) + f * 16 + (lane & 15)];
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
        // peeled last stage: the destination tables (k_schur_big)
        constexpr int RLT = RLN / SB_THREADS;
        int64_t t_code = 0, t_uv = 0;
        int t_fst = 0, t_rl[RLT];
#pragma unroll
        for (int u = 0; u < RLT; ++u) t_rl[u] = 0;
        if (tbl) {
            if (tix < CPN) {
                const int al = tix / SB_BN, c = tix % SB_BN;
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
                const int e = tix + u * SB_THREADS, bl = e / SB_BM, rr = e % SB_BM;
                if (bl < NB && rr < mrows) {
                    const int rec = (s_ra[rr] - a0) * SB_TB + bl;
                    if (s_dld[rec] >= 0) t_rl[u] = lmap[s_dmb[rec] + s_rg[rr]];
                }
            }
        }
        mfma_stage(nst - 1);
        __syncthreads();
        if (tbl) {
            if (tix < CPN) s_cp[tix] = t_code ? t_code : (t_uv - t_fst) * 8;
#pragma unroll
            for (int u = 0; u < RLT; ++u) s_rl[tix + u * SB_THREADS] = t_rl[u];
        }
        if (tix == 0) s_next = (int)claim;

        // ---- epilogue (k_schur_big's)
        T *sC = smem;
        constexpr int TPR = SB_THREADS / SB_BM, CPT = PASSW / TPR;
        const int r = tix & (SB_BM - 1), q = tix / SB_BM;
        const int gr = s_rg[r], a = s_ra[r];
        auto stage_c = [&](int pass) {
#pragma unroll
            for (int fn = 0; fn < FN; ++fn) {
                const int c0 = wc * 16 * FN + fn * 16;
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
        // the next tile (SGPRs), read once every thread has its gr / a
        int tn = ntiles;
        TileItem ti_n = ti;
        KInfo<T> ki_n = ki;
        auto next_descriptor = [&]() {
            tn = __builtin_amdgcn_readfirstlane(s_next);
            if (tn < ntiles) {
                ti_n = sload(tiles + tn);
                ki_n = sload(kinfo + ti_n.kslot);
            }
        };
        // its tables straight into LDS (fast path only: the slow path reads
        // s_cg / s_cb until its last pass)
        auto next_tables = [&]() {
            const int row0n = ti_n.tm * SB_BM, col0n = ti_n.tn * SB_BN;
            const int mrn = min(SB_BM, ki_n.m - row0n), ncn = min(SB_BN, ki_n.n - col0n);
            const int w = __builtin_amdgcn_readfirstlane(wid), l = lane;
            const int h = (w & 1) * 64 + l; // row / column of wave pair (2v, 2v + 1)
            const int rr = row0n + min(h, mrn - 1), cc = col0n + min(h, ncn - 1);
            const int *src = w < 2 ? ki_n.rg + rr : w < 4 ? ki_n.ra + rr : w < 6 ? ki_n.cg + cc : ki_n.cb + cc;
            int *dst = (w < 2 ? s_rg : w < 4 ? s_ra : w < 6 ? s_cg : s_cb) + (w & 1) * 64;
            lds_dma4(src, dst);
            if (w < 2) {
                lds_dma4(ki_n.ct0 + cc, s_ct0 + (w & 1) * 64);
            } else if (w < 6) { // the int64 offsets as dword pairs
                const int d = (w - 2) * 64 + l, c = col0n + min(d >> 1, ncn - 1);
                lds_dma4((const int *)(ki_n.cvoff + c) + (d & 1), (int *)s_cvo + (w - 2) * 64);
            } else {
                // the next tile's destination records, if it has tables:
                // wave 6 the base / mb dword pairs, wave 7 the ld words
                const int a0n = sload(ki_n.ra + row0n), b0n = sload(ki_n.cb + col0n);
                const int NAn = sload(ki_n.ra + row0n + mrn - 1) - a0n + 1;
                const int NBn = sload(ki_n.cb + col0n + ncn - 1) - b0n + 1;
                if (NAn <= SB_TB && NBn <= SB_TB) {
                    const int rec = w == 6 ? (l & 31) >> 1 : l & 15, al = rec / SB_TB, bl = rec % SB_TB;
                    const bool ok = al < NAn && bl < NBn;
                    const int *pr = (const int *)(ki_n.prec + (int64_t)(a0n + al) * ki_n.nub + b0n + bl);
                    if (w == 6) {
                        if (ok) lds_dma4(pr + (l < 32 ? 0 : 2) + (l & 1), (int *)s_dbm);
                        else ((int *)s_dbm)[l] = 0;
                    } else if (l < 16) {
                        if (ok) lds_dma4(pr + 4, s_dld);
                        else s_dld[l] = -1;
                    }
                }
            }
        };
        bool meta_n = false;
        if (tbl) {
            int rl[SB_TB];
            const int al = a - a0;
#pragma nounroll
            for (int pass = 0; pass < SB_BN / PASSW; ++pass) {
                stage_c(pass);
                __syncthreads();
                if (pass == 0) {
#pragma unroll
                    for (int bl = 0; bl < SB_TB; ++bl) rl[bl] = s_rl[bl * SB_BM + r];
                    next_descriptor();
                    if (prefetch && tn < ntiles) {
                        next_tables();
                        meta_n = true;
                    }
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
                                int rp = gr;
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
            // slow path (tiles over more blocks): per-element table walk
            constexpr int EB = CPT < 4 ? CPT : 4;
            const int *prow = ki.pair + (int64_t)a * ki.nub;
            int lastb = -1, h = 0, ldh = 0;
            int64_t rbase = 0;
#pragma nounroll
            for (int pass = 0; pass < SB_BN / PASSW; ++pass) {
                stage_c(pass);
                __syncthreads();
                if (pass == 0) next_descriptor();
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
                                        rbase = L.colvoff + lmap[L.mapoff + gr - L.frow] - (int64_t)L.fcol * L.ld;
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
        if (tn >= ntiles) break;
        if (meta_n) { // every wave's table DMA has landed, then one barrier
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            __syncthreads();
        }
        t = tn;
        ti = ti_n;
        ki = ki_n;
        meta = meta_n;
    }
}

} // namespace slu

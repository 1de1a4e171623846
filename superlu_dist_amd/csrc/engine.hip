// MI355X numeric factorization engine: plan construction (host), level-
// synchronous execution of the batched kernels in kernels.h, RCCL panel
// exchange for 2D grids, and the engine C API of include/slu_mi355x.h.
//
// Algorithm (what replaces the k-loop of SRC/pdgstrf.c:1108-1756):
//   The supernodal dependency DAG (k -> ib for every block L(ib,k), k -> jb
//   for every block U(k,jb)) is levelled once at plan time.  Supernodes of one
//   level are independent, so for each level the engine launches
//     1. k_diag_lu  on all diagonal blocks of the level owned by this rank,
//     2. (grids) broadcast of the factored diagonal blocks along process rows
//        and columns,
//     3. k_trsm_l / k_trsm_u on every local L / U panel block of the level,
//     4. (grids) broadcast of L panels along process rows and U panels along
//        process columns (RCCL grouped broadcasts),
//     5. k_schur over every (L row tile x U column tile) of every supernode of
//        the level, scattering straight into the destination blocks.
//   The set of updates and the per-element arithmetic are those of the
//   reference; only the order in which independent updates are applied
//   differs (the reference orders them by its static schedule,
//   SRC/dstatic_schedule.c:39).  Two supernodes of one level that update the
//   same destination block use atomic fp adds for those blocks.
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <algorithm>
#include <chrono>
#include <cstring>
#include <memory>
#include <numeric>
#include <string>
#include <vector>

#include "common.h"
#include "kernels.h"
#include "slu_mi355x.h"

using std::vector;

namespace slu {

static thread_local std::string g_last_error;
void set_last_error(const std::string &s) { g_last_error = s; }

template <typename T> struct DevBuf {
    T *p = nullptr;
    size_t n = 0;
    DevBuf() = default;
    DevBuf(const DevBuf &) = delete;
    DevBuf &operator=(const DevBuf &) = delete;
    ~DevBuf() { release(); }
    void release() {
        if (p) (void)hipFree(p);
        p = nullptr;
        n = 0;
    }
    void alloc(size_t cnt) {
        release();
        n = cnt;
        if (cnt) HIPCHK(hipMalloc(&p, cnt * sizeof(T)));
    }
    void upload(const vector<T> &v) {
        alloc(v.size());
        if (!v.empty()) HIPCHK(hipMemcpy(p, v.data(), v.size() * sizeof(T), hipMemcpyHostToDevice));
    }
    size_t bytes() const { return n * sizeof(T); }
};

} // namespace slu

// ------------------------------------------------------------------ comm
struct slu_comm {
    int nprow = 1, npcol = 1, iam = 0, myrow = 0, mycol = 0, device = 0;
    ncclComm_t world = nullptr, row = nullptr, col = nullptr;
};

namespace slu {

using i64 = int64_t;

struct LevelRange {
    int diag_off = 0, diag_n = 0;
    int tl_off = 0, tl_n = 0;
    int tu_off = 0, tu_n = 0;
    int k_off = 0, k_n = 0;
    int tile_off = 0, tile_n = 0;
    int big_off = 0, big_n = 0; // 128x128 Schur tiles
    int df_off = 0, df_n = 0;   // fast diag items
    int lf_off = 0, lf_n = 0;   // fast L-panel TRSM items
    int uf_off = 0, uf_n = 0;   // fast U-panel TRSM items
    double schur_flops = 0;
    bool big = false;
};

struct PlanBase {
    virtual ~PlanBase() = default;
    virtual void upload() = 0;
    virtual void factor(double anorm, int *info, int *tiny) = 0;
    virtual void download() = 0;
    virtual void snapshot() = 0;
    virtual void restore() = 0;
    virtual void sync() = 0;
    slu_plan_stats stats{};
};

// One rank's plan for value type T (double / float / zc) over the host
// LUstruct layout LocalLU / LUS.
template <typename T, typename HT, typename LocalLU, typename LUS>
struct Plan : PlanBase {
    // ---- problem
    int n = 0, nsupers = 0, Pr = 1, Pc = 1, iam = 0, myrow = 0, mycol = 0;
    slu_comm *comm = nullptr;
    slu_engine_opts opts{};
    LUS *LU = nullptr;
    vector<i64> xsup;
    int nlc = 0, nlr = 0;
    hipStream_t stream = nullptr;

    // ---- local storage layout
    vector<i64> lval_off, uval_off; // per local column / row, -1 if empty
    vector<int> lval_ld;            // nsupr per local column
    i64 lval_total = 0, uval_total = 0;
    bool l_contig = false, u_contig = false;
    // L blocks (column-major order of columns, storage order within)
    vector<LBlk> lblk;
    vector<int> lblk_ib, lblk_rowstart, lblk_nrows;
    vector<int> lcol_first, lcol_nblk; // per local column
    vector<int> lmap;
    // U blocks
    vector<UBlk> ublk;
    vector<int> ublk_jb;
    vector<int> urow_first, urow_nblk;
    vector<i64> ucol_voff;
    vector<int> ucol_fst;

    // ---- schedule
    vector<int> level_of;
    vector<LevelRange> levels;
    vector<DiagItem<T>> diag_items;
    vector<TrsmLItem<T>> tl_items;
    vector<TrsmUItem<T>> tu_items;
    vector<KInfo<T>> kinfos;
    vector<TileItem> tiles, tiles_big;
    vector<DiagItemF<T>> df_items;
    vector<TrsmItemF<T>> lf_items, uf_items;
    i64 dinv_level_off = 0, dinv_max = 0; // per-level Dinv scratch
    // per-k panel arrays (device copies referenced by KInfo / TrsmUItem)
    vector<int> h_rg, h_ra, h_cg, h_cb, h_pair, h_ct0;
    vector<i64> h_cvoff;

    // ---- device
    DevBuf<T> d_L, d_U;
    DevBuf<LBlk> d_lblk;
    DevBuf<int> d_lmap;
    DevBuf<UBlk> d_ublk;
    DevBuf<i64> d_ucol_voff;
    DevBuf<int> d_ucol_fst;
    DevBuf<DiagItem<T>> d_diag;
    DevBuf<TrsmLItem<T>> d_tl;
    DevBuf<TrsmUItem<T>> d_tu;
    DevBuf<KInfo<T>> d_kinfo;
    DevBuf<TileItem> d_tiles, d_tiles_big;
    DevBuf<DiagItemF<T>> d_df;
    DevBuf<TrsmItemF<T>> d_lf, d_uf;
    DevBuf<T> d_dinv;
    DevBuf<int> d_rg, d_ra, d_cg, d_cb, d_pair, d_ct0;
    DevBuf<i64> d_cvoff;
    DevBuf<int> d_counters; // [0] tiny pivots, [1..] unused
    DevBuf<int> d_zpiv;     // per supernode: max zero-pivot column + 1

    int W(i64 k) const { return (int)(xsup[k + 1] - xsup[k]); }

    Plan(LUS *lu, int n_, int nprow, int npcol, int iam_, slu_comm *c,
         const slu_engine_opts *o) {
        LU = lu;
        n = n_;
        Pr = nprow;
        Pc = npcol;
        iam = iam_;
        myrow = iam / Pc;
        mycol = iam % Pc;
        comm = c;
        if (o) opts = *o;
        SLU_REQUIRE(Pr * Pc == 1 || (comm && comm->world),
                    "a %dx%d grid needs an RCCL communicator", Pr, Pc);
        if (comm) HIPCHK(hipSetDevice(comm->device));
        HIPCHK(hipStreamCreateWithFlags(&stream, hipStreamNonBlocking));
        int_t *hx = LU->Glu_persist->xsup;
        nsupers = (int)(LU->Glu_persist->supno[n - 1] + 1);
        xsup.assign(hx, hx + nsupers + 1);
        nlc = (nsupers + Pc - 1) / Pc;
        nlr = (nsupers + Pr - 1) / Pr;
        for (int k = 0; k < nsupers; ++k)
            SLU_REQUIRE(W(k) <= 512, "supernode %d has %d columns (> MAX_SUPER_SIZE 512)", k, W(k));
        SLU_REQUIRE(Pr * Pc == 1, "multi-rank grids: see build_exchange (not yet enabled)");
        build_local();
        build_schedule();
        build_device();
    }

    ~Plan() override {
        if (stream) (void)hipStreamDestroy(stream);
    }

    // ------------------------------------------------------- local layout
    void build_local() {
        LocalLU *Llu = LU->Llu;
        lval_off.assign(nlc, -1);
        lval_ld.assign(nlc, 0);
        lcol_first.assign(nlc, 0);
        lcol_nblk.assign(nlc, 0);
        i64 off = 0;
        l_contig = Llu->Lnzval_bc_dat != nullptr;
        for (int ljb = 0; ljb < nlc; ++ljb) {
            int jb = ljb * Pc + mycol;
            int_t *index = Llu->Lrowind_bc_ptr[ljb];
            lcol_first[ljb] = (int)lblk.size();
            if (!index) continue;
            int nb = (int)index[0], nsupr = (int)index[1];
            lval_off[ljb] = off;
            lval_ld[ljb] = nsupr;
            if (Llu->Lnzval_bc_dat && (HT *)Llu->Lnzval_bc_ptr[ljb] != (HT *)Llu->Lnzval_bc_dat + off)
                l_contig = false;
            i64 p = SLU_BC_HEADER;
            int rs = 0;
            for (int b = 0; b < nb; ++b) {
                int gb = (int)index[p], nr = (int)index[p + 1];
                LBlk L{};
                L.colvoff = off;
                L.mapoff = (i64)lmap.size();
                L.ld = nsupr;
                L.fcol = (int)xsup[jb];
                L.frow = (int)xsup[gb];
                lmap.resize(lmap.size() + W(gb), -1);
                for (int i = 0; i < nr; ++i) {
                    i64 gr = index[p + 2 + i];
                    lmap[L.mapoff + gr - xsup[gb]] = rs + i;
                }
                lblk.push_back(L);
                lblk_ib.push_back(gb);
                lblk_rowstart.push_back(rs);
                lblk_nrows.push_back(nr);
                rs += nr;
                p += SLU_LB_DESCRIPTOR + nr;
            }
            SLU_REQUIRE(rs == nsupr, "L column %d: block rows %d != nsupr %d", jb, rs, nsupr);
            lcol_nblk[ljb] = nb;
            off += (i64)nsupr * W(jb);
        }
        lval_total = off;

        uval_off.assign(nlr, -1);
        urow_first.assign(nlr, 0);
        urow_nblk.assign(nlr, 0);
        off = 0;
        u_contig = Llu->Unzval_br_dat != nullptr;
        for (int lb = 0; lb < nlr; ++lb) {
            int gb = lb * Pr + myrow;
            int_t *index = Llu->Ufstnz_br_ptr[lb];
            urow_first[lb] = (int)ublk.size();
            if (!index) continue;
            int nb = (int)index[0];
            i64 len = index[1];
            uval_off[lb] = off;
            if (Llu->Unzval_br_dat && (HT *)Llu->Unzval_br_ptr[lb] != (HT *)Llu->Unzval_br_dat + off)
                u_contig = false;
            i64 p = SLU_BR_HEADER, run = 0;
            i64 klst = xsup[gb + 1];
            for (int b = 0; b < nb; ++b) {
                int jb = (int)index[p];
                UBlk U{};
                U.coloff = (i64)ucol_voff.size();
                U.fcol = (int)xsup[jb];
                for (int c = 0; c < W(jb); ++c) {
                    i64 fst = index[p + SLU_UB_DESCRIPTOR + c];
                    ucol_voff.push_back(off + run);
                    ucol_fst.push_back((int)fst);
                    run += klst - fst;
                }
                ublk.push_back(U);
                ublk_jb.push_back(jb);
                p += SLU_UB_DESCRIPTOR + W(jb);
            }
            SLU_REQUIRE(run == len, "U row %d: segment lengths %lld != %lld", gb, (long long)run, (long long)len);
            urow_nblk[lb] = nb;
            off += len;
        }
        uval_total = off;
    }

    int find_lblk(int ib, int jb) const { // local column jb, block ib
        int ljb = jb / Pc, f = lcol_first[ljb], nb = lcol_nblk[ljb];
        auto b = lblk_ib.begin() + f, e = b + nb;
        auto it = std::lower_bound(b, e, ib);
        SLU_REQUIRE(it != e && *it == ib, "missing L block (%d,%d)", ib, jb);
        return (int)(it - lblk_ib.begin());
    }
    int find_ublk(int ib, int jb) const { // local row ib, block jb
        int lb = ib / Pr, f = urow_first[lb], nb = urow_nblk[lb];
        auto b = ublk_jb.begin() + f, e = b + nb;
        auto it = std::lower_bound(b, e, jb);
        SLU_REQUIRE(it != e && *it == jb, "missing U block (%d,%d)", ib, jb);
        return (int)(it - ublk_jb.begin());
    }

    // ------------------------------------------------------- schedule
    void build_schedule() {
        // dependency levels (1x1: the whole DAG is local)
        level_of.assign(nsupers, 0);
        int maxlev = 0;
        for (int k = 0; k < nsupers; ++k) {
            int lk = level_of[k];
            maxlev = std::max(maxlev, lk);
            int ljb = k / Pc;
            for (int b = 0; b < lcol_nblk[ljb]; ++b) {
                int ib = lblk_ib[lcol_first[ljb] + b];
                if (ib != k) level_of[ib] = std::max(level_of[ib], lk + 1);
            }
            int lb = k / Pr;
            for (int b = 0; b < urow_nblk[lb]; ++b) {
                int jb = ublk_jb[urow_first[lb] + b];
                level_of[jb] = std::max(level_of[jb], lk + 1);
            }
        }
        vector<vector<int>> bylev(maxlev + 1);
        for (int k = 0; k < nsupers; ++k) bylev[level_of[k]].push_back(k);
        levels.resize(maxlev + 1);
        stats.nsupers = nsupers;
        stats.nlevels = maxlev + 1;

        vector<int> owner(lblk.size() + ublk.size(), -1), touched;
        for (int L = 0; L <= maxlev; ++L) {
            LevelRange &R = levels[L];
            R.diag_off = (int)diag_items.size();
            R.tl_off = (int)tl_items.size();
            R.tu_off = (int)tu_items.size();
            R.k_off = (int)kinfos.size();
            R.tile_off = (int)tiles.size();
            R.big_off = (int)tiles_big.size();
            R.df_off = (int)df_items.size();
            R.lf_off = (int)lf_items.size();
            R.uf_off = (int)uf_items.size();
            dinv_level_off = 0;
            for (int k : bylev[L]) add_supernode(k, R);
            dinv_max = std::max(dinv_max, dinv_level_off);
            R.big_n = (int)tiles_big.size() - R.big_off;
            R.df_n = (int)df_items.size() - R.df_off;
            R.lf_n = (int)lf_items.size() - R.lf_off;
            R.uf_n = (int)uf_items.size() - R.uf_off;
            R.diag_n = (int)diag_items.size() - R.diag_off;
            R.tl_n = (int)tl_items.size() - R.tl_off;
            R.tu_n = (int)tu_items.size() - R.tu_off;
            R.k_n = (int)kinfos.size() - R.k_off;
            R.tile_n = (int)tiles.size() - R.tile_off;
            // conflicting destinations inside the level -> atomics
            touched.clear();
            for (int s = R.k_off; s < R.k_off + R.k_n; ++s) {
                KInfoHost &kh = khost[s];
                for (int h : kh.dests) {
                    int key = h >= 0 ? h : (int)lblk.size() + ~h;
                    if (owner[key] == -1) {
                        owner[key] = s;
                        touched.push_back(key);
                    } else if (owner[key] != s) {
                        kinfos[owner[key]].atomic = 1;
                        kinfos[s].atomic = 1;
                    }
                }
            }
            for (int key : touched) owner[key] = -1;
        }
        khost.clear();
    }

    struct KInfoHost {
        vector<int> dests;
    };
    vector<KInfoHost> khost;

    static constexpr bool cplx = sizeof(T) == 16;

    void add_supernode(int k, LevelRange &R) {
        LocalLU *Llu = LU->Llu;
        const int w = W(k);
        const int ljb = k / Pc, lb = k / Pr;
        const bool lcol_local = (k % Pc) == mycol && Llu->Lrowind_bc_ptr[ljb];
        const bool diag_here = lcol_local && (k % Pr) == myrow;
        // ---- diagonal block
        i64 diag_off = -1;
        int diag_ld = 0;
        constexpr int PW = PWOf<T>::v, RB = cplx ? RBOf<T>::v : 16 * TR_WAVES;
        const bool fast = w <= FAST_MAXW;
        const int nbk = (w + PW - 1) / PW;
        const i64 dinv_off = dinv_level_off;           // U^{-1} blocks at +0, (L^{-1})^T at +nbk*PW*PW
        if (fast) dinv_level_off += 2 * (i64)nbk * PW * PW;
        if (diag_here) {
            diag_off = lval_off[ljb];
            diag_ld = lval_ld[ljb];
            SLU_REQUIRE(lblk_ib[lcol_first[ljb]] == k, "diagonal block of %d is not first", k);
            if (fast) {
                DiagItemF<T> d{};
                d.a = (T *)(intptr_t)diag_off; // relocated in build_device
                d.dinv = (T *)(intptr_t)dinv_off;
                d.ld = diag_ld;
                d.w = w;
                d.k = k;
                d.fcol = (int)xsup[k];
                df_items.push_back(d);
            } else {
                DiagItem<T> d{};
                d.a = (T *)(intptr_t)diag_off; // relocated in build_device
                d.ld = diag_ld;
                d.w = w;
                d.k = k;
                d.fcol = (int)xsup[k];
                diag_items.push_back(d);
            }
            stats.n_diag++;
            // SRC/pdgstrf2.c:252,262 (complex weights SRC/pzgstrf2.c:253,263)
            double wd = w, s1 = wd * (wd - 1) / 2, s2 = (wd - 1) * wd * (2 * wd - 1) / 6;
            stats.panel_flops += cplx ? 6 * s1 + 10 * wd + 8 * s2 : s1 + 2 * s2;
        }
        // ---- L panel (rows of column k below the diagonal block)
        int r0 = 0, m = 0;
        vector<int> lbs; // L block ids of the panel (excluding the diagonal block)
        if (lcol_local) {
            int f = lcol_first[ljb], nb = lcol_nblk[ljb];
            for (int b = 0; b < nb; ++b) {
                if (lblk_ib[f + b] == k) { r0 += lblk_nrows[f + b]; continue; }
                lbs.push_back(f + b);
                m += lblk_nrows[f + b];
            }
            if (m > 0 && fast) {
                for (int c0 = 0; c0 < m; c0 += RB) {
                    TrsmItemF<T> t{};
                    t.x = (T *)(intptr_t)(lval_off[ljb] + r0 + c0);
                    t.t = (const T *)(intptr_t)diag_off;
                    t.dinv = (const T *)(intptr_t)dinv_off;
                    t.ldx = lval_ld[ljb];
                    t.ldt = diag_ld;
                    t.w = w;
                    t.nrows = std::min(RB, m - c0);
                    lf_items.push_back(t);
                    stats.n_trsm_items++;
                }
                stats.panel_flops += (cplx ? 4.0 : 1.0) * (double)w * (w + 1) * m;
            } else if (m > 0) {
                for (int c0 = 0; c0 < m; c0 += TRSM_THREADS) {
                    TrsmLItem<T> t{};
                    t.x = (T *)(intptr_t)(lval_off[ljb] + r0 + c0);
                    t.u = (const T *)(intptr_t)diag_off;
                    t.ldx = lval_ld[ljb];
                    t.ldu = diag_ld;
                    t.w = w;
                    t.nrows = std::min(TRSM_THREADS, m - c0);
                    tl_items.push_back(t);
                    stats.n_trsm_items++;
                }
                stats.panel_flops += (cplx ? 4.0 : 1.0) * (double)w * (w + 1) * m;
            }
        }
        // ---- U panel (nonempty columns of block row k)
        vector<int> ubs; // U block ids
        int ncols = 0, kmin = w;
        const int cols_off = (int)h_cg.size();
        if ((k % Pr) == myrow && Llu->Ufstnz_br_ptr[lb]) {
            int f = urow_first[lb], nb = urow_nblk[lb];
            i64 klst = xsup[k + 1];
            for (int b = 0; b < nb; ++b) {
                int ub = f + b, jb = ublk_jb[ub];
                int bidx = (int)ubs.size();
                bool any = false;
                for (int c = 0; c < W(jb); ++c) {
                    i64 e = ublk[ub].coloff + c;
                    int fst = ucol_fst[e];
                    if (fst >= klst) continue;
                    any = true;
                    h_cg.push_back((int)xsup[jb] + c);
                    h_cb.push_back(bidx);
                    h_cvoff.push_back(ucol_voff[e]);
                    int t0 = (int)(fst - xsup[k]);
                    h_ct0.push_back(t0);
                    kmin = std::min(kmin, t0);
                    ++ncols;
                    double seg = (double)(klst - fst);
                    stats.panel_flops += seg * (seg + 1);
                }
                if (any) ubs.push_back(ub);
            }
            for (int c0 = 0; fast && c0 < ncols; c0 += RB) {
                TrsmItemF<T> t{};
                t.x = nullptr; // Uval
                t.voff = (const i64 *)(intptr_t)(cols_off + c0);
                t.t0 = (const int *)(intptr_t)(cols_off + c0);
                t.t = (const T *)(intptr_t)diag_off;
                t.dinv = (const T *)(intptr_t)(dinv_off + (i64)nbk * PW * PW);
                t.ldt = diag_ld;
                t.w = w;
                t.nrows = std::min(RB, ncols - c0);
                uf_items.push_back(t);
                stats.n_trsm_items++;
            }
            for (int c0 = 0; !fast && c0 < ncols; c0 += TRSM_THREADS) {
                TrsmUItem<T> t{};
                t.l = (const T *)(intptr_t)diag_off;
                t.ldl = diag_ld;
                t.w = w;
                t.ncols = std::min(TRSM_THREADS, ncols - c0);
                t.voff = (const i64 *)(intptr_t)(cols_off + c0); // relocated
                t.t0 = (const int *)(intptr_t)(cols_off + c0);
                int km = w;
                for (int c = 0; c < t.ncols; ++c) km = std::min(km, h_ct0[cols_off + c0 + c]);
                t.kmin = km;
                tu_items.push_back(t);
                stats.n_trsm_items++;
            }
        }
        if (m == 0 || ncols == 0) return; // nothing to update from k here
        // ---- Schur update of k
        KInfo<T> ki{};
        ki.a = (const T *)(intptr_t)(lval_off[ljb] + r0);
        ki.lda = lval_ld[ljb];
        ki.m = m;
        ki.n = ncols;
        ki.kmin = kmin;
        ki.kw = w - kmin;
        ki.nub = (int)ubs.size();
        ki.cvoff = (const i64 *)(intptr_t)cols_off;
        ki.ct0 = (const int *)(intptr_t)cols_off;
        ki.cg = (const int *)(intptr_t)cols_off;
        ki.cb = (const int *)(intptr_t)cols_off;
        ki.ubase = nullptr; // Uval
        const int rows_off = (int)h_rg.size();
        for (size_t a = 0; a < lbs.size(); ++a)
            for (int i = 0; i < lblk_nrows[lbs[a]]; ++i) {
                h_rg.push_back(0); // filled from the index array below
                h_ra.push_back((int)a);
            }
        // fill global rows from the index array of column k
        {
            int_t *index = Llu->Lrowind_bc_ptr[ljb];
            i64 p = SLU_BC_HEADER;
            int w_ = rows_off;
            for (int b = 0; b < (int)index[0]; ++b) {
                int gb = (int)index[p], nr = (int)index[p + 1];
                if (gb != k)
                    for (int i = 0; i < nr; ++i) h_rg[w_++] = (int)index[p + 2 + i];
                p += SLU_LB_DESCRIPTOR + nr;
            }
        }
        ki.rg = (const int *)(intptr_t)rows_off;
        ki.ra = (const int *)(intptr_t)rows_off;
        const int pair_off = (int)h_pair.size();
        KInfoHost kh;
        for (size_t a = 0; a < lbs.size(); ++a) {
            int ib = lblk_ib[lbs[a]];
            for (size_t b = 0; b < ubs.size(); ++b) {
                int jb = ublk_jb[ubs[b]];
                int h = ib >= jb ? find_lblk(ib, jb) : ~find_ublk(ib, jb);
                h_pair.push_back(h);
                kh.dests.push_back(h);
            }
        }
        ki.pair = (const int *)(intptr_t)pair_off;
        ki.atomic = 0;
        kinfos.push_back(ki);
        khost.push_back(std::move(kh));
        const int slot = (int)kinfos.size() - 1 - R.k_off;
        const bool big = !cplx && m >= SB_BM && ncols >= SB_BN;
        const int BM = big ? SB_BM : SC_BM, BN = big ? SB_BN : SC_BN;
        const int tm = (m + BM - 1) / BM, tn = (ncols + BN - 1) / BN;
        for (int i = 0; i < tm; ++i)
            for (int j = 0; j < tn; ++j) (big ? tiles_big : tiles).push_back(TileItem{slot, i, j});
        // algorithmic work: exact unpadded flops and padded flops
        double fl = 0;
        for (int c = 0; c < ncols; ++c) fl += 2.0 * m * (w - h_ct0[cols_off + c]);
        double mult = sizeof(T) == 16 ? 4.0 : 1.0; // complex: 8 real flops per multiply-add
        stats.schur_flops += fl * mult;
        stats.schur_flops_padded += 2.0 * m * ncols * (double)(w - kmin) * mult;
        stats.scatter_bytes += 3.0 * sizeof(T) * (double)m * ncols;
        stats.n_schur_tiles += (i64)tm * tn;
        stats.n_diag += 0;
        R.schur_flops += fl * mult;
        if (w >= 64 && m >= 256 && ncols >= 256) R.big = true;
    }

    // ------------------------------------------------------- device
    void build_device() {
        d_L.alloc(std::max<i64>(lval_total, 1));
        d_U.alloc(std::max<i64>(uval_total, 1));
        T *L = d_L.p, *U = d_U.p;
        d_rg.upload(h_rg);
        d_ra.upload(h_ra);
        d_cg.upload(h_cg);
        d_cb.upload(h_cb);
        d_pair.upload(h_pair);
        d_ct0.upload(h_ct0);
        d_cvoff.upload(h_cvoff);
        for (auto &d : diag_items) d.a = L + (intptr_t)d.a;
        for (auto &t : tl_items) {
            t.x = L + (intptr_t)t.x;
            t.u = L + (intptr_t)t.u;
        }
        for (auto &t : tu_items) {
            t.l = L + (intptr_t)t.l;
            t.ubase = U;
            intptr_t co = (intptr_t)t.voff;
            t.voff = d_cvoff.p + co;
            t.t0 = d_ct0.p + co;
        }
        for (auto &k : kinfos) {
            k.a = L + (intptr_t)k.a;
            k.ubase = U;
            intptr_t co = (intptr_t)k.cvoff, ro = (intptr_t)k.rg, po = (intptr_t)k.pair;
            k.cvoff = d_cvoff.p + co;
            k.ct0 = d_ct0.p + co;
            k.cg = d_cg.p + co;
            k.cb = d_cb.p + co;
            k.rg = d_rg.p + ro;
            k.ra = d_ra.p + ro;
            k.pair = d_pair.p + po;
        }
        d_dinv.alloc(std::max<i64>(dinv_max, 1));
        for (auto &d : df_items) {
            d.a = L + (intptr_t)d.a;
            d.dinv = d_dinv.p + (intptr_t)d.dinv;
        }
        for (auto &t : lf_items) {
            t.x = L + (intptr_t)t.x;
            t.t = L + (intptr_t)t.t;
            t.dinv = d_dinv.p + (intptr_t)t.dinv;
        }
        for (auto &t : uf_items) {
            t.x = U;
            intptr_t co = (intptr_t)t.voff;
            t.voff = d_cvoff.p + co;
            t.t0 = d_ct0.p + co;
            t.t = L + (intptr_t)t.t;
            t.dinv = d_dinv.p + (intptr_t)t.dinv;
        }
        d_df.upload(df_items);
        d_lf.upload(lf_items);
        d_uf.upload(uf_items);
        d_diag.upload(diag_items);
        d_tl.upload(tl_items);
        d_tu.upload(tu_items);
        d_kinfo.upload(kinfos);
        d_tiles.upload(tiles);
        d_tiles_big.upload(tiles_big);
        d_lblk.upload(lblk);
        d_lmap.upload(lmap);
        d_ublk.upload(ublk);
        d_ucol_voff.upload(ucol_voff);
        d_ucol_fst.upload(ucol_fst);
        d_counters.alloc(4);
        d_zpiv.alloc(nsupers);
        stats.lu_bytes = (double)(lval_total + uval_total) * sizeof(T);
        stats.index_bytes = (double)(d_lblk.bytes() + d_lmap.bytes() + d_ublk.bytes() +
                                     d_ucol_voff.bytes() + d_ucol_fst.bytes() + d_diag.bytes() +
                                     d_tl.bytes() + d_tu.bytes() + d_kinfo.bytes() + d_tiles_big.bytes() +
                                     d_df.bytes() + d_lf.bytes() + d_uf.bytes() + d_dinv.bytes() +
                                     d_tiles.bytes() + d_rg.bytes() + d_ra.bytes() +
                                     d_cg.bytes() + d_cb.bytes() + d_pair.bytes() +
                                     d_ct0.bytes() + d_cvoff.bytes());
    }

    // ------------------------------------------------------- values
    void upload() override {
        LocalLU *Llu = LU->Llu;
        if (l_contig && lval_total) {
            HIPCHK(hipMemcpy(d_L.p, Llu->Lnzval_bc_dat, lval_total * sizeof(T), hipMemcpyHostToDevice));
        } else {
            for (int ljb = 0; ljb < nlc; ++ljb)
                if (lval_off[ljb] >= 0)
                    HIPCHK(hipMemcpy(d_L.p + lval_off[ljb], Llu->Lnzval_bc_ptr[ljb],
                                     (size_t)lval_ld[ljb] * W(ljb * Pc + mycol) * sizeof(T),
                                     hipMemcpyHostToDevice));
        }
        if (u_contig && uval_total) {
            HIPCHK(hipMemcpy(d_U.p, Llu->Unzval_br_dat, uval_total * sizeof(T), hipMemcpyHostToDevice));
        } else {
            for (int lb = 0; lb < nlr; ++lb)
                if (uval_off[lb] >= 0)
                    HIPCHK(hipMemcpy(d_U.p + uval_off[lb], Llu->Unzval_br_ptr[lb],
                                     (size_t)Llu->Ufstnz_br_ptr[lb][1] * sizeof(T),
                                     hipMemcpyHostToDevice));
        }
    }

    DevBuf<T> d_L0, d_U0; // pristine copies (snapshot)
    void snapshot() override {
        d_L0.alloc(d_L.n);
        d_U0.alloc(d_U.n);
        HIPCHK(hipMemcpyAsync(d_L0.p, d_L.p, d_L.bytes(), hipMemcpyDeviceToDevice, stream));
        HIPCHK(hipMemcpyAsync(d_U0.p, d_U.p, d_U.bytes(), hipMemcpyDeviceToDevice, stream));
        HIPCHK(hipStreamSynchronize(stream));
    }
    void restore() override {
        SLU_REQUIRE(d_L0.p && d_U0.p, "restore without snapshot");
        HIPCHK(hipMemcpyAsync(d_L.p, d_L0.p, d_L.bytes(), hipMemcpyDeviceToDevice, stream));
        HIPCHK(hipMemcpyAsync(d_U.p, d_U0.p, d_U.bytes(), hipMemcpyDeviceToDevice, stream));
    }
    void sync() override { HIPCHK(hipStreamSynchronize(stream)); }

    void download() override {
        LocalLU *Llu = LU->Llu;
        HIPCHK(hipStreamSynchronize(stream));
        if (l_contig && lval_total) {
            HIPCHK(hipMemcpy(Llu->Lnzval_bc_dat, d_L.p, lval_total * sizeof(T), hipMemcpyDeviceToHost));
        } else {
            for (int ljb = 0; ljb < nlc; ++ljb)
                if (lval_off[ljb] >= 0)
                    HIPCHK(hipMemcpy(Llu->Lnzval_bc_ptr[ljb], d_L.p + lval_off[ljb],
                                     (size_t)lval_ld[ljb] * W(ljb * Pc + mycol) * sizeof(T),
                                     hipMemcpyDeviceToHost));
        }
        if (u_contig && uval_total) {
            HIPCHK(hipMemcpy(Llu->Unzval_br_dat, d_U.p, uval_total * sizeof(T), hipMemcpyDeviceToHost));
        } else {
            for (int lb = 0; lb < nlr; ++lb)
                if (uval_off[lb] >= 0)
                    HIPCHK(hipMemcpy(Llu->Unzval_br_ptr[lb], d_U.p + uval_off[lb],
                                     (size_t)Llu->Ufstnz_br_ptr[lb][1] * sizeof(T),
                                     hipMemcpyDeviceToHost));
        }
    }

    void launch_trsm_fast(const LevelRange &R) {
        if constexpr (sizeof(T) == 16) {
            if (R.lf_n)
                hipLaunchKernelGGL((k_trsm_blk<T, 0>), dim3(R.lf_n), dim3(256), 0, stream,
                                   d_lf.p + R.lf_off);
            if (R.uf_n)
                hipLaunchKernelGGL((k_trsm_blk<T, 1>), dim3(R.uf_n), dim3(256), 0, stream,
                                   d_uf.p + R.uf_off);
        } else {
            if (R.lf_n)
                hipLaunchKernelGGL((k_trsm_reg<T, 0>), dim3(R.lf_n), dim3(64 * TR_WAVES), 0, stream,
                                   d_lf.p + R.lf_off);
            if (R.uf_n)
                hipLaunchKernelGGL((k_trsm_reg<T, 1>), dim3(R.uf_n), dim3(64 * TR_WAVES), 0, stream,
                                   d_uf.p + R.uf_off);
        }
    }

    void launch_big(const LevelRange &R) {
        if constexpr (sizeof(T) == 16) {
            SLU_REQUIRE(false, "no 128x128 Schur tiles for complex");
        } else {
            hipLaunchKernelGGL(k_schur_big<T>, dim3(R.big_n), dim3(256), 0, stream,
                               d_tiles_big.p + R.big_off, d_kinfo.p + R.k_off, d_L.p, d_U.p,
                               d_lblk.p, d_lmap.p, d_ublk.p, d_ucol_voff.p, d_ucol_fst.p);
        }
    }

    // ------------------------------------------------------- factor
    void factor(double anorm, int *info, int *tiny) override {
        // thresh = smach_dist("Epsilon") * anorm (SRC/pdgstrf.c:412-413); in
        // psgstrf thresh is a float product.
        const float s_eps = 5.9604644775390625e-08f; // FLT_EPSILON * 0.5
        double thresh = sizeof(T) == 4 ? (double)(float)(s_eps * (float)anorm) : (double)s_eps * anorm;
        HIPCHK(hipMemsetAsync(d_counters.p, 0, d_counters.bytes(), stream));
        HIPCHK(hipMemsetAsync(d_zpiv.p, 0, d_zpiv.bytes(), stream));
        const bool timing = opts.timing != 0;
        vector<hipEvent_t> ev;
        auto mark = [&]() -> int {
            hipEvent_t e;
            HIPCHK(hipEventCreate(&e));
            HIPCHK(hipEventRecord(e, stream));
            ev.push_back(e);
            return (int)ev.size() - 1;
        };
        struct Span { int a, b, kind; bool big; };
        vector<Span> spans;
        int e_start = timing ? mark() : -1;
        stats.n_schur_launches = 0;
        for (size_t L = 0; L < levels.size(); ++L) {
            const LevelRange &R = levels[L];
            if (R.diag_n) {
                int a = timing ? mark() : -1;
                hipLaunchKernelGGL(k_diag_lu<T>, dim3(R.diag_n), dim3(DIAG_THREADS), 0, stream,
                                   d_diag.p + R.diag_off, thresh, opts.replace_tiny_pivot,
                                   d_counters.p, d_zpiv.p);
                if (timing) spans.push_back({a, mark(), 0, false});
            }
            if (R.df_n) {
                int a = timing ? mark() : -1;
                hipLaunchKernelGGL(k_diag_lu_blk<T>, dim3(R.df_n), dim3(256), 0, stream,
                                   d_df.p + R.df_off, thresh, opts.replace_tiny_pivot,
                                   d_counters.p, d_zpiv.p);
                if (timing) spans.push_back({a, mark(), 0, false});
            }
            if (R.lf_n || R.uf_n) {
                int a = timing ? mark() : -1;
                launch_trsm_fast(R);
                if (timing) spans.push_back({a, mark(), 1, false});
            }
            if (R.tl_n || R.tu_n) {
                int a = timing ? mark() : -1;
                if (R.tl_n)
                    hipLaunchKernelGGL(k_trsm_l<T>, dim3(R.tl_n), dim3(TRSM_THREADS), 0, stream,
                                       d_tl.p + R.tl_off);
                if (R.tu_n)
                    hipLaunchKernelGGL(k_trsm_u<T>, dim3(R.tu_n), dim3(TRSM_THREADS), 0, stream,
                                       d_tu.p + R.tu_off);
                if (timing) spans.push_back({a, mark(), 1, false});
            }
            if (R.tile_n || R.big_n) {
                int a = timing ? mark() : -1;
                if (R.big_n) launch_big(R);
                if (R.tile_n)
                    hipLaunchKernelGGL(k_schur<T>, dim3(R.tile_n), dim3(SC_THREADS), 0, stream,
                                       d_tiles.p + R.tile_off, d_kinfo.p + R.k_off, d_L.p, d_U.p,
                                       d_lblk.p, d_lmap.p, d_ublk.p, d_ucol_voff.p, d_ucol_fst.p);
                stats.n_schur_launches++;
                if (timing) spans.push_back({a, mark(), 2, R.big});
            }
        }
        HIPCHK(hipGetLastError());
        int e_end = timing ? mark() : -1;
        HIPCHK(hipStreamSynchronize(stream));
        int hc[4];
        HIPCHK(hipMemcpy(hc, d_counters.p, sizeof hc, hipMemcpyDeviceToHost));
        vector<int> zp(nsupers);
        HIPCHK(hipMemcpy(zp.data(), d_zpiv.p, nsupers * sizeof(int), hipMemcpyDeviceToHost));
        // per-rank info: the zero pivot of the last supernode (in elimination
        // order) that had one (SRC/pdgstrf2.c:246-247 overwrites *info)
        int my_info = 0;
        for (int k = 0; k < nsupers; ++k)
            if (zp[k]) my_info = zp[k];
        *info = my_info;
        *tiny = hc[0];
        if (timing) {
            float ms;
            HIPCHK(hipEventElapsedTime(&ms, ev[e_start], ev[e_end]));
            stats.t_total_ms = ms;
            stats.t_diag_ms = stats.t_trsm_ms = stats.t_schur_ms = stats.t_schur_big_ms = 0;
            stats.schur_big_flops = 0;
            for (auto &s : spans) {
                HIPCHK(hipEventElapsedTime(&ms, ev[s.a], ev[s.b]));
                if (s.kind == 0) stats.t_diag_ms += ms;
                else if (s.kind == 1) stats.t_trsm_ms += ms;
                else {
                    stats.t_schur_ms += ms;
                    if (s.big) stats.t_schur_big_ms += ms;
                }
            }
            for (auto &R : levels)
                if (R.big) stats.schur_big_flops += R.schur_flops;
            for (auto e : ev) (void)hipEventDestroy(e);
        }
    }
};

template <typename P> PlanBase *make_plan(void *LU, int n, int pr, int pc, int iam, slu_comm *c,
                                          const slu_engine_opts *o) {
    return new P((decltype(std::declval<P>().LU))LU, n, pr, pc, iam, c, o);
}

} // namespace slu

struct slu_plan {
    int dtype = 0;
    std::unique_ptr<slu::PlanBase> impl;
};

using namespace slu;

extern "C" {

const char *slu_last_error(void) { return g_last_error.c_str(); }

int slu_comm_unique_id(void *uid) {
    try {
        ncclUniqueId id;
        NCCLCHK(ncclGetUniqueId(&id));
        memcpy(uid, &id, sizeof id);
        return 0;
    } catch (const std::exception &e) {
        set_last_error(e.what());
        return -1;
    }
}

slu_comm *slu_comm_create(const void *uid, int nprow, int npcol, int iam, int device) {
    try {
        auto *c = new slu_comm;
        c->nprow = nprow;
        c->npcol = npcol;
        c->iam = iam;
        c->myrow = iam / npcol;
        c->mycol = iam % npcol;
        c->device = device;
        HIPCHK(hipSetDevice(device));
        if (nprow * npcol > 1) {
            SLU_REQUIRE(uid != nullptr, "uid required for a %dx%d grid", nprow, npcol);
            ncclUniqueId id;
            memcpy(&id, uid, sizeof id);
            NCCLCHK(ncclCommInitRank(&c->world, nprow * npcol, id, iam));
            NCCLCHK(ncclCommSplit(c->world, c->myrow, c->mycol, &c->row, nullptr));
            NCCLCHK(ncclCommSplit(c->world, c->mycol, c->myrow, &c->col, nullptr));
        }
        return c;
    } catch (const std::exception &e) {
        set_last_error(e.what());
        return nullptr;
    }
}

void slu_comm_destroy(slu_comm *c) {
    if (!c) return;
    if (c->row) ncclCommDestroy(c->row);
    if (c->col) ncclCommDestroy(c->col);
    if (c->world) ncclCommDestroy(c->world);
    delete c;
}

slu_plan *slu_plan_create(int dtype, void *LU, int n, int nprow, int npcol, int iam,
                          slu_comm *comm, const slu_engine_opts *opts, char *err, int errlen) {
    try {
        auto *p = new slu_plan;
        p->dtype = dtype;
        switch (dtype) {
        case SLU_D:
            p->impl.reset(make_plan<Plan<double, double, dLocalLU_t, dLUstruct_t>>(LU, n, nprow, npcol, iam, comm, opts));
            break;
        case SLU_S:
            p->impl.reset(make_plan<Plan<float, float, sLocalLU_t, sLUstruct_t>>(LU, n, nprow, npcol, iam, comm, opts));
            break;
        case SLU_Z:
            p->impl.reset(make_plan<Plan<zc, doublecomplex, zLocalLU_t, zLUstruct_t>>(LU, n, nprow, npcol, iam, comm, opts));
            break;
        default:
            throw Error(fmt("bad dtype %d", dtype));
        }
        return p;
    } catch (const std::exception &e) {
        set_last_error(e.what());
        if (err && errlen > 0) snprintf(err, errlen, "%s", e.what());
        return nullptr;
    }
}

int slu_plan_upload(slu_plan *p) {
    try {
        p->impl->upload();
        return 0;
    } catch (const std::exception &e) {
        set_last_error(e.what());
        return -1;
    }
}

int slu_plan_factor(slu_plan *p, double anorm, int *info, int *tiny) {
    try {
        int i = 0, t = 0;
        p->impl->factor(anorm, &i, &t);
        if (info) *info = i;
        if (tiny) *tiny = t;
        return 0;
    } catch (const std::exception &e) {
        set_last_error(e.what());
        return -1;
    }
}

int slu_plan_download(slu_plan *p) {
    try {
        p->impl->download();
        return 0;
    } catch (const std::exception &e) {
        set_last_error(e.what());
        return -1;
    }
}

int slu_plan_snapshot(slu_plan *p) {
    try {
        p->impl->snapshot();
        return 0;
    } catch (const std::exception &e) {
        set_last_error(e.what());
        return -1;
    }
}

int slu_plan_restore(slu_plan *p) {
    try {
        p->impl->restore();
        return 0;
    } catch (const std::exception &e) {
        set_last_error(e.what());
        return -1;
    }
}

int slu_plan_sync(slu_plan *p) {
    try {
        p->impl->sync();
        return 0;
    } catch (const std::exception &e) {
        set_last_error(e.what());
        return -1;
    }
}

void slu_plan_destroy(slu_plan *p) { delete p; }

int slu_plan_get_stats(const slu_plan *p, slu_plan_stats *st) {
    *st = p->impl->stats;
    return 0;
}

} // extern "C"

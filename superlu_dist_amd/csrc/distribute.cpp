// Structural pddistribute: the LU storage the reference's
// pddistribute builds for one rank of a Pr x Pc grid from the symbolic
// factorization (Glu_persist + Glu_freeable) and A in the LUstruct's
// coordinates -- the first-time branch of SRC/pddistribute.c (Fact !=
// SamePattern_SameRowPerm, :673-1340, :1460-1509), restated on host threads.
//
// What the reference does, and what is kept bit for bit:
//   * U block row lb (gb = lb*Pr + myrow): blocks in ascending jb (the order
//     the jb loop first meets them, :991-1046); index = [nblocks, len(nzval),
//     len(index), {jb, nnz, fstnz[nsupc(jb)]}..., -1] with fstnz = xsup[gb+1]
//     for an empty column (:1020-1022); nzval = the column segments
//     [irow, xsup[gb+1]) in (jb, column) order.
//   * L block column ljb (jb = ljb*Pc + mycol): row blocks in the order lsub
//     first meets them, rows within a block in lsub order (:1057-1174), then
//     the blocks sorted by block row -- all of them, or all but the first
//     (the diagonal block) on the diagonal process row (quickSortM on
//     Lindval_loc_bc_ptr, :1179-1229; the keys are distinct, so any correct
//     sort gives the reference's order); nzval nsupr x nsupc column major.
//   * values: A's entries dropped into zeroed storage (the reference routes
//     them through its dense SPA; an entry outside the structure is lost in
//     both), the *_dat arrays contiguous in local block order with one spare
//     element (:1261-1352, :1461-1509).
//   * ToRecv / ToSendD / ToSendR from the U structure (:767-801), and bufmax
//     as the MAX over all ranks of the per-rank buffer sizes (:821-822,
//     :1132-1134, MPI_Allreduce :2370), computed here for every rank at once.
// The triangular-solve metadata of the reference (fmod / bmod / plists /
// trees, :1543-2236) is not built: the factorization does not read it.
//
// Why it is fast: the reference mallocs every block, fills it through a
// dense SPA of n x maxsup values, sorts into a second copy and then copies
// everything once more into the *_dat arrays (three passes and fresh pages
// over all of L and U: 25 s at 100^3 with MMD).  Here the sizes come first,
// the *_dat arrays are allocated once, and every block column / row is
// written exactly once by one thread.
#include "slu_mi355x.h"

#include <algorithm>
#include <atomic>
#include <cstdlib>
#include <chrono>
#include <sys/mman.h>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <memory>
#include <numeric>
#include <vector>

#include "common.h"

using std::vector;

namespace {

using i64 = int64_t;

template <typename T> inline T zero_of() { return T{}; }

// calloc (free()-able: the reference's Destroy_LU frees the *_dat arrays)
// with the 2 MB-aligned interior advised as transparent huge pages: the
// value arrays' first touch (A's entries here, the refill's zeroing, the
// factor download) then faults once per 2 MB instead of once per 4 KB
inline void *calloc_huge(size_t n, size_t sz) {
    void *p = calloc(n, sz);
    constexpr uintptr_t HP = uintptr_t(2) << 20;
    const uintptr_t a = ((uintptr_t)p + HP - 1) & ~(HP - 1), e = ((uintptr_t)p + n * sz) & ~(HP - 1);
    if (p && e > a) madvise((void *)a, e - a, MADV_HUGEPAGE);
    return p;
}

// the same for storage every element of which is written here (index
// arrays, the U segment list), first touched on the worker threads
inline void *malloc_huge(size_t bytes) {
    void *p = malloc(bytes);
    constexpr uintptr_t HP = uintptr_t(2) << 20;
    const uintptr_t a = ((uintptr_t)p + HP - 1) & ~(HP - 1), e = ((uintptr_t)p + bytes) & ~(HP - 1);
    if (p && e > a) madvise((void *)a, e - a, MADV_HUGEPAGE);
    return p;
}
struct FreeDeleter {
    void operator()(void *p) const { free(p); }
};

// Per-thread scratch of -1s, reset when a new call (generation) first uses
// it on a thread: parallel_for's workers are fresh threads, but the calling
// thread keeps its thread_locals from one call to the next.
struct Scratch {
    i64 gen = -1;
    vector<i64> v;
    void fresh(i64 g, i64 size) {
        if (gen != g || (i64)v.size() < size) v.assign(size, -1);
        gen = g;
    }
};
inline i64 next_generation() {
    static std::atomic<i64> g{0};
    return ++g;
}

template <typename T, typename LocalLU, typename LUstruct>
void *distribute_glu_t(i64 n, const int_t *xsup_in, const int_t *supno_in, const int_t *xlsub,
                       const int_t *lsub, const int_t *xusub, const int_t *usub, const i64 *xa,
                       const i64 *asub, const T *a, int Pr, int Pc, int myrow, int mycol,
                       bool place_a = true) {
    SLU_REQUIRE(n > 0 && Pr > 0 && Pc > 0 && myrow >= 0 && myrow < Pr && mycol >= 0 && mycol < Pc,
                "distribute: bad arguments (n %lld, grid %dx%d, rank (%d,%d))", (long long)n, Pr,
                Pc, myrow, mycol);
    const i64 ns = supno_in[n - 1] + 1;
    vector<i64> xsup(xsup_in, xsup_in + ns + 1);
    const int_t *supno = supno_in;
    auto W = [&](i64 k) { return xsup[k + 1] - xsup[k]; };
    const i64 nlc = (ns + Pc - 1) / Pc, nlr = (ns + Pr - 1) / Pr;

    // SLU_DIST_TIME=1: phase times on stderr (diagnostics)
    const bool dtime = getenv("SLU_DIST_TIME") != nullptr;
    auto dt0 = std::chrono::steady_clock::now();
    auto dtick = [&](const char *what) {
        if (!dtime) return;
        const auto t = std::chrono::steady_clock::now();
        fprintf(stderr, "[distribute] %-28s %8.1f ms\n", what, std::chrono::duration<double, std::milli>(t - dt0).count());
        dt0 = t;
    };
    // ---- U segments by block row: (column j, first row irow), j ascending
    //      (so jb ascending, then column), as the reference's jb loop meets them
    //      A counting sort on host threads: the columns in NCH chunks of about
    //      equal usub length, per (chunk, block row) counts, then each chunk
    //      fills its slice of every bucket (chunk order = column order)
    vector<i64> ucnt(ns + 1, 0);
    // (uninitialised storage: the fill below touches every entry on the
    // threads, where a vector's value-initialisation wrote GBs serially)
    // (int32 pairs: n < 2^31 is checked below; half the bytes to write)
    std::unique_ptr<std::pair<int32_t, int32_t>[], FreeDeleter> useg;
    {
        const int NCH = std::max(1, std::min(4 * slu::plan_threads(), (int)std::min<i64>(n, 64)));
        vector<i64> cb(NCH + 1, 0); // chunk c: columns [cb[c], cb[c + 1])
        for (int c = 1; c < NCH; ++c) {
            const i64 target = (i64)xusub[n] * c / NCH;
            cb[c] = std::max(cb[c - 1], (i64)(std::lower_bound(xusub, xusub + n + 1, (int_t)target) - xusub));
        }
        cb[NCH] = n;
        vector<i64> cc((size_t)NCH * ns, 0); // [chunk][block row] counts, then fill cursors
        std::atomic<int> bad(0);
        slu::parallel_for(NCH, [&](int c) {
            i64 *cnt = cc.data() + (size_t)c * ns;
            for (i64 j = cb[c]; j < cb[c + 1]; ++j)
                for (i64 i = xusub[j]; i < xusub[j + 1]; ++i) {
                    const i64 gb = supno[usub[i]];
                    if (gb >= supno[j]) bad = 1;
                    else cnt[gb]++;
                }
        }, 1);
        SLU_REQUIRE(!bad, "usub: a row is not above its column's diagonal block");
        dtick("U segments: counts");
        // bucket sizes, offsets, and per (chunk, bucket) start positions
        const int NB = (int)((ns + 4095) / 4096);
        slu::parallel_for(NB, [&](int t) {
            for (i64 gb = (i64)t * 4096; gb < std::min<i64>(ns, (i64)(t + 1) * 4096); ++gb) {
                i64 tot = 0;
                for (int c = 0; c < NCH; ++c) tot += cc[(size_t)c * ns + gb];
                ucnt[gb + 1] = tot;
            }
        }, 1);
        for (i64 k = 0; k < ns; ++k) ucnt[k + 1] += ucnt[k];
        slu::parallel_for(NB, [&](int t) {
            for (i64 gb = (i64)t * 4096; gb < std::min<i64>(ns, (i64)(t + 1) * 4096); ++gb) {
                i64 pos = ucnt[gb];
                for (int c = 0; c < NCH; ++c) {
                    const i64 k = cc[(size_t)c * ns + gb];
                    cc[(size_t)c * ns + gb] = pos;
                    pos += k;
                }
            }
        }, 1);
        SLU_REQUIRE(n < INT32_MAX, "distribute: n = %lld too large", (long long)n);
        dtick("U segments: offsets");
        useg.reset((std::pair<int32_t, int32_t> *)malloc_huge((size_t)ucnt[ns] * sizeof(std::pair<int32_t, int32_t>)));
        SLU_REQUIRE(useg || !ucnt[ns], "distribute: out of host memory (U segments)");
        slu::parallel_for(NCH, [&](int c) {
            i64 *fill = cc.data() + (size_t)c * ns;
            for (i64 j = cb[c]; j < cb[c + 1]; ++j)
                for (i64 i = xusub[j]; i < xusub[j + 1]; ++i) {
                    const i64 irow = usub[i];
                    useg[fill[supno[irow]]++] = {(int32_t)j, (int32_t)irow};
                }
        }, 1);
    }

    LUstruct *LU = (LUstruct *)calloc(1, sizeof(LUstruct));
    LU->Glu_persist = (Glu_persist_t *)calloc(1, sizeof(Glu_persist_t));
    LU->Glu_persist->xsup = (int_t *)malloc((ns + 1) * sizeof(int_t));
    LU->Glu_persist->supno = (int_t *)malloc(n * sizeof(int_t));
    std::copy(xsup.begin(), xsup.end(), LU->Glu_persist->xsup);
    std::copy(supno, supno + n, LU->Glu_persist->supno);
    LocalLU *Llu = (LocalLU *)calloc(1, sizeof(LocalLU));
    LU->Llu = Llu;
    LU->dt = sizeof(T) == 4 ? 's' : sizeof(T) == 8 ? 'd' : 'z';

    if (dtime) fprintf(stderr, "[distribute] %lld U segments\n", (long long)ucnt[ns]);
    dtick("U segments");
    // ---- U: per block row and process column, the reference's Urb_length,
    //      Urb_fstnz, Ucbs (:786-791) -> index / value sizes; bufmax[2], [3]
    //      over all ranks; the schedule arrays (:779-797) for this rank
    Llu->ToRecv = (int *)calloc(std::max<i64>(ns, 1), sizeof(int));
    Llu->ToSendD = (int *)calloc(std::max<i64>(nlr, 1), sizeof(int));
    Llu->ToSendR = (int **)malloc(std::max<i64>(nlc, 1) * sizeof(int *));
    int *tsr = (int *)malloc(std::max<i64>(nlc * Pc, 1) * sizeof(int));
    for (i64 i = 0; i < nlc * Pc; ++i) tsr[i] = SLU_EMPTY;
    for (i64 i = 0; i < nlc; ++i) Llu->ToSendR[i] = tsr + i * Pc;
    vector<i64> u_len(nlr, 0), u_len1(nlr, 0);
    vector<i64> bmax2(ns, 0), bmax3(ns, 0);
    slu::parallel_for((int)ns, [&](int gb) {
        thread_local vector<i64> len, fst, cbs, seen;
        len.assign(Pc, 0);
        fst.assign(Pc, 0);
        cbs.assign(Pc, 0);
        seen.assign(Pc, -1);
        const i64 klst = xsup[gb + 1];
        for (i64 e = ucnt[gb]; e < ucnt[gb + 1]; ++e) {
            const i64 j = useg[e].first, irow = useg[e].second, jb = supno[j];
            const int pc = (int)(jb % Pc);
            len[pc] += klst - irow;
            if (seen[pc] != jb) {
                seen[pc] = jb;
                fst[pc] += W(jb);
                cbs[pc]++;
            }
            if (mycol == gb % Pc && mycol != pc) Llu->ToSendR[gb / Pc][pc] = SLU_YES;
            if (mycol == pc) {
                if (myrow == gb % Pr) {
                    Llu->ToSendD[gb / Pr] = SLU_YES;
                    Llu->ToRecv[gb] = 1;
                } else {
                    Llu->ToRecv[gb] = 2;
                }
            }
        }
        for (int pc = 0; pc < Pc; ++pc)
            if (len[pc]) {
                const i64 len1 = fst[pc] + SLU_BR_HEADER + cbs[pc] * SLU_UB_DESCRIPTOR;
                bmax2[gb] = std::max(bmax2[gb], len1);
                bmax3[gb] = std::max(bmax3[gb], len[pc]);
                if (pc == mycol && gb % Pr == myrow) {
                    u_len[gb / Pr] = len[pc];
                    u_len1[gb / Pr] = len1;
                }
            }
    }, 256);

    dtick("U sizes");
    // ---- L: per block column and process row, rows and blocks (:1057-1134);
    //      bufmax[0], [1], [4] over all ranks; this rank's sizes
    vector<i64> l_len(nlc, 0), l_nrbl(nlc, 0);
    vector<i64> bmax0(ns, 0), bmax1(ns, 0), bmax4(ns, 0);
    const i64 gen = next_generation();
    slu::parallel_for((int)ns, [&](int jb) {
        thread_local vector<i64> rows, blks;
        thread_local Scratch mark;
        rows.assign(Pr, 0);
        blks.assign(Pr, 0);
        mark.fresh(gen, ns);
        const i64 f = xsup[jb];
        for (i64 i = xlsub[f]; i < xlsub[f + 1]; ++i) {
            const i64 gb = supno[lsub[i]];
            const int pr = (int)(gb % Pr);
            rows[pr]++;
            if (mark.v[gb] != jb) {
                mark.v[gb] = jb;
                blks[pr]++;
            }
        }
        for (int pr = 0; pr < Pr; ++pr)
            if (rows[pr]) {
                const i64 len1 = rows[pr] + SLU_BC_HEADER + blks[pr] * SLU_LB_DESCRIPTOR;
                bmax0[jb] = std::max(bmax0[jb], len1);
                bmax1[jb] = std::max(bmax1[jb], rows[pr] * W(jb));
                bmax4[jb] = std::max(bmax4[jb], rows[pr]);
            }
        if (jb % Pc == mycol && rows[myrow]) {
            l_len[jb / Pc] = rows[myrow];
            l_nrbl[jb / Pc] = blks[myrow];
        }
    }, 256);
    for (int i = 0; i < SLU_NBUFFERS; ++i) Llu->bufmax[i] = 0;
    for (i64 k = 0; k < ns; ++k) {
        Llu->bufmax[0] = std::max<int_t>(Llu->bufmax[0], bmax0[k]);
        Llu->bufmax[1] = std::max<int_t>(Llu->bufmax[1], bmax1[k]);
        Llu->bufmax[2] = std::max<int_t>(Llu->bufmax[2], bmax2[k]);
        Llu->bufmax[3] = std::max<int_t>(Llu->bufmax[3], bmax3[k]);
        Llu->bufmax[4] = std::max<int_t>(Llu->bufmax[4], bmax4[k]);
    }

    dtick("L sizes");
    // ---- contiguous *_dat arrays in local block order (+1 spare element)
    Llu->Lrowind_bc_ptr = (int_t **)calloc(std::max<i64>(nlc, 1), sizeof(int_t *));
    Llu->Lnzval_bc_ptr = (T **)calloc(std::max<i64>(nlc, 1), sizeof(T *));
    Llu->Lrowind_bc_offset = (long *)malloc(std::max<i64>(nlc, 1) * sizeof(long));
    Llu->Lnzval_bc_offset = (long *)malloc(std::max<i64>(nlc, 1) * sizeof(long));
    i64 li = 0, lv = 0;
    for (i64 ljb = 0; ljb < nlc; ++ljb) {
        if (!l_len[ljb]) {
            Llu->Lrowind_bc_offset[ljb] = Llu->Lnzval_bc_offset[ljb] = -1;
            continue;
        }
        Llu->Lrowind_bc_offset[ljb] = li;
        Llu->Lnzval_bc_offset[ljb] = lv;
        li += l_len[ljb] + SLU_BC_HEADER + l_nrbl[ljb] * SLU_LB_DESCRIPTOR;
        lv += l_len[ljb] * W(ljb * Pc + mycol);
    }
    Llu->Lrowind_bc_cnt = li + 1;
    Llu->Lnzval_bc_cnt = lv + 1;
    Llu->Lrowind_bc_dat = (int_t *)malloc_huge((li + 1) * sizeof(int_t));
    // a == nullptr: index arrays only (no value storage; the coarse symbolic
    // of frontend.cpp reads the structure of the 1x1 layout)
    // value arrays zeroed by calloc: fresh zero pages from the kernel for
    // these sizes, so only the pages A's entries land on are ever touched
    // here (the factorization writes the rest; 16.8 GB at 100^3)
    Llu->Lnzval_bc_dat = a ? (T *)calloc_huge((size_t)(lv + 1), sizeof(T)) : nullptr;
    SLU_REQUIRE(Llu->Lrowind_bc_dat && (Llu->Lnzval_bc_dat || !a), "distribute: out of host memory (L)");
    Llu->Lrowind_bc_dat[li] = 0;
    if (a) Llu->Lnzval_bc_dat[lv] = zero_of<T>();
    Llu->Ufstnz_br_ptr = (int_t **)calloc(std::max<i64>(nlr, 1), sizeof(int_t *));
    Llu->Unzval_br_ptr = (T **)calloc(std::max<i64>(nlr, 1), sizeof(T *));
    Llu->Ufstnz_br_offset = (long *)malloc(std::max<i64>(nlr, 1) * sizeof(long));
    Llu->Unzval_br_offset = (long *)malloc(std::max<i64>(nlr, 1) * sizeof(long));
    i64 ui = 0, uv = 0;
    for (i64 lb = 0; lb < nlr; ++lb) {
        if (!u_len[lb]) {
            Llu->Ufstnz_br_offset[lb] = Llu->Unzval_br_offset[lb] = -1;
            continue;
        }
        Llu->Ufstnz_br_offset[lb] = ui;
        Llu->Unzval_br_offset[lb] = uv;
        ui += u_len1[lb] + 1; // index[len1] = -1 end marker (:811, :826)
        uv += u_len[lb];
    }
    Llu->Ufstnz_br_cnt = ui + 1;
    Llu->Unzval_br_cnt = uv + 1;
    Llu->Ufstnz_br_dat = (int_t *)malloc_huge((ui + 1) * sizeof(int_t));
    Llu->Unzval_br_dat = a ? (T *)calloc_huge((size_t)(uv + 1), sizeof(T)) : nullptr;
    SLU_REQUIRE(Llu->Ufstnz_br_dat && (Llu->Unzval_br_dat || !a), "distribute: out of host memory (U)");
    Llu->Ufstnz_br_dat[ui] = 0;
    if (a) Llu->Unzval_br_dat[uv] = zero_of<T>();

    dtick("dat arrays");
    // ---- U block rows (one thread per row: index, zeroed segments, A's values)
    slu::parallel_for((int)nlr, [&](int lb) {
        if (!u_len[lb]) return;
        const i64 gb = (i64)lb * Pr + myrow, klst = xsup[gb + 1];
        int_t *index = Llu->Ufstnz_br_dat + Llu->Ufstnz_br_offset[lb];
        T *uval = a ? Llu->Unzval_br_dat + Llu->Unzval_br_offset[lb] : nullptr;
        const bool put = a && place_a;
        Llu->Ufstnz_br_ptr[lb] = index;
        Llu->Unzval_br_ptr[lb] = uval;
        const i64 len1 = u_len1[lb];
        index[1] = u_len[lb];
        index[2] = len1;
        index[len1] = -1;
        i64 nb = 0, ip = SLU_BR_HEADER, desc = -1, vo = 0, cur = -1;
        for (i64 e = ucnt[gb]; e < ucnt[gb + 1]; ++e) {
            const i64 j = useg[e].first, irow = useg[e].second, jb = supno[j];
            if (jb % Pc != mycol) continue;
            if (jb != cur) { // first segment of block jb (:1010-1022)
                cur = jb;
                ++nb;
                desc = ip;
                index[ip] = jb;
                index[ip + 1] = 0;
                for (i64 c = 0; c < W(jb); ++c) index[ip + SLU_UB_DESCRIPTOR + c] = klst;
                ip += SLU_UB_DESCRIPTOR + W(jb);
            }
            index[desc + SLU_UB_DESCRIPTOR + (j - xsup[jb])] = irow;
            const i64 k = klst - irow;
            index[desc + 1] += k;
            if (put) {
                T *seg = uval + vo; // (zero from calloc)
                for (i64 p = xa[j]; p < xa[j + 1]; ++p) {
                    const i64 r = asub[p];
                    if (r >= irow && r < klst) seg[r - irow] = a[p];
                }
            }
            vo += k;
        }
        index[0] = nb;
        SLU_REQUIRE(vo == u_len[lb] && ip == len1, "distribute: U row %lld sizes", (long long)gb);
    }, 16);

    dtick("U rows");
    // ---- L block columns (one thread per column)
    slu::parallel_for((int)nlc, [&](int ljb) {
        if (!l_len[ljb]) return;
        // per block row: block slot; per global row: position (-1 between uses)
        thread_local Scratch blk_s, pos_s;
        thread_local vector<i64> order, cnt, start;
        blk_s.fresh(gen, ns);
        pos_s.fresh(gen, n);
        vector<i64> &blk_of = blk_s.v, &pos = pos_s.v;
        const i64 jb = (i64)ljb * Pc + mycol, f = xsup[jb], w = W(jb);
        const i64 len = l_len[ljb], nrbl = l_nrbl[ljb];
        int_t *index = Llu->Lrowind_bc_dat + Llu->Lrowind_bc_offset[ljb];
        T *lusup = a ? Llu->Lnzval_bc_dat + Llu->Lnzval_bc_offset[ljb] : nullptr;
        Llu->Lrowind_bc_ptr[ljb] = index;
        Llu->Lnzval_bc_ptr[ljb] = lusup;
        // blocks in first-appearance order, rows per block
        order.clear();
        cnt.clear();
        for (i64 i = xlsub[f]; i < xlsub[f + 1]; ++i) {
            const i64 gb = supno[lsub[i]];
            if (gb % Pr != myrow) continue;
            if (blk_of[gb] < 0) {
                blk_of[gb] = (i64)order.size();
                order.push_back(gb);
                cnt.push_back(0);
            }
            cnt[blk_of[gb]]++;
        }
        SLU_REQUIRE((i64)order.size() == nrbl, "distribute: L column %lld blocks", (long long)jb);
        // the reference's sort (:1181-1191): by block row, the first block kept
        // in place on the diagonal process row
        vector<i64> sorted(order);
        std::sort(sorted.begin() + (myrow == jb % Pr ? 1 : 0), sorted.end());
        if (myrow == jb % Pr)
            SLU_REQUIRE(sorted.empty() || sorted[0] == jb,
                        "distribute: the first L block of column %lld is not its diagonal block",
                        (long long)jb);
        start.assign(nrbl, 0);
        index[0] = nrbl;
        index[1] = len;
        i64 ip = SLU_BC_HEADER, r = 0;
        for (i64 b = 0; b < nrbl; ++b) {
            const i64 gb = sorted[b], s = blk_of[gb], nr = cnt[s];
            index[ip] = gb;
            index[ip + 1] = nr;
            start[s] = ip + SLU_LB_DESCRIPTOR; // next row subscript of the block
            ip += SLU_LB_DESCRIPTOR + nr;
            cnt[s] = r;                        // next row position of the block
            r += nr;
        }
        for (i64 i = xlsub[f]; i < xlsub[f + 1]; ++i) {
            const i64 row = lsub[i], gb = supno[row];
            if (gb % Pr != myrow) continue;
            const i64 s = blk_of[gb];
            index[start[s]++] = row;
            pos[row] = cnt[s]++;
        }
        // (lusup is zero from calloc)
        for (i64 c = 0; a && place_a && c < w; ++c) {
            const i64 j = f + c;
            for (i64 p = xa[j]; p < xa[j + 1]; ++p) {
                const i64 row = asub[p];
                if (supno[row] < jb || supno[row] % Pr != myrow) continue;
                const i64 q = pos[row];
                if (q >= 0) lusup[q + c * len] = a[p];
            }
        }
        for (i64 gb : order) blk_of[gb] = -1;
        for (i64 i = xlsub[f]; i < xlsub[f + 1]; ++i) pos[lsub[i]] = -1;
    }, 16);
    dtick("L columns");
    return LU;
}

// pddistribute's Fact == SamePattern_SameRowPerm branch
// (SRC/pddistribute.c:545-672): the structure stays, L and U are zeroed and
// A's entries (CSC of the LUstruct's coordinates) dropped into it.
template <typename T, typename LocalLU, typename LUstruct>
void refill_values_t(LUstruct *LU, i64 n, const i64 *xa, const i64 *asub, const T *a, int Pr,
                     int Pc, int myrow, int mycol) {
    const int_t *xsup = LU->Glu_persist->xsup, *supno = LU->Glu_persist->supno;
    LocalLU *Llu = LU->Llu;
    const i64 ns = supno[n - 1] + 1, nlc = (ns + Pc - 1) / Pc, nlr = (ns + Pr - 1) / Pr;
    auto W = [&](i64 k) { return (i64)(xsup[k + 1] - xsup[k]); };
    const i64 gen = next_generation();
    slu::parallel_for((int)nlr, [&](int lb) {
        const int_t *index = Llu->Ufstnz_br_ptr[lb];
        if (!index) return;
        T *uval = (T *)Llu->Unzval_br_ptr[lb];
        const i64 gb = (i64)lb * Pr + myrow, klst = xsup[gb + 1];
        i64 ip = SLU_BR_HEADER, vo = 0;
        for (i64 b = 0; b < index[0]; ++b) {
            const i64 jb = index[ip];
            for (i64 c = 0; c < W(jb); ++c) {
                const i64 j = xsup[jb] + c, irow = index[ip + SLU_UB_DESCRIPTOR + c], k = klst - irow;
                T *seg = uval + vo;
                std::fill(seg, seg + k, zero_of<T>());
                for (i64 p = xa[j]; p < xa[j + 1]; ++p) {
                    const i64 r = asub[p];
                    if (r >= irow && r < klst) seg[r - irow] = a[p];
                }
                vo += k;
            }
            ip += SLU_UB_DESCRIPTOR + W(jb);
        }
    }, 16);
    slu::parallel_for((int)nlc, [&](int ljb) {
        const int_t *index = Llu->Lrowind_bc_ptr[ljb];
        if (!index) return;
        thread_local Scratch pos_s;
        pos_s.fresh(gen, n);
        vector<i64> &pos = pos_s.v;
        T *lusup = (T *)Llu->Lnzval_bc_ptr[ljb];
        const i64 jb = (i64)ljb * Pc + mycol, f = xsup[jb], w = W(jb), len = index[1];
        i64 ip = SLU_BC_HEADER, r = 0;
        for (i64 b = 0; b < index[0]; ++b) {
            const i64 nr = index[ip + 1];
            for (i64 i = 0; i < nr; ++i) pos[index[ip + SLU_LB_DESCRIPTOR + i]] = r++;
            ip += SLU_LB_DESCRIPTOR + nr;
        }
        std::fill(lusup, lusup + len * w, zero_of<T>());
        for (i64 c = 0; c < w; ++c) {
            const i64 j = f + c;
            for (i64 p = xa[j]; p < xa[j + 1]; ++p) {
                const i64 row = asub[p];
                if (supno[row] < jb || supno[row] % Pr != myrow) continue;
                const i64 q = pos[row];
                if (q >= 0) lusup[q + c * len] = a[p];
            }
        }
        ip = SLU_BC_HEADER;
        for (i64 b = 0; b < index[0]; ++b) {
            const i64 nr = index[ip + 1];
            for (i64 i = 0; i < nr; ++i) pos[index[ip + SLU_LB_DESCRIPTOR + i]] = -1;
            ip += SLU_LB_DESCRIPTOR + nr;
        }
    }, 16);
}

} // namespace

extern "C" {

int slu_refill_values(int dtype, void *LU, int64_t n, const int64_t *xa, const int64_t *asub,
                      const void *a, int nprow, int npcol, int myrow, int mycol) {
    try {
        switch (dtype) {
        case SLU_D:
            refill_values_t<double, dLocalLU_t>((dLUstruct_t *)LU, n, xa, asub, (const double *)a,
                                                nprow, npcol, myrow, mycol);
            return 0;
        case SLU_S:
            refill_values_t<float, sLocalLU_t>((sLUstruct_t *)LU, n, xa, asub, (const float *)a,
                                               nprow, npcol, myrow, mycol);
            return 0;
        case SLU_Z:
            refill_values_t<doublecomplex, zLocalLU_t>((zLUstruct_t *)LU, n, xa, asub,
                                                       (const doublecomplex *)a, nprow, npcol,
                                                       myrow, mycol);
            return 0;
        }
        throw slu::Error(slu::fmt("refill: bad dtype %d", dtype));
    } catch (const std::exception &e) {
        slu::set_last_error(e.what());
        return -1;
    }
}

void *slu_distribute_glu(int dtype, int64_t n, const int_t *xsup, const int_t *supno,
                         const int_t *xlsub, const int_t *lsub, const int_t *xusub,
                         const int_t *usub, const int64_t *xa, const int64_t *asub, const void *a,
                         int nprow, int npcol, int myrow, int mycol) {
    try {
        switch (dtype) {
        case SLU_D:
            return distribute_glu_t<double, dLocalLU_t, dLUstruct_t>(
                n, xsup, supno, xlsub, lsub, xusub, usub, xa, asub, (const double *)a, nprow,
                npcol, myrow, mycol);
        case SLU_S:
            return distribute_glu_t<float, sLocalLU_t, sLUstruct_t>(
                n, xsup, supno, xlsub, lsub, xusub, usub, xa, asub, (const float *)a, nprow,
                npcol, myrow, mycol);
        case SLU_Z:
            return distribute_glu_t<doublecomplex, zLocalLU_t, zLUstruct_t>(
                n, xsup, supno, xlsub, lsub, xusub, usub, xa, asub, (const doublecomplex *)a,
                nprow, npcol, myrow, mycol);
        }
        throw slu::Error(slu::fmt("distribute: bad dtype %d", dtype));
    } catch (const std::exception &e) {
        slu::set_last_error(e.what());
        return nullptr;
    }
}

// pddistribute of the device-resident library (abi.cpp): the value arrays
// allocated (zero) but A's entries not placed -- its pdgstrf fills the
// device storage from the A it keeps (real fp64 only)
void *slu_distribute_glu_deferred(int64_t n, const int_t *xsup, const int_t *supno,
                                  const int_t *xlsub, const int_t *lsub, const int_t *xusub,
                                  const int_t *usub, const int64_t *xa, const int64_t *asub,
                                  const double *a, int nprow, int npcol, int myrow, int mycol) {
    try {
        return distribute_glu_t<double, dLocalLU_t, dLUstruct_t>(n, xsup, supno, xlsub, lsub, xusub, usub,
                                                                 xa, asub, a, nprow, npcol, myrow, mycol,
                                                                 false);
    } catch (const std::exception &e) {
        slu::set_last_error(e.what());
        return nullptr;
    }
}

} // extern "C"

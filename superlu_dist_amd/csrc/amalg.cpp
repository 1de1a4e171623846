// Engine-side supernode amalgamation: analysis, coarse LUstruct, expand /
// compress programs (amalg.h explains what and why).  Host C++, run once per
// structure by the plan; the host apply() mirrors the device programs for
// the CPU tests (tests/test_amalg.py).
#include "amalg.h"

#include <algorithm>
#include <atomic>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <complex>
#include <cstring>

#include "common.h"

namespace slu {

namespace {

using i64 = int64_t;

// One original supernode's structure as the plan needs it.
struct SnInfo {
    i64 nsupr = 0, ulen = 0, ucols = 0; // L rows, U values, U column entries
    i64 ucne = 0;                       // non-empty U column entries
    double schur = 0, trsv = 0;         // 2 m seglen, seglen (seglen + 1) over U columns
    int parent = -1;                    // first block row below the diagonal block
    int b = 0;                          // L rows below the diagonal block
    bool sym = false, nested = false, ok = false;
};

// columns of U(s,:) with a non-empty segment, with their first rows
template <typename F> inline void for_ucols(const int_t *ux, const int_t *xsup, F &&f) {
    if (!ux) return;
    i64 p = SLU_BR_HEADER;
    for (i64 b = 0; b < ux[0]; ++b) {
        const i64 jb = ux[p], w = xsup[jb + 1] - xsup[jb];
        for (i64 c = 0; c < w; ++c) f(xsup[jb] + c, ux[p + SLU_UB_DESCRIPTOR + c]);
        p += SLU_UB_DESCRIPTOR + w;
    }
}

} // namespace

// U row J of the coarse partition: merged block columns J' with the first
// rows of every column
struct Amalg::URow {
    std::vector<int> blk;      // J' ascending
    std::vector<int32_t> fst;  // all columns of all blocks, first row (end: empty)
    std::vector<i64> colstart; // per block: first column entry
};
// what pass 4 (the programs) needs from passes 1-3
struct Amalg::Work {
    const int_t *xsup = nullptr;
    const int_t *const *lidx = nullptr;
    const int_t *const *uidx = nullptr;
    std::vector<int> gstart;
    std::vector<URow> urow;
    std::vector<i64> lval_len, ucol_len, lsrc, usrc, lmap, fcol;
};

std::vector<int> amalg_chains(int64_t n, int ns, const int_t *xsup, const int_t *const *lidx,
                              const int_t *const *uidx, double zero_frac, int maxw, int a0, int a1,
                              AmalgFlops *fl, std::vector<int64_t> *ucne) {
    const bool prof = getenv("SLU_AMALG_TIME") != nullptr;
    auto t0 = std::chrono::steady_clock::now();
    auto tick = [&](const char *what) {
        if (!prof) return;
        const auto t = std::chrono::steady_clock::now();
        fprintf(stderr, "[slu amalg] %s %.1f ms\n", what,
                std::chrono::duration<double, std::milli>(t - t0).count());
        t0 = t;
    };
    auto W = [&](i64 k) { return (int)(xsup[k + 1] - xsup[k]); };
    SLU_REQUIRE(n < (1ll << 31), "amalgamation: n %lld does not fit int32", (long long)n);
    const int nr = a1 - a0;

    // ---- pass 1: per supernode structure facts (parallel).  Set tests by
    // stamps in a per-thread row marker (no sorting: the reference's rows
    // come in symbfact's order, not ascending)
    std::vector<SnInfo> inf(nr);
    parallel_for(nr, [&](int si) {
        const int s = a0 + si;
        thread_local std::vector<uint32_t> mark;
        thread_local uint32_t stamp = 0;
        if ((i64)mark.size() < n) { mark.assign(n, 0); stamp = 0; }
        if (stamp > 0xFFFFFFF0u) { std::fill(mark.begin(), mark.end(), 0); stamp = 0; }
        SnInfo &I = inf[si];
        const int_t *ux = uidx[s];
        const int_t *ix = lidx[s];
        // L: diagonal block first and full, then mark below(s)
        const bool lok = ix && ix[0] >= 1 && ix[SLU_BC_HEADER] == s && ix[SLU_BC_HEADER + 1] == W(s);
        const uint32_t sb = ++stamp;
        if (ix) I.nsupr = ix[1];
        if (lok) {
            int b = 0;
            i64 p = SLU_BC_HEADER;
            for (i64 k = 0; k < ix[0]; ++k) {
                const i64 gb = ix[p], nrw = ix[p + 1];
                if (gb != s) {
                    for (i64 i = 0; i < nrw; ++i) mark[ix[p + 2 + i]] = sb;
                    b += (int)nrw;
                }
                p += SLU_LB_DESCRIPTOR + nrw;
            }
            I.b = b;
            SLU_REQUIRE(I.nsupr == W(s) + I.b, "amalgamation: L column %d rows %lld != %d + %d", s,
                        (long long)I.nsupr, W(s), I.b);
            if (ix[0] > 1) I.parent = (int)ix[SLU_BC_HEADER + SLU_LB_DESCRIPTOR + ix[SLU_BC_HEADER + 1]];
        }
        // U, once: column counts, and against the mark the symmetric test
        const i64 end = xsup[s + 1];
        int nuc = 0;
        bool sym = true;
        if (ux) {
            I.ulen = ux[1];
            i64 p = SLU_BR_HEADER;
            for (i64 k = 0; k < ux[0]; ++k) {
                const i64 jb = ux[p], w = xsup[jb + 1] - xsup[jb];
                I.ucols += w;
                for (i64 c = 0; c < w; ++c) {
                    const i64 fst = ux[p + SLU_UB_DESCRIPTOR + c];
                    if (fst >= end) continue;
                    ++nuc;
                    if (!lok) continue;
                    sym = sym && mark[xsup[jb] + c] == sb;
                    const double seg = (double)(end - fst);
                    I.trsv += seg * (seg + 1);
                    I.schur += 2.0 * I.b * seg;
                }
                p += SLU_UB_DESCRIPTOR + w;
            }
        }
        I.ucne = nuc;
        if (!lok) return;
        I.sym = sym && nuc == I.b; // (rows and columns are distinct: equal sets)
        I.ok = true;
        // nested into s+1: below(s) within cols(s+1) u below(s+1)
        if (I.parent == s + 1 && s + 1 < a1) {
            const uint32_t s2 = ++stamp;
            const int_t *i2 = lidx[s + 1];
            if (i2) {
                i64 p = SLU_BC_HEADER;
                for (i64 k = 0; k < i2[0]; ++k) {
                    const i64 nrw = i2[p + 1];
                    if (i2[p] != s + 1)
                        for (i64 i = 0; i < nrw; ++i) mark[i2[p + 2 + i]] = s2;
                    p += SLU_LB_DESCRIPTOR + nrw;
                }
            }
            const i64 f1 = xsup[s + 1], l1 = xsup[s + 2];
            bool nest = true;
            i64 p = SLU_BC_HEADER;
            for (i64 k = 0; nest && k < ix[0]; ++k) {
                const i64 nrw = ix[p + 1];
                if (ix[p] != s)
                    for (i64 i = 0; i < nrw; ++i) {
                        const i64 r = ix[p + 2 + i];
                        if ((r < f1 || r >= l1) && mark[r] != s2) { nest = false; break; }
                    }
                p += SLU_LB_DESCRIPTOR + nrw;
            }
            I.nested = nest;
        }
    }, 16);

    if (fl)
        for (int si = 0; si < nr; ++si) {
            const double w = W(a0 + si);
            fl->w += w;
            fl->s1 += w * (w - 1) / 2;
            fl->s2 += (w - 1) * w * (2 * w - 1) / 6;
            fl->trsm += w * (w + 1) * inf[si].b;
            fl->trsv += inf[si].trsv;
            fl->schur += inf[si].schur;
        }
    if (ucne) {
        ucne->resize(nr);
        for (int si = 0; si < nr; ++si) (*ucne)[si] = inf[si].ucne;
    }
    tick("pass 1 (structure facts)");
    // ---- pass 2: greedy chains (never across a1).  A chain only grows over
    // links e -> e + 1 that pass 1 allows, so the maximal runs of allowed
    // links are independent: runs in parallel, each greedy in order.
    auto link = [&](int e) {
        const SnInfo &A = inf[e - a0];
        return e + 1 < a1 && A.ok && A.sym && A.nested && A.parent == e + 1 && inf[e + 1 - a0].ok &&
               inf[e + 1 - a0].sym;
    };
    std::vector<int> runs; // first supernode of every run (end: a1)
    for (int s = a0; s < a1;) {
        runs.push_back(s);
        int e = s;
        while (link(e)) ++e;
        s = e + 1;
    }
    const int nruns = (int)runs.size();
    runs.push_back(a1);
    std::vector<std::vector<int>> rstart(nruns);
    parallel_for(nruns, [&](int ri) {
        thread_local std::vector<int32_t> ff; // first row of column g in the open chain
        if ((i64)ff.size() < n) ff.assign(n, -1);
        thread_local std::vector<int32_t> touched;
        const int r1 = runs[ri + 1];
        std::vector<int> &out = rstart[ri];
        int s = runs[ri];
        while (s < r1) {
            out.push_back(s);
            int e = s;
            const SnInfo &I0 = inf[s - a0];
            int wJ = W(s);
            i64 orig = (i64)W(s) * I0.nsupr + I0.ulen;
            touched.clear();
            if (e + 1 < r1)
                for_ucols(uidx[s], xsup, [&](i64 g, i64 fst) {
                    if (fst < xsup[s + 1]) { ff[g] = (int32_t)fst; touched.push_back((int32_t)g); }
                });
            while (e + 1 < r1 && wJ + W(e + 1) <= maxw) {
                const int c = e + 1;
                const i64 endc = xsup[c + 1];
                double S = 0;
                i64 b = 0;
                for_ucols(uidx[c], xsup, [&](i64 g, i64 fst) {
                    if (fst >= endc) return;
                    S += (double)(ff[g] >= 0 ? ff[g] : fst);
                    ++b;
                });
                const i64 w2 = wJ + W(c);
                const double merged = (double)w2 * (double)(w2 + b) + (double)b * (double)endc - S;
                const double orig2 = (double)orig + (double)W(c) * inf[c - a0].nsupr + inf[c - a0].ulen;
                if (merged - orig2 > zero_frac * merged) break;
                for_ucols(uidx[c], xsup, [&](i64 g, i64 fst) {
                    if (fst < endc && ff[g] < 0) { ff[g] = (int32_t)fst; touched.push_back((int32_t)g); }
                });
                wJ = (int)w2;
                orig = (i64)orig2;
                e = c;
            }
            for (int32_t g : touched) ff[g] = -1;
            s = e + 1;
        }
    }, 1);
    std::vector<int> gstart;
    for (auto &v : rstart) gstart.insert(gstart.end(), v.begin(), v.end());
    if (prof) { // the longest run bounds the pass (its chains are sequential)
        i64 tot = 0, mx = 0, mxlen = 0;
        for (int ri = 0; ri < nruns; ++ri) {
            i64 c = 0;
            for (int s = runs[ri]; s < runs[ri + 1]; ++s) c += inf[s - a0].ucols;
            tot += c;
            if (c > mx) { mx = c; mxlen = runs[ri + 1] - runs[ri]; }
        }
        fprintf(stderr, "[slu amalg] pass 2: %d runs, U column entries %lld, longest run %lld supernodes %lld entries\n",
                nruns, (long long)tot, (long long)mxlen, (long long)mx);
    }
    tick("pass 2 (chains)");
    return gstart;
}

bool Amalg::build(int64_t n_, int ns, const int_t *xsup, const int_t *const *lidx,
                  const int_t *const *uidx, double zero_frac, int maxw) {
    n = n_;
    ns1 = ns;
    const bool prof = getenv("SLU_AMALG_TIME") != nullptr;
    auto t0 = std::chrono::steady_clock::now();
    auto tick = [&](const char *what) {
        if (!prof) return;
        const auto t = std::chrono::steady_clock::now();
        fprintf(stderr, "[slu amalg] %s %.1f ms\n", what,
                std::chrono::duration<double, std::milli>(t - t0).count());
        t0 = t;
    };
    auto W = [&](i64 k) { return (int)(xsup[k + 1] - xsup[k]); };
    AmalgFlops fl;
    std::vector<i64> ucne; // non-empty U column entries per supernode
    std::vector<int> gstart = amalg_chains(n, ns, xsup, lidx, uidx, zero_frac, maxw, 0, ns, &fl, &ucne);
    fl_w = fl.w;
    fl_s1 = fl.s1;
    fl_s2 = fl.s2;
    fl_trsm = fl.trsm;
    fl_trsv = fl.trsv;
    fl_schur = fl.schur;
    ns2 = (int)gstart.size();
    tick("pass 2 (chains)");
    if (ns2 == ns1) return false;
    gstart.push_back(ns);
    grp.assign(ns, 0);
    xsup2.assign(ns2 + 1, 0);
    for (int J = 0; J < ns2; ++J) {
        for (int s = gstart[J]; s < gstart[J + 1]; ++s) grp[s] = J;
        xsup2[J] = xsup[gstart[J]];
        if (gstart[J + 1] - gstart[J] > 1) ++n_merged_groups;
    }
    xsup2[ns2] = xsup[ns];
    supno2.assign(n, 0);
    for (int J = 0; J < ns2; ++J)
        for (i64 c = xsup2[J]; c < xsup2[J + 1]; ++c) supno2[c] = J;
    auto W2 = [&](i64 J) { return (int)(xsup2[J + 1] - xsup2[J]); };

    // original value offsets (contiguous in supernode order) and program offsets
    std::vector<i64> lsrc(ns + 1, 0), usrc(ns + 1, 0), lmap(ns + 1, 0), fcol(ns + 1, 0);
    for (int s = 0; s < ns; ++s) {
        lsrc[s + 1] = lsrc[s] + (lidx[s] ? (i64)lidx[s][1] * W(s) : 0);
        usrc[s + 1] = usrc[s] + (uidx[s] ? (i64)uidx[s][1] : 0);
        lmap[s + 1] = lmap[s] + (lidx[s] ? (i64)lidx[s][1] : 0);
        fcol[s + 1] = fcol[s] + ucne[s];
    }
    lval1 = lsrc[ns];
    uval1 = usrc[ns];

    // ---- pass 3a: merged structure sizes per J (parallel)
    work.reset(new Work);
    Work &wk = *work;
    wk.xsup = xsup;
    wk.lidx = lidx;
    wk.uidx = uidx;
    wk.gstart = gstart;
    std::vector<URow> &urow = wk.urow;
    urow.resize(ns2);
    std::vector<i64> &lval_len = wk.lval_len, &ucol_len = wk.ucol_len;
    lval_len.assign(ns2 + 1, 0);
    ucol_len.assign(ns2 + 1, 0);
    std::vector<i64> lidx_len(ns2 + 1, 0), uidx_len(ns2 + 1, 0), uval_len(ns2 + 1, 0);
    std::vector<int> nblk2(ns2, 0);
    parallel_for(ns2, [&](int J) {
        thread_local std::vector<int32_t> ff;
        if ((i64)ff.size() < n) ff.assign(n, -1);
        const int s0 = gstart[J], e = gstart[J + 1] - 1, wJ = W2(J);
        const i64 endJ = xsup2[J + 1];
        // L: diagonal block + e's blocks below J grouped by merged block row
        const int_t *ix = lidx[e];
        i64 nb = 1, rows = wJ;
        if (ix) {
            i64 p = SLU_BC_HEADER, last = -1;
            for (i64 b = 0; b < ix[0]; ++b) {
                const i64 gb = ix[p], nr = ix[p + 1];
                if (gb != e) {
                    const int I = grp[gb];
                    if (I != last) { ++nb; last = I; }
                    rows += nr;
                }
                p += SLU_LB_DESCRIPTOR + nr;
            }
        }
        nblk2[J] = (int)nb;
        lidx_len[J + 1] = SLU_BC_HEADER + SLU_LB_DESCRIPTOR * nb + rows;
        lval_len[J + 1] = rows * wJ;
        // U: first rows over the members (the first member holding a column)
        URow &U = urow[J];
        std::vector<int32_t> cols;
        for (int a = s0; a <= e; ++a)
            for_ucols(uidx[a], xsup, [&](i64 g, i64 fst) {
                if (fst >= xsup[a + 1] || g < endJ) return;
                if (ff[g] < 0) { ff[g] = (int32_t)fst; cols.push_back((int32_t)g); }
            });
        std::sort(cols.begin(), cols.end());
        i64 len = 0, ncol = 0;
        for (size_t i = 0; i < cols.size();) {
            const int Jp = supno2[cols[i]];
            U.blk.push_back(Jp);
            U.colstart.push_back(ncol);
            for (i64 c = xsup2[Jp]; c < xsup2[Jp + 1]; ++c) {
                const int32_t f = ff[c] >= 0 ? ff[c] : (int32_t)endJ;
                U.fst.push_back(f);
                len += endJ - f;
            }
            ncol += W2(Jp);
            while (i < cols.size() && supno2[cols[i]] == Jp) ++i;
        }
        for (int32_t g : cols) ff[g] = -1;
        ucol_len[J + 1] = ncol;
        uidx_len[J + 1] = U.blk.empty() ? 0 : SLU_BR_HEADER + SLU_UB_DESCRIPTOR * (i64)U.blk.size() + ncol + 1;
        uval_len[J + 1] = len;
    }, 1);
    for (int J = 0; J < ns2; ++J) {
        lidx_len[J + 1] += lidx_len[J];
        lval_len[J + 1] += lval_len[J];
        uidx_len[J + 1] += uidx_len[J];
        uval_len[J + 1] += uval_len[J];
        ucol_len[J + 1] += ucol_len[J];
    }
    tick("pass 3a (merged sizes)");
    lval2 = lval_len[ns2];
    uval2 = uval_len[ns2];
    if (on_sizes) on_sizes(lval2, uval2);
    Lidx2.resize_uninit(lidx_len[ns2]);
    Uidx2.resize_uninit(uidx_len[ns2]);
    Loff2.assign(ns2, -1);
    Lvoff2.assign(ns2, -1);
    Uoff2.assign(ns2, -1);
    Uvoff2.assign(ns2, -1);
    // D: U-kind entries (one per merged U column entry), then L-kind (w_J per J)
    DL0 = ucol_len[ns2];
    SLU_REQUIRE(DL0 + n < (1ll << 31), "amalgamation: destination table exceeds int32");

    // ---- pass 3b: merged index arrays (parallel)
    parallel_for(ns2, [&](int J) {
        const int e = gstart[J + 1] - 1, wJ = W2(J);
        const i64 x2J = xsup2[J], endJ = xsup2[J + 1];
        const i64 nsupr2 = (lval_len[J + 1] - lval_len[J]) / wJ;
        // L index
        Loff2[J] = lidx_len[J];
        Lvoff2[J] = lval_len[J];
        int_t *L = &Lidx2[lidx_len[J]];
        L[0] = nblk2[J];
        L[1] = nsupr2;
        i64 q = SLU_BC_HEADER;
        L[q] = J;
        L[q + 1] = wJ;
        for (int c = 0; c < wJ; ++c) L[q + 2 + c] = x2J + c;
        q += SLU_LB_DESCRIPTOR + wJ;
        {
            const int_t *ix = lidx[e];
            i64 p = SLU_BC_HEADER, desc = -1, last = -1;
            for (i64 b = 0; ix && b < ix[0]; ++b) {
                const i64 gb = ix[p], nr = ix[p + 1];
                if (gb != e) {
                    const int I = grp[gb];
                    if (I != last) {
                        desc = q;
                        L[q] = I;
                        L[q + 1] = 0;
                        q += SLU_LB_DESCRIPTOR;
                        last = I;
                    }
                    for (i64 i = 0; i < nr; ++i) L[q++] = ix[p + 2 + i];
                    L[desc + 1] += nr;
                }
                p += SLU_LB_DESCRIPTOR + nr;
            }
        }
        SLU_REQUIRE(q == lidx_len[J + 1] - lidx_len[J], "amalgamation: L index length of %d", J);
        // rows ascending within each block below the diagonal (the layout is
        // the engine's own: ascending rows keep the Schur scatter's
        // destination addresses in runs)
        {
            i64 p = SLU_BC_HEADER + SLU_LB_DESCRIPTOR + wJ;
            for (i64 b = 1; b < L[0]; ++b) {
                const i64 nr = L[p + 1];
                std::sort(L + p + 2, L + p + 2 + nr);
                p += SLU_LB_DESCRIPTOR + nr;
            }
        }
        // U index
        const URow &U = urow[J];
        if (!U.blk.empty()) {
            Uoff2[J] = uidx_len[J];
            Uvoff2[J] = uval_len[J];
            int_t *X = &Uidx2[uidx_len[J]];
            const i64 len1 = uidx_len[J + 1] - uidx_len[J] - 1;
            X[0] = (int_t)U.blk.size();
            X[1] = uval_len[J + 1] - uval_len[J];
            X[2] = len1;
            X[len1] = -1;
            i64 p = SLU_BR_HEADER, ce = 0;
            for (size_t b = 0; b < U.blk.size(); ++b) {
                const int Jp = U.blk[b];
                X[p] = Jp;
                i64 nnz = 0;
                for (int c = 0; c < W2(Jp); ++c, ++ce) {
                    const int32_t f = U.fst[ce];
                    X[p + SLU_UB_DESCRIPTOR + c] = f;
                    nnz += endJ - f;
                }
                X[p + 1] = nnz;
                p += SLU_UB_DESCRIPTOR + W2(Jp);
            }
        }
    }, 1);
    tick("pass 3b (merged index arrays)");
    // explicit zeros introduced
    zeros = (lval2 + uval2) - (lval1 + uval1);
    wk.lsrc = std::move(lsrc);
    wk.usrc = std::move(usrc);
    wk.lmap = std::move(lmap);
    wk.fcol = std::move(fcol);
    if (!programs) work.reset();
    else if (!defer_programs) build_programs();
    return true;
}

void Amalg::set_index(const int_t *const *lidx, const int_t *const *uidx) {
    SLU_REQUIRE(work, "amalgamation: no deferred programs to build");
    work->lidx = lidx;
    work->uidx = uidx;
}

Amalg::Amalg() = default;
Amalg::~Amalg() = default;

// ---- pass 4: D, the expand programs (parallel over merged supernodes; the
// index arrays of pass 3b give every group's row positions)
void Amalg::build_programs() {
    SLU_REQUIRE(work, "amalgamation: programs without an analysis");
    const bool prof = getenv("SLU_AMALG_TIME") != nullptr;
    const auto t0 = std::chrono::steady_clock::now();
    Work &wk = *work;
    const int_t *xsup = wk.xsup;
    const int_t *const *lidx = wk.lidx;
    const int_t *const *uidx = wk.uidx;
    const std::vector<int> &gstart = wk.gstart;
    const std::vector<i64> &lsrc = wk.lsrc, &usrc = wk.usrc, &lmap = wk.lmap, &fcol = wk.fcol,
                           &lval_len = wk.lval_len, &ucol_len = wk.ucol_len;
    const int ns = ns1;
    auto W = [&](i64 k) { return (int)(xsup[k + 1] - xsup[k]); };
    auto W2 = [&](i64 J) { return (int)(xsup2[J + 1] - xsup2[J]); };
    // (uninitialised: every entry is written below, the first touch spread
    // over the threads)
    D.resize_uninit(DL0 + n);
    lcols.resize(ns);
    lrow.resize_uninit(lmap[ns]);
    urows.resize(ns);
    ucd.resize_uninit(fcol[ns]);
    ucl.resize_uninit(fcol[ns]);
    parallel_for(ns2, [&](int J) {
        thread_local std::vector<int32_t> rowpos;
        if ((i64)rowpos.size() < n) rowpos.assign(n, -1);
        const int s0 = gstart[J], e = gstart[J + 1] - 1, wJ = W2(J);
        const i64 x2J = xsup2[J], endJ = xsup2[J + 1];
        const i64 nsupr2 = (lval_len[J + 1] - lval_len[J]) / wJ;
        const int_t *L = Lidx2.data() + Loff2[J];
        {
            i64 p = SLU_BC_HEADER + SLU_LB_DESCRIPTOR + wJ;
            int32_t r = wJ;
            for (i64 b = 1; b < L[0]; ++b) {
                const i64 nr = L[p + 1];
                for (i64 i = 0; i < nr; ++i) rowpos[L[p + 2 + i]] = r++;
                p += SLU_LB_DESCRIPTOR + nr;
            }
        }
        // D (U kind)
        const URow &U = wk.urow[J];
        if (!U.blk.empty()) {
            i64 ce = 0, seg = 0;
            const i64 d0 = ucol_len[J];
            for (size_t b = 0; b < U.blk.size(); ++b)
                for (int c = 0; c < W2(U.blk[b]); ++c, ++ce) {
                    const int32_t f = U.fst[ce];
                    D[d0 + ce] = Uvoff2[J] + seg - f;
                    seg += endJ - f;
                }
        }
        // D (L kind): row fst of column g inside J -> Lvoff2 + (g - x2J) * ld2 + fst - x2J
        for (int c = 0; c < wJ; ++c) D[DL0 + x2J + c] = Lvoff2[J] + (i64)c * nsupr2 - x2J;
        // expand programs of the members
        for (int a = s0; a <= e; ++a) {
            const int_t *ix = lidx[a];
            LCol &C = lcols[a];
            C.src = lsrc[a];
            C.dst = Lvoff2[J] + (xsup[a] - x2J) * nsupr2;
            C.map = lmap[a];
            C.nsupr = ix ? (int32_t)ix[1] : 0;
            C.w = W(a);
            C.ld2 = (int32_t)nsupr2;
            C.pad = 0;
            if (ix) {
                i64 p = SLU_BC_HEADER, o = lmap[a];
                for (i64 b = 0; b < ix[0]; ++b) {
                    const i64 nr = ix[p + 1];
                    for (i64 i = 0; i < nr; ++i) {
                        const i64 r = ix[p + 2 + i];
                        const int32_t pos = r < endJ ? (int32_t)(r - x2J) : rowpos[r];
                        SLU_REQUIRE(pos >= 0, "amalgamation: row %lld of L column %d not in group %d",
                                    (long long)r, a, J);
                        lrow[o++] = pos;
                    }
                    p += SLU_LB_DESCRIPTOR + nr;
                }
            }
            const int_t *ux = uidx[a];
            URowX &R = urows[a];
            R.src = usrc[a];
            R.c0 = fcol[a];
            R.nc = (int32_t)(fcol[a + 1] - fcol[a]);
            R.end = (int32_t)xsup[a + 1];
            R.w = W(a);
            R.pad = 0;
            if (!ux) continue;
            i64 p = SLU_BR_HEADER, f0 = fcol[a];
            for (i64 b = 0; b < ux[0]; ++b) {
                const i64 jb = ux[p], w = W(jb);
                i64 d0;
                if (grp[jb] == J) {
                    d0 = DL0 + xsup[jb];
                } else {
                    const int Jp = grp[jb];
                    const auto it = std::lower_bound(U.blk.begin(), U.blk.end(), Jp);
                    SLU_REQUIRE(it != U.blk.end() && *it == Jp,
                                "amalgamation: U block (%d,%lld) not in merged row %d", a, (long long)jb, J);
                    d0 = ucol_len[J] + U.colstart[it - U.blk.begin()] + (xsup[jb] - xsup2[Jp]);
                }
                for (i64 c = 0; c < w; ++c) {
                    const i64 fst = ux[p + SLU_UB_DESCRIPTOR + c];
                    if (fst >= R.end) continue;
                    SLU_REQUIRE(R.end - fst <= 65536, "amalgamation: U segment of %lld rows (> 65536)",
                                (long long)(R.end - fst));
                    ucd[f0] = (int32_t)(d0 + c);
                    ucl[f0] = (uint16_t)(R.end - fst - 1);
                    ++f0;
                }
                p += SLU_UB_DESCRIPTOR + w;
            }
            SLU_REQUIRE(f0 == fcol[a + 1], "amalgamation: U row %d non-empty columns", a);
        }
        {
            i64 p = SLU_BC_HEADER + SLU_LB_DESCRIPTOR + wJ;
            for (i64 b = 1; b < L[0]; ++b) {
                const i64 nr = L[p + 1];
                for (i64 q = 0; q < nr; ++q) rowpos[L[p + 2 + q]] = -1;
                p += SLU_LB_DESCRIPTOR + nr;
            }
        }
    }, 1);
    work.reset(); // (the analysis state is not needed again)
    if (prof)
        fprintf(stderr, "[slu amalg] pass 4 (programs) %.1f ms\n",
                std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count());
}

void Amalg::coarse_glu(std::vector<int_t> &xlsub, std::vector<int_t> &lsub,
                       std::vector<int_t> &xusub, std::vector<int_t> &usub) const {
    xlsub.assign(n + 1, 0);
    lsub.clear();
    lsub.reserve(Lidx2.size());
    for (int J = 0; J < ns2; ++J) {
        const int_t *ix = Lidx2.data() + Loff2[J];
        xlsub[xsup2[J]] = (int_t)lsub.size();
        i64 p = SLU_BC_HEADER;
        for (i64 b = 0; b < ix[0]; ++b) {
            const i64 nr = ix[p + 1];
            lsub.insert(lsub.end(), ix + p + 2, ix + p + 2 + nr);
            p += SLU_LB_DESCRIPTOR + nr;
        }
        for (i64 c = xsup2[J] + 1; c <= xsup2[J + 1]; ++c) xlsub[c] = (int_t)lsub.size();
    }
    // U: per column, the first row of its segment in every coarse block row
    xusub.assign(n + 1, 0);
    auto walk = [&](auto &&f) {
        for (int I = 0; I < ns2; ++I) {
            if (Uoff2[I] < 0) continue;
            const int_t *ux = Uidx2.data() + Uoff2[I];
            const i64 end = xsup2[I + 1];
            i64 p = SLU_BR_HEADER;
            for (i64 b = 0; b < ux[0]; ++b) {
                const i64 Jp = ux[p], w = xsup2[Jp + 1] - xsup2[Jp];
                for (i64 c = 0; c < w; ++c) {
                    const i64 fst = ux[p + SLU_UB_DESCRIPTOR + c];
                    if (fst < end) f(xsup2[Jp] + c, fst);
                }
                p += SLU_UB_DESCRIPTOR + w;
            }
        }
    };
    walk([&](i64 g, i64) { ++xusub[g + 1]; });
    for (i64 j = 0; j < n; ++j) xusub[j + 1] += xusub[j];
    usub.assign(std::max<i64>(xusub[n], 1), 0);
    std::vector<int_t> fill(xusub.begin(), xusub.end() - 1);
    walk([&](i64 g, i64 fst) { usub[fill[g]++] = fst; });
}

template <typename T> void Amalg::apply(T *oL, T *oU, T *mL, T *mU, int dir) const {
    parallel_for((int)lcols.size(), [&](int s) {
        const LCol &C = lcols[s];
        for (int c = 0; c < C.w; ++c)
            for (int i = 0; i < C.nsupr; ++i) {
                T *o = oL + C.src + (i64)c * C.nsupr + i;
                T *m = mL + C.dst + (i64)c * C.ld2 + lrow[C.map + i];
                if (dir == 0) *m = *o;
                else *o = *m;
            }
    });
    parallel_for((int)urows.size(), [&](int a) {
        const URowX &R = urows[a];
        i64 src = R.src;
        for (int c = 0; c < R.nc; ++c) {
            const i64 d = ucd[R.c0 + c], len = ucl[R.c0 + c] + 1;
            T *m = (d >= DL0 ? mL : mU) + D[d] + R.end - len;
            for (i64 i = 0; i < len; ++i) {
                if (dir == 0) m[i] = oU[src + i];
                else oU[src + i] = m[i];
            }
            src += len;
        }
    });
}

template void Amalg::apply<double>(double *, double *, double *, double *, int) const;
template void Amalg::apply<float>(float *, float *, float *, float *, int) const;
template void Amalg::apply<std::complex<double>>(std::complex<double> *, std::complex<double> *,
                                                 std::complex<double> *, std::complex<double> *,
                                                 int) const;

} // namespace slu


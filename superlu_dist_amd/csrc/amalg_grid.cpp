// Amalgamation on process grids (amalg.h, "grids"): structure streams to the
// analysis owners, the partition, and each rank's relayout -- the structure
// of the pieces it sends, its local coarse LUstruct and the pack / unpack
// programs.  Host C++; the engine moves the streams and the values with its
// transport (engine.hip, GridAmalgPlan), the CPU tests run every rank of a
// grid in one process (amalg_api.cpp, slu_gamalg_*).
//
// Stream formats (int64):
//   phase 1, to the analysis owner of s:
//     [nL] nL x [s, nblk, nblk x (gb, nr, rows[nr])]    my blocks of L(:,s)
//     [nU] nU x [s, nub, nub x (jb, fst[w(jb)])]        my blocks of U(s,:)
//   phase 3, to the owner of the coarse block:
//     [nL] nL x [s, nblk, nblk x (gb, nr, rows[nr])]    my blocks of L(:,s) for it
//     [nU] nU x [s, jb, fst[w(jb)]]                     one block of U(s,:)
// A phase-3 L entry's values follow in the send buffer as one column-major
// (sum nr) x w(s) piece, rows in entry order; a U entry's as the block's
// segments back to back.  Senders emit L entries by local block column, U
// entries by local block row and block, receivers parse sources in rank
// order -- the order of the values in each pair's section.
#include <algorithm>
#include <complex>
#include <cstring>

#include "amalg.h"
#include "common.h"

namespace slu {

namespace {
using i64 = int64_t;
inline int Wd(const int_t *xsup, i64 k) { return (int)(xsup[k + 1] - xsup[k]); }
constexpr i64 CHUNK = 65536; // values per k_amalg_l item
} // namespace

int ga_owner(int ns, int P, int s) {
    int r = (int)std::min<i64>(P - 1, (i64)s * P / std::max(ns, 1));
    while (r + 1 < P && ga_range(ns, P, r + 1) <= s) ++r;
    while (r > 0 && ga_range(ns, P, r) > s) --r;
    return r;
}

// ------------------------------------------------------------------ phase 1
GaStreams ga_structure_out(const GaFine &f) {
    const int P = f.P();
    GaStreams Lb(P), Ub(P);
    std::vector<i64> nL(P, 0), nU(P, 0);
    for (int ljb = 0; ljb < f.nlc(); ++ljb) {
        const int_t *ix = f.lidx[ljb];
        if (!ix) continue;
        const int s = ljb * f.Pc + f.mycol, o = ga_owner(f.ns, P, s);
        std::vector<i64> &v = Lb[o];
        v.push_back(s);
        v.push_back(ix[0]);
        i64 p = SLU_BC_HEADER;
        for (i64 b = 0; b < ix[0]; ++b) {
            const i64 nr = ix[p + 1];
            v.insert(v.end(), ix + p, ix + p + SLU_LB_DESCRIPTOR + nr);
            p += SLU_LB_DESCRIPTOR + nr;
        }
        ++nL[o];
    }
    for (int lb = 0; lb < f.nlr(); ++lb) {
        const int_t *ux = f.uidx[lb];
        if (!ux) continue;
        const int s = lb * f.Pr + f.myrow, o = ga_owner(f.ns, P, s);
        std::vector<i64> &v = Ub[o];
        v.push_back(s);
        v.push_back(ux[0]);
        i64 p = SLU_BR_HEADER;
        for (i64 b = 0; b < ux[0]; ++b) {
            const i64 jb = ux[p], w = Wd(f.xsup, jb);
            v.push_back(jb);
            v.insert(v.end(), ux + p + SLU_UB_DESCRIPTOR, ux + p + SLU_UB_DESCRIPTOR + w);
            p += SLU_UB_DESCRIPTOR + w;
        }
        ++nU[o];
    }
    GaStreams out(P);
    for (int o = 0; o < P; ++o) {
        std::vector<i64> &v = out[o];
        v.reserve(2 + Lb[o].size() + Ub[o].size());
        v.push_back(nL[o]);
        v.insert(v.end(), Lb[o].begin(), Lb[o].end());
        v.push_back(nU[o]);
        v.insert(v.end(), Ub[o].begin(), Ub[o].end());
    }
    return out;
}

GaChains ga_analyse(const GaFine &f, const GaStreams &in, double zero_frac, int maxw) {
    const int P = f.P(), me = f.iam();
    const int a0 = ga_range(f.ns, P, me), a1 = ga_range(f.ns, P, me + 1), nr = a1 - a0;
    const int_t *xsup = f.xsup;
    // every block of L(:,s) / U(s,:) of my range, from whichever rank holds it
    std::vector<std::vector<const i64 *>> Lb(nr), Ub(nr);
    for (const std::vector<i64> &v : in) {
        if (v.empty()) continue;
        size_t p = 0;
        const i64 nL = v[p++];
        for (i64 e = 0; e < nL; ++e) {
            const i64 s = v[p], nb = v[p + 1];
            p += 2;
            SLU_REQUIRE(s >= a0 && s < a1, "grid amalgamation: L column %lld sent to the wrong owner", (long long)s);
            for (i64 b = 0; b < nb; ++b) {
                Lb[s - a0].push_back(&v[p]);
                p += SLU_LB_DESCRIPTOR + v[p + 1];
            }
        }
        const i64 nU = v[p++];
        for (i64 e = 0; e < nU; ++e) {
            const i64 s = v[p], nb = v[p + 1];
            p += 2;
            SLU_REQUIRE(s >= a0 && s < a1, "grid amalgamation: U row %lld sent to the wrong owner", (long long)s);
            for (i64 b = 0; b < nb; ++b) {
                Ub[s - a0].push_back(&v[p]);
                p += 1 + Wd(xsup, v[p]);
            }
        }
        SLU_REQUIRE(p == v.size(), "grid amalgamation: structure stream length");
    }
    // the 1x1 reference-format index arrays of my range (diagonal block
    // first, then blocks by block row; U blocks by block column)
    std::vector<std::vector<int_t>> lx(nr), ux(nr);
    parallel_for(nr, [&](int si) {
        const int s = a0 + si;
        std::vector<const i64 *> &L = Lb[si];
        if (!L.empty()) {
            std::sort(L.begin(), L.end(), [&](const i64 *a, const i64 *b) {
                const bool da = a[0] == s, db = b[0] == s;
                return da != db ? da : a[0] < b[0];
            });
            i64 rows = 0, len = SLU_BC_HEADER;
            for (const i64 *b : L) {
                rows += b[1];
                len += SLU_LB_DESCRIPTOR + b[1];
            }
            std::vector<int_t> &o = lx[si];
            o.reserve(len);
            o.push_back((int_t)L.size());
            o.push_back(rows);
            for (const i64 *b : L) o.insert(o.end(), b, b + SLU_LB_DESCRIPTOR + b[1]);
        }
        std::vector<const i64 *> &U = Ub[si];
        if (!U.empty()) {
            std::sort(U.begin(), U.end(), [](const i64 *a, const i64 *b) { return a[0] < b[0]; });
            const i64 end = xsup[s + 1];
            std::vector<int_t> &o = ux[si];
            o.assign(SLU_BR_HEADER, 0);
            i64 tot = 0;
            for (const i64 *b : U) {
                const int w = Wd(xsup, b[0]);
                i64 nnz = 0;
                for (int c = 0; c < w; ++c) nnz += end - b[1 + c];
                o.push_back(b[0]);
                o.push_back(nnz);
                o.insert(o.end(), b + 1, b + 1 + w);
                tot += nnz;
            }
            o[0] = (int_t)U.size();
            o[1] = tot;
            o[2] = (int_t)o.size();
            o.push_back(-1);
        }
    }, 16);
    std::vector<const int_t *> lidx(f.ns, nullptr), uidx(f.ns, nullptr);
    for (int si = 0; si < nr; ++si) {
        if (!lx[si].empty()) lidx[a0 + si] = lx[si].data();
        if (!ux[si].empty()) uidx[a0 + si] = ux[si].data();
    }
    GaChains out;
    if (nr > 0) {
        std::vector<int> gs = amalg_chains(f.n, f.ns, xsup, lidx.data(), uidx.data(), zero_frac, maxw,
                                           a0, a1, &out.fl);
        out.gstart.assign(gs.begin(), gs.end());
    }
    return out;
}

GaPartition ga_partition(const GaFine &f, const std::vector<std::vector<int64_t>> &gstarts) {
    GaPartition g;
    std::vector<i64> gs;
    for (const auto &v : gstarts) gs.insert(gs.end(), v.begin(), v.end());
    SLU_REQUIRE(!gs.empty() && gs[0] == 0, "grid amalgamation: the partition does not start at 0");
    for (size_t i = 1; i < gs.size(); ++i)
        SLU_REQUIRE(gs[i] > gs[i - 1] && gs[i] < f.ns, "grid amalgamation: group starts out of order");
    g.ns2 = (int)gs.size();
    gs.push_back(f.ns);
    g.grp.assign(f.ns, 0);
    g.xsup2.assign(g.ns2 + 1, 0);
    for (int J = 0; J < g.ns2; ++J) {
        for (i64 s = gs[J]; s < gs[J + 1]; ++s) g.grp[s] = J;
        g.xsup2[J] = f.xsup[gs[J]];
    }
    g.xsup2[g.ns2] = f.xsup[f.ns];
    g.supno2.assign(f.n, 0);
    for (int J = 0; J < g.ns2; ++J)
        for (i64 c = g.xsup2[J]; c < g.xsup2[J + 1]; ++c) g.supno2[c] = J;
    return g;
}

// ------------------------------------------------------------------ phase 3
void ga_send_side(const GaFine &f, const GaPartition &g, GaRelay &r) {
    const int P = f.P(), Pr = f.Pr, Pc = f.Pc;
    const int_t *xsup = f.xsup;
    auto owner = [&](int I, int J) { return (I % Pr) * Pc + (J % Pc); };
    // caller value layout: contiguous per local block column / row in order
    r.lsrc.assign(f.nlc() + 1, 0);
    for (int ljb = 0; ljb < f.nlc(); ++ljb) {
        const int_t *ix = f.lidx[ljb];
        r.lsrc[ljb + 1] = r.lsrc[ljb] + (ix ? (i64)ix[1] * Wd(xsup, ljb * Pc + f.mycol) : 0);
    }
    r.usrc.assign(f.nlr() + 1, 0);
    for (int lb = 0; lb < f.nlr(); ++lb) {
        const int_t *ux = f.uidx[lb];
        r.usrc[lb + 1] = r.usrc[lb] + (ux ? (i64)ux[1] : 0);
    }
    r.lval = r.lsrc[f.nlc()];
    r.uval = r.usrc[f.nlr()];
    // pass 1: values per destination
    r.scount.assign(P, 0);
    for (int ljb = 0; ljb < f.nlc(); ++ljb) {
        const int_t *ix = f.lidx[ljb];
        if (!ix) continue;
        const int s = ljb * Pc + f.mycol, w = Wd(xsup, s), J = g.grp[s];
        i64 p = SLU_BC_HEADER;
        for (i64 b = 0; b < ix[0]; ++b) {
            r.scount[owner(g.grp[ix[p]], J)] += ix[p + 1] * w;
            p += SLU_LB_DESCRIPTOR + ix[p + 1];
        }
    }
    for (int lb = 0; lb < f.nlr(); ++lb) {
        const int_t *ux = f.uidx[lb];
        if (!ux) continue;
        const int I = g.grp[lb * Pr + f.myrow];
        i64 p = SLU_BR_HEADER;
        for (i64 b = 0; b < ux[0]; ++b) {
            const int Jp = g.grp[ux[p]];
            r.scount[owner(I, Jp == I ? I : Jp)] += ux[p + 1];
            p += SLU_UB_DESCRIPTOR + Wd(xsup, ux[p]);
        }
    }
    r.soff.assign(P + 1, 0);
    for (int q = 0; q < P; ++q) r.soff[q + 1] = r.soff[q] + r.scount[q];
    SLU_REQUIRE(r.soff[P] == r.lval + r.uval, "grid amalgamation: every caller value goes somewhere");
    // pass 2: streams and pack programs
    std::vector<i64> at(r.soff.begin(), r.soff.end() - 1), nL(P, 0), nU(P, 0);
    GaStreams Ls(P), Us(P);
    std::vector<std::vector<std::pair<i64, i64>>> byq(P); // (block offset in ix, first local row)
    for (int ljb = 0; ljb < f.nlc(); ++ljb) {
        const int_t *ix = f.lidx[ljb];
        if (!ix) continue;
        const int s = ljb * Pc + f.mycol, w = Wd(xsup, s), J = g.grp[s];
        const i64 nsupr = ix[1];
        for (auto &v : byq) v.clear();
        i64 p = SLU_BC_HEADER, row = 0;
        for (i64 b = 0; b < ix[0]; ++b) {
            byq[owner(g.grp[ix[p]], J)].push_back({p, row});
            row += ix[p + 1];
            p += SLU_LB_DESCRIPTOR + ix[p + 1];
        }
        for (int q = 0; q < P; ++q) {
            if (byq[q].empty()) continue;
            std::vector<i64> &st = Ls[q];
            st.push_back(s);
            st.push_back((i64)byq[q].size());
            const i64 map = (i64)r.pack_lrow.size();
            i64 rows = 0;
            for (auto &br : byq[q]) {
                const i64 bp = br.first, nr = ix[bp + 1];
                st.insert(st.end(), ix + bp, ix + bp + SLU_LB_DESCRIPTOR + nr);
                for (i64 i = 0; i < nr; ++i) r.pack_lrow.push_back((int32_t)(br.second + i));
                rows += nr;
            }
            const int cpi = (int)std::max<i64>(1, CHUNK / std::max<i64>(rows, 1));
            for (int c0 = 0; c0 < w; c0 += cpi)
                r.pack_l.push_back({at[q], r.lsrc[ljb], map, (int32_t)rows, c0, std::min(w, c0 + cpi),
                                    (int32_t)nsupr});
            at[q] += rows * w;
            ++nL[q];
        }
    }
    for (int lb = 0; lb < f.nlr(); ++lb) {
        const int_t *ux = f.uidx[lb];
        if (!ux) continue;
        const int s = lb * Pr + f.myrow, I = g.grp[s];
        i64 p = SLU_BR_HEADER, voff = r.usrc[lb];
        for (i64 b = 0; b < ux[0]; ++b) {
            const i64 jb = ux[p], nnz = ux[p + 1];
            const int w = Wd(xsup, jb), Jp = g.grp[jb], q = owner(I, Jp == I ? I : Jp);
            std::vector<i64> &st = Us[q];
            st.push_back(s);
            st.push_back(jb);
            st.insert(st.end(), ux + p + SLU_UB_DESCRIPTOR, ux + p + SLU_UB_DESCRIPTOR + w);
            if (nnz) r.pack_u.push_back({voff, at[q], nnz});
            at[q] += nnz;
            voff += nnz;
            ++nU[q];
            p += SLU_UB_DESCRIPTOR + w;
        }
    }
    for (int q = 0; q < P; ++q)
        SLU_REQUIRE(at[q] == r.soff[q + 1], "grid amalgamation: send region %d", q);
    r.sstruct.assign(P, {});
    for (int q = 0; q < P; ++q) {
        std::vector<i64> &v = r.sstruct[q];
        v.reserve(2 + Ls[q].size() + Us[q].size());
        v.push_back(nL[q]);
        v.insert(v.end(), Ls[q].begin(), Ls[q].end());
        v.push_back(nU[q]);
        v.insert(v.end(), Us[q].begin(), Us[q].end());
    }
}

void ga_receive_side(const GaFine &f, const GaPartition &g, const GaStreams &in, GaRelay &r) {
    const int P = f.P(), Pr = f.Pr, Pc = f.Pc, myrow = f.myrow, mycol = f.mycol;
    const int_t *xsup = f.xsup;
    const int ns2 = g.ns2;
    const std::vector<int_t> &x2 = g.xsup2;
    auto W2 = [&](i64 J) { return (int)(x2[J + 1] - x2[J]); };
    r.nlc2 = (ns2 + Pc - 1) / Pc;
    r.nlr2 = (ns2 + Pr - 1) / Pr;
    SLU_REQUIRE((int)in.size() == P, "grid amalgamation: %zu streams for %d ranks", in.size(), P);
    // ---- pass A: the union of what arrives = my coarse structure
    std::vector<std::vector<std::pair<int, int32_t>>> lrows(r.nlc2); // (coarse block row, row)
    std::vector<std::vector<std::pair<int32_t, int32_t>>> ufst(r.nlr2); // (column, first row)
    r.rcount.assign(P, 0);
    for (int src = 0; src < P; ++src) {
        const std::vector<i64> &v = in[src];
        SLU_REQUIRE(!v.empty(), "grid amalgamation: empty stream from rank %d", src);
        size_t p = 0;
        const i64 nL = v[p++];
        for (i64 e = 0; e < nL; ++e) {
            const i64 s = v[p], nb = v[p + 1];
            p += 2;
            const int J = g.grp[s], w = Wd(xsup, s);
            SLU_REQUIRE(J % Pc == mycol, "grid amalgamation: L piece of column %lld on the wrong rank", (long long)s);
            i64 rows = 0;
            for (i64 b = 0; b < nb; ++b) {
                const i64 gb = v[p], nr = v[p + 1];
                const int I = g.grp[gb];
                SLU_REQUIRE(I % Pr == myrow, "grid amalgamation: L block (%lld,%lld) on the wrong rank",
                            (long long)gb, (long long)s);
                if (I != J)
                    for (i64 i = 0; i < nr; ++i) lrows[J / Pc].push_back({I, (int32_t)v[p + 2 + i]});
                rows += nr;
                p += SLU_LB_DESCRIPTOR + nr;
            }
            r.rcount[src] += rows * w;
        }
        const i64 nU = v[p++];
        for (i64 e = 0; e < nU; ++e) {
            const i64 s = v[p], jb = v[p + 1];
            p += 2;
            const int I = g.grp[s], Jp = g.grp[jb], w = Wd(xsup, jb);
            const i64 end = xsup[s + 1];
            SLU_REQUIRE(I % Pr == myrow && (Jp == I ? I : Jp) % Pc == mycol,
                        "grid amalgamation: U block (%lld,%lld) on the wrong rank", (long long)s, (long long)jb);
            for (int c = 0; c < w; ++c) {
                const i64 fst = v[p + c];
                if (fst < end) {
                    r.rcount[src] += end - fst;
                    if (Jp != I) ufst[I / Pr].push_back({(int32_t)(xsup[jb] + c), (int32_t)fst});
                }
            }
            p += w;
        }
        SLU_REQUIRE(p == v.size(), "grid amalgamation: relay stream length from rank %d", src);
    }
    r.roff.assign(P + 1, 0);
    for (int q = 0; q < P; ++q) r.roff[q + 1] = r.roff[q] + r.rcount[q];
    r.received = r.roff[P];

    // ---- local coarse L block columns: diagonal block (where mine), then
    // block rows ascending, rows ascending within each
    r.Lidx2.assign(r.nlc2, {});
    r.Lvoff2.assign(r.nlc2, -1);
    std::vector<int64_t> lnsupr(r.nlc2, 0);
    parallel_for(r.nlc2, [&](int lj) {
        const int J = lj * Pc + mycol;
        if (J >= ns2) return;
        auto &rw = lrows[lj];
        std::sort(rw.begin(), rw.end());
        rw.erase(std::unique(rw.begin(), rw.end()), rw.end());
        const bool diag = J % Pr == myrow;
        if (!diag && rw.empty()) return;
        std::vector<int_t> &o = r.Lidx2[lj];
        o.assign(SLU_BC_HEADER, 0);
        i64 nblk = 0, rows = 0;
        if (diag) {
            o.push_back(J);
            o.push_back(W2(J));
            for (i64 c = x2[J]; c < x2[J + 1]; ++c) o.push_back(c);
            ++nblk;
            rows += W2(J);
        }
        for (size_t i = 0; i < rw.size();) {
            const int I = rw[i].first;
            const size_t d = o.size();
            o.push_back(I);
            o.push_back(0);
            while (i < rw.size() && rw[i].first == I) o.push_back(rw[i++].second);
            o[d + 1] = (int_t)(o.size() - d - SLU_LB_DESCRIPTOR);
            rows += o[d + 1];
            ++nblk;
        }
        o[0] = nblk;
        o[1] = rows;
        lnsupr[lj] = rows;
    }, 16);
    r.lval2 = 0;
    for (int lj = 0; lj < r.nlc2; ++lj)
        if (!r.Lidx2[lj].empty()) {
            r.Lvoff2[lj] = r.lval2;
            r.lval2 += lnsupr[lj] * W2(lj * Pc + mycol);
        }
    // ---- local coarse U block rows: blocks by block column, every column of
    // a block, first row = min over the arriving segments (empty: end)
    r.Uidx2.assign(r.nlr2, {});
    r.Uvoff2.assign(r.nlr2, -1);
    std::vector<i64> ucols(r.nlr2 + 1, 0), ulen(r.nlr2, 0);
    std::vector<std::vector<std::pair<int, i64>>> ublk(r.nlr2); // (block column, first column entry in row)
    parallel_for(r.nlr2, [&](int li) {
        const int I = li * Pr + myrow;
        if (I >= ns2) return;
        auto &uf = ufst[li];
        if (uf.empty()) return;
        std::sort(uf.begin(), uf.end()); // by column, then first row: the first is the minimum
        const i64 endI = x2[I + 1];
        std::vector<int_t> &o = r.Uidx2[li];
        o.assign(SLU_BR_HEADER, 0);
        i64 nblk = 0, tot = 0, ce = 0;
        for (size_t i = 0; i < uf.size();) {
            const int Jp = g.supno2[uf[i].first];
            const size_t d = o.size();
            o.push_back(Jp);
            o.push_back(0);
            ublk[li].push_back({Jp, ce});
            i64 nnz = 0;
            for (i64 c = x2[Jp]; c < x2[Jp + 1]; ++c) {
                i64 fst = endI;
                if (i < uf.size() && uf[i].first == c) {
                    fst = uf[i].second;
                    while (i < uf.size() && uf[i].first == c) ++i;
                }
                o.push_back(fst);
                nnz += endI - fst;
            }
            o[d + 1] = nnz;
            tot += nnz;
            ce += W2(Jp);
            ++nblk;
        }
        o[0] = nblk;
        o[1] = tot;
        o[2] = (int_t)o.size();
        o.push_back(-1);
        ulen[li] = tot;
        ucols[li + 1] = ce;
    }, 16);
    for (int li = 0; li < r.nlr2; ++li) ucols[li + 1] += ucols[li];
    r.uval2 = 0;
    for (int li = 0; li < r.nlr2; ++li)
        if (!r.Uidx2[li].empty()) {
            r.Uvoff2[li] = r.uval2;
            r.uval2 += ulen[li];
        }
    // D: U-kind entries per local coarse U column entry, then L-kind per
    // global column (diagonal blocks that are mine)
    r.DL0 = ucols[r.nlr2];
    SLU_REQUIRE(r.DL0 + f.n < (1ll << 31), "grid amalgamation: destination table exceeds int32");
    r.D.assign(r.DL0 + f.n, 0);
    parallel_for(r.nlr2, [&](int li) {
        if (r.Uidx2[li].empty()) return;
        const int I = li * Pr + myrow;
        const i64 endI = x2[I + 1];
        const int_t *o = r.Uidx2[li].data();
        i64 p = SLU_BR_HEADER, d = ucols[li], seg = r.Uvoff2[li];
        for (i64 b = 0; b < o[0]; ++b) {
            const int Jp = (int)o[p];
            for (int c = 0; c < W2(Jp); ++c, ++d) {
                const i64 fst = o[p + SLU_UB_DESCRIPTOR + c];
                r.D[d] = seg - fst;
                seg += endI - fst;
            }
            p += SLU_UB_DESCRIPTOR + W2(Jp);
        }
    }, 16);
    for (int lj = 0; lj < r.nlc2; ++lj) {
        const int J = lj * Pc + mycol;
        if (J >= ns2 || J % Pr != myrow || r.Lidx2[lj].empty()) continue;
        for (i64 c = x2[J]; c < x2[J + 1]; ++c)
            r.D[r.DL0 + c] = r.Lvoff2[lj] + (c - x2[J]) * lnsupr[lj] - x2[J];
    }
    // ---- pass B: unpack programs, sources in rank order
    // per local coarse column: block row -> (offset in Lidx2, position of its
    // first row); ascending (the diagonal block J comes first, every other
    // block row of L(:,J) is below it)
    std::vector<std::vector<std::pair<int, std::pair<i64, i64>>>> lbk(r.nlc2);
    for (int lj = 0; lj < r.nlc2; ++lj) {
        const std::vector<int_t> &o = r.Lidx2[lj];
        if (o.empty()) continue;
        i64 p = SLU_BC_HEADER, pos = 0;
        for (i64 b = 0; b < o[0]; ++b) {
            lbk[lj].push_back({(int)o[p], {p, pos}});
            pos += o[p + 1];
            p += SLU_LB_DESCRIPTOR + o[p + 1];
        }
    }
    for (int src = 0; src < P; ++src) {
        const std::vector<i64> &v = in[src];
        size_t p = 0;
        i64 off = r.roff[src];
        const i64 nL = v[p++];
        for (i64 e = 0; e < nL; ++e) {
            const i64 s = v[p], nb = v[p + 1];
            p += 2;
            const int J = g.grp[s], lj = J / Pc, w = Wd(xsup, s);
            const i64 map = (i64)r.unpack_lrow.size();
            i64 rows = 0;
            for (i64 b = 0; b < nb; ++b) {
                const i64 gb = v[p], nr = v[p + 1];
                const int I = g.grp[gb];
                if (I == J) {
                    for (i64 i = 0; i < nr; ++i) r.unpack_lrow.push_back((int32_t)(v[p + 2 + i] - x2[J]));
                } else {
                    const auto &bk = lbk[lj];
                    auto it = std::lower_bound(bk.begin(), bk.end(), I,
                                               [](const std::pair<int, std::pair<i64, i64>> &a, int k) { return a.first < k; });
                    SLU_REQUIRE(it != bk.end() && it->first == I, "grid amalgamation: coarse block (%d,%d) missing", I, J);
                    const int_t *rb = r.Lidx2[lj].data() + it->second.first + SLU_LB_DESCRIPTOR;
                    const i64 bnr = r.Lidx2[lj][it->second.first + 1];
                    for (i64 i = 0; i < nr; ++i) {
                        const int_t row = v[p + 2 + i];
                        const int_t *q = std::lower_bound(rb, rb + bnr, row);
                        SLU_REQUIRE(q != rb + bnr && *q == row, "grid amalgamation: row not in coarse block");
                        r.unpack_lrow.push_back((int32_t)(it->second.second + (q - rb)));
                    }
                }
                rows += nr;
                p += SLU_LB_DESCRIPTOR + nr;
            }
            const int cpi = (int)std::max<i64>(1, CHUNK / std::max<i64>(rows, 1));
            const i64 dst = r.Lvoff2[lj] + (xsup[s] - x2[J]) * lnsupr[lj];
            for (int c0 = 0; c0 < w; c0 += cpi)
                r.unpack_l.push_back({off, dst, map, (int32_t)rows, c0, std::min(w, c0 + cpi), (int32_t)lnsupr[lj]});
            off += rows * w;
        }
        const i64 nU = v[p++];
        for (i64 e = 0; e < nU; ++e) {
            const i64 s = v[p], jb = v[p + 1];
            p += 2;
            const int I = g.grp[s], Jp = g.grp[jb], w = Wd(xsup, jb), li = I / Pr;
            const i64 end = xsup[s + 1];
            i64 ce0 = -1;
            if (Jp != I) {
                const auto &bk = ublk[li];
                auto it = std::lower_bound(bk.begin(), bk.end(), Jp,
                                           [](const std::pair<int, i64> &a, int k) { return a.first < k; });
                SLU_REQUIRE(it != bk.end() && it->first == Jp, "grid amalgamation: coarse U block (%d,%d) missing", I, Jp);
                ce0 = ucols[li] + it->second + (xsup[jb] - x2[Jp]);
            }
            // chunks of <= 64 non-empty columns
            int nc = 0;
            for (int c = 0; c < w; ++c) {
                const i64 fst = v[p + c];
                if (fst >= end) continue;
                if (nc == 0) r.unpack_u.push_back({off, (i64)r.unpack_ucd.size(), 0, (int32_t)end});
                const i64 didx = Jp == I ? r.DL0 + xsup[jb] + c : ce0 + c;
                r.unpack_ucd.push_back((int32_t)didx);
                SLU_REQUIRE(end - fst <= 65536, "grid amalgamation: U segment of %lld rows (> 65536)",
                            (long long)(end - fst));
                r.unpack_ucl.push_back((uint16_t)(end - fst - 1));
                off += end - fst;
                r.unpack_u.back().nc = ++nc;
                if (nc == 64) nc = 0;
            }
            p += w;
        }
        SLU_REQUIRE(off == r.roff[src + 1], "grid amalgamation: receive region %d", src);
    }
}

// ------------------------------------------------------------------ host programs
template <typename T> void ga_pack(const GaRelay &r, T *cL, T *cU, T *send, int dir) {
    parallel_for((int)r.pack_l.size(), [&](int k) {
        const LColX &x = r.pack_l[k];
        for (int c = x.c0; c < x.c1; ++c)
            for (int i = 0; i < x.nsupr; ++i) {
                T *o = send + x.src + (i64)c * x.nsupr + i;
                T *m = cL + x.dst + (i64)c * x.ld2 + r.pack_lrow[x.map + i];
                if (dir == 0) *o = *m;
                else *m = *o;
            }
    });
    parallel_for((int)r.pack_u.size(), [&](int k) {
        const GaSpan &x = r.pack_u[k];
        for (i64 i = 0; i < x.len; ++i) {
            if (dir == 0) send[x.dst + i] = cU[x.src + i];
            else cU[x.src + i] = send[x.dst + i];
        }
    });
}

template <typename T> void ga_unpack(const GaRelay &r, T *recv, T *mL, T *mU, int dir) {
    parallel_for((int)r.unpack_l.size(), [&](int k) {
        const LColX &x = r.unpack_l[k];
        for (int c = x.c0; c < x.c1; ++c)
            for (int i = 0; i < x.nsupr; ++i) {
                T *o = recv + x.src + (i64)c * x.nsupr + i;
                T *m = mL + x.dst + (i64)c * x.ld2 + r.unpack_lrow[x.map + i];
                if (dir == 0) *m = *o;
                else *o = *m;
            }
    });
    parallel_for((int)r.unpack_u.size(), [&](int k) {
        const UChunk &x = r.unpack_u[k];
        i64 src = x.src;
        for (int c = 0; c < x.nc; ++c) {
            const i64 d = r.unpack_ucd[x.c0 + c], len = r.unpack_ucl[x.c0 + c] + 1;
            T *m = (d >= r.DL0 ? mL : mU) + r.D[d] + x.end - len;
            for (i64 i = 0; i < len; ++i) {
                if (dir == 0) m[i] = recv[src + i];
                else recv[src + i] = m[i];
            }
            src += len;
        }
    });
}

template void ga_pack<double>(const GaRelay &, double *, double *, double *, int);
template void ga_pack<float>(const GaRelay &, float *, float *, float *, int);
template void ga_pack<std::complex<double>>(const GaRelay &, std::complex<double> *, std::complex<double> *,
                                            std::complex<double> *, int);
template void ga_unpack<double>(const GaRelay &, double *, double *, double *, int);
template void ga_unpack<float>(const GaRelay &, float *, float *, float *, int);
template void ga_unpack<std::complex<double>>(const GaRelay &, std::complex<double> *, std::complex<double> *,
                                              std::complex<double> *, int);

} // namespace slu

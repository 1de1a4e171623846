// Column ordering post-pass and symbolic factorization:
// the two serial steps pdgssvx runs between the column ordering and
// pddistribute (SRC/pdgssvx.c:1046-1076):
//
//   sp_colorder  SRC/sp_colorder.c:81-221   etree of Pc(A'+A)Pc' (or the
//                column etree of A Pc'), its postorder folded into perm_c,
//                A's columns permuted to A Pc'
//   symbfact     SRC/symbfact.c:81-215      supernodal symbolic LU without
//                pivoting: relaxed leaf supernodes, per-column depth-first
//                search over the pruned graph of L, fundamental supernode
//                detection, symmetric pruning; L subscripts per supernode,
//                U segments ("skeleton") per column
//
// Both give the reference's arrays exactly (tests/test_symbolic.py against
// goldens of the reference run on the same inputs): the depth-first search
// order decides the order of each supernode's L subscripts, and pddistribute
// lays the factor blocks out in that order.
#include <algorithm>
#include <atomic>
#include <memory>
#include <chrono>
#include <cstdio>
#include <cstdint>
#include <cstdlib>
#include <cstring>
#include <stdexcept>
#include <string>
#include <type_traits>
#include <vector>

#include "common.h"
#include "noinit_vec.h"
#include "slu_abi.h"

// csrc/symbolic_dev.hip (the full library links both)
bool slu_symb_epilogue_dev(int64_t n, int64_t nsup, const int32_t *raw, int64_t raw_len, const int64_t *xlsub_raw,
                           const int32_t *xsup, const int32_t *supno, const int32_t *usub, int64_t nu,
                           slu::i64_vec &lsub, std::vector<int64_t> &xlsub, int64_t *nnzL, int64_t *nnzU,
                           std::string &err);
bool slu_symb_have_device();

namespace slu {
namespace symb {

using I = int64_t;

// where the last symbfact ran its epilogue (countnz + fixupL): 0 host, 1 device
static int g_last_epilogue = 0;

// SLU_SYMB_DEVICE=1: the epilogue on the GPU (an error without one); else on
// the host threads, for every caller.  (Round 6: the host epilogue on the
// host threads with uninitialised index storage takes 0.34 s at 100^3 in the
// build container, 1.8 s before; the device one cost 0.67 s on the box, most
// of it initialising HIP from inside the symbolic phase.)  The search stays
// on the host either way.
static bool use_device_epilogue(I m, I n, I nsup, bool dev_default) {
    (void)nsup;
    (void)dev_default;
    const char *e = getenv("SLU_SYMB_DEVICE");
    if (e && atoi(e) != 0) {
        if (!slu_symb_have_device()) throw Error("symbfact: SLU_SYMB_DEVICE=1 but no GPU is visible");
        return m == n;
    }
    return false;
}
using std::vector;
constexpr I NONE = -1;

// ---------------------------------------------------------------- etree ---
// Elimination tree of a symmetric pattern given column by column through
// `cols(k, f)` calling f(i) for the (permuted) row indices of column k;
// entries with i >= k are ignored (SRC/etree.c:156-200 uses the upper
// triangle the same way).  The tree is unique; ancestor path compression
// instead of the reference's disjoint sets.
template <class Cols>
static void etree_liu(I n, Cols cols, I *parent) {
    vector<I> anc(n, NONE);
    for (I k = 0; k < n; ++k) {
        parent[k] = n;
        cols(k, [&](I i) {
            if (i >= k) return;
            I r = i;
            while (anc[r] != NONE && anc[r] != k) {
                const I nx = anc[r];
                anc[r] = k;
                r = nx;
            }
            if (anc[r] == NONE) {
                anc[r] = k;
                parent[r] = k;
            }
        });
    }
}

// Postorder of a forest given by parent pointers (roots point at n), children
// visited in increasing order: post[v] = position of v (SRC/etree.c:393-430
// returns the same inverse numbering).  post has n + 1 entries, post[n] = n.
static vector<I> postorder(I n, const I *parent) {
    vector<I> head(n + 1, NONE), next(n + 1, NONE), post(n + 1, 0), stack;
    for (I v = n - 1; v >= 0; --v) {
        next[v] = head[parent[v]];
        head[parent[v]] = v;
    }
    I num = 0;
    stack.reserve(64);
    stack.push_back(n);
    while (!stack.empty()) {
        const I v = stack.back();
        if (head[v] != NONE) {
            const I c = head[v];
            head[v] = next[c]; // next child of v on the next visit
            stack.push_back(c);
        } else {
            post[v] = num++;
            stack.pop_back();
        }
    }
    return post;
}

// sp_colorder (SRC/sp_colorder.c:81-221).  colbeg / colend receive A Pc''s
// column pointers; with recompute (Fact = DOFACT or SamePattern) the etree
// is recomputed and perm_c / etree / colbeg / colend follow its postorder.
static void colorder(I m, I n, const I *colptr, const I *rowind, bool ata, bool recompute,
                     I *perm_c, I *etree, I *colbeg, I *colend) {
    for (I i = 0; i < n; ++i) {
        colbeg[perm_c[i]] = colptr[i];
        colend[perm_c[i]] = colptr[i + 1];
    }
    if (!recompute) return;
    if (m != n || ata) {
        // column etree of A Pc' (SRC/etree.c:223-286): row r's edges replaced
        // by a star centred at its first column
        vector<I> first(m, n);
        for (I c = 0; c < n; ++c)
            for (I p = colbeg[c]; p < colend[c]; ++p) first[rowind[p]] = std::min(first[rowind[p]], c);
        etree_liu(n, [&](I k, auto f) {
            for (I p = colbeg[k]; p < colend[k]; ++p) f(first[rowind[p]]);
        }, etree);
    } else {
        // etree of Pc (A' + A) Pc': column k of the sum = column c = iperm[k]
        // of A and row c of A (A' column c), both relabelled by perm_c
        vector<I> iperm(n), tptr(n + 1, 0), tind(colptr[n]);
        for (I i = 0; i < n; ++i) iperm[perm_c[i]] = i;
        for (I p = 0; p < colptr[n]; ++p) tptr[rowind[p] + 1]++;
        for (I r = 0; r < n; ++r) tptr[r + 1] += tptr[r];
        {
            vector<I> at(tptr.begin(), tptr.end() - 1);
            for (I c = 0; c < n; ++c)
                for (I p = colptr[c]; p < colptr[c + 1]; ++p) tind[at[rowind[p]]++] = c;
        }
        etree_liu(n, [&](I k, auto f) {
            const I c = iperm[k];
            for (I p = colptr[c]; p < colptr[c + 1]; ++p) f(perm_c[rowind[p]]);
            for (I p = tptr[c]; p < tptr[c + 1]; ++p) f(perm_c[tind[p]]);
        }, etree);
    }
    const vector<I> post = postorder(n, etree);
    vector<I> w(n);
    for (I i = 0; i < n; ++i) w[post[i]] = post[etree[i]];
    std::copy(w.begin(), w.end(), etree);
    for (I i = 0; i < n; ++i) w[post[i]] = colbeg[i];
    std::copy(w.begin(), w.end(), colbeg);
    for (I i = 0; i < n; ++i) w[post[i]] = colend[i];
    std::copy(w.begin(), w.end(), colend);
    for (I i = 0; i < n; ++i) perm_c[i] = post[perm_c[i]];
}

// ------------------------------------------------------------ symbfact ---
// Last column of the relaxed supernode starting at each column, NONE
// elsewhere: maximal subtrees of the postordered etree with fewer than
// `relax` descendants (SRC/symbfact.c:227-271).
static vector<I> relaxed_ends(I n, const I *et, I relax) {
    vector<I> desc(n + 1, 0), end(n, NONE);
    for (I j = 0; j < n; ++j)
        if (et[j] != n) desc[et[j]] += desc[j] + 1;
    for (I j = 0; j < n;) {
        const I f = j;
        while (et[j] != n && desc[et[j]] < relax) j = et[j];
        end[f] = j;
        ++j;
        while (j < n && desc[j] != 0) ++j;
    }
    return end;
}

struct Result {
    I n = 0;
    vector<I> xsup, supno, xlsub, xusub;
    i64_vec lsub, usub; // (filled on the host threads or by the device epilogue's copy)
    I nnzL = 0, nnzU = 0, nnzLU = 0, lsub_size = 0;
};

// The symbolic factorization state: the reference's Glu_persist /
// Glu_freeable arrays and its work arrays (SRC/symbfact.c:115-131).  Row and
// column indices in T (int32 when n fits: the search is bound by random
// accesses into marker / supno / lsub), positions in lsub / usub in I.
// Pivots are diagonal (pivotL, SRC/symbfact.c:729-731), so the reference's
// perm_r is the identity on the columns done so far: "row r pivoted" is
// r < j while column j is searched, r <= j while it prunes.
#ifdef SLU_SYMB_COUNT
static long long g_cnt[8];
#define SYMB_CNT(i, v) (g_cnt[i] += (v))
#else
#define SYMB_CNT(i, v) ((void)0)
#endif
template <class T>
struct Walker {
    // input: A Pc' with rows relabelled by perm_c (NCP)
    const I *cb, *ce;
    const T *ri;
    I maxsuper;
    vector<T> xsup, supno, marker, repfnz, parent, segrep;
    std::vector<T, NoInit<T>> lsub, usub; // (grown without zeroing: written before read)
    vector<I> xlsub, xusub, xprune, xplore;
    I nextu = 0;

    Walker(I m, I n, I cap) : xsup(n + 2, 0), supno(n + 1, 0), marker(m, (T)NONE),
                              repfnz(m, (T)NONE), parent(m, 0), segrep(m, 0), lsub(cap),
                              usub(cap / 2 + 1024), xlsub(n + 1, 0), xusub(n + 1, 0),
                              xprune(n, 0), xplore(m, 0) {
        supno[0] = (T)NONE;
    }

    I m = 0;
    // room for `more` entries past `at`: checked once per column (a column's
    // list has at most m entries), not per entry
    void reserve(I at, I more) {
        if (at + more > (I)lsub.size()) lsub.resize(std::max<I>(2 * lsub.size(), at + more + 1024));
    }
    void lput(I at, T v) { lsub[at] = v; }

    // relaxed supernode j..k: union of the columns' row structures, a copy
    // of it for pruning when k > j (SRC/symbfact.c:291-370)
    void relaxed(I j, I k) {
        const T ns = ++supno[j];
        I nextl = xlsub[j];
        reserve(nextl, 2 * m);
        for (I i = j; i <= k; ++i) {
            for (I p = cb[i]; p < ce[i]; ++p) {
                const T r = ri[p];
                if (marker[r] != (T)k) {
                    marker[r] = (T)k;
                    lput(nextl++, r);
                }
            }
            supno[i] = ns;
            xusub[i + 1] = nextu;
        }
        if (j < k) {
            I to = nextl;
            for (I f = xlsub[j]; f < nextl; ++f) lput(to++, lsub[f]);
            for (I i = j + 1; i <= k; ++i) xlsub[i] = nextl;
            nextl = to;
        }
        xsup[ns + 1] = (T)(k + 1);
        supno[k + 1] = ns;
        xprune[k] = nextl;
        xlsub[k + 1] = nextl;
    }

    // depth-first search of column j over the pruned graph; returns the
    // number of U segments (representatives in segrep, in the order the
    // search finishes them) and decides whether j extends j-1's supernode
    // (SRC/symbfact.c:458-671)
    I column(I j) {
        const T tj = (T)j, tj1 = (T)(j - 1);
        I ns = supno[j], nextl = xlsub[j], nseg = 0;
        bool js = true; // j joins j-1's supernode
        reserve(nextl, m);
        // local copies of the arrays the search touches (registers, no reloads)
        T *const L = lsub.data(), *const mk = marker.data(), *const rf = repfnz.data(),
                 *const par = parent.data(), *const sg = segrep.data();
        const T *const xs = xsup.data(), *const sn = supno.data();
        const I *const xl = xlsub.data(), *const xp = xprune.data();
        I *const xo = xplore.data();
        for (I p = cb[j]; p < ce[j]; ++p) {
            const T r = ri[p], km = mk[r];
            if (km == tj) continue;
            mk[r] = tj;
            if (r >= tj) { // row not pivoted yet: in L(:, j)
                L[nextl++] = r;
                if (km != tj1) js = false;
                continue;
            }
            T rep = xs[sn[r] + 1] - 1;
            if (rf[rep] != (T)NONE) {
                if (r < rf[rep]) rf[rep] = r;
                continue;
            }
            par[rep] = (T)NONE;
            rf[rep] = r;
            I x = xl[rep], xe = xp[rep];
            for (;;) {
                while (x < xe) {
                    const T c = L[x++], cm = mk[c];
                    if (cm == tj) continue;
                    mk[c] = tj;
                    if (c >= tj) {
                        L[nextl++] = c;
                        if (cm != tj1) js = false;
                        continue;
                    }
                    const T crep = xs[sn[c] + 1] - 1;
                    if (rf[crep] != (T)NONE) {
                        if (c < rf[crep]) rf[crep] = c;
                        continue;
                    }
                    xo[rep] = x; // descend
                    par[crep] = rep;
                    rep = crep;
                    rf[rep] = c;
                    x = xl[rep];
                    xe = xp[rep];
                }
                sg[nseg++] = rep; // finished: back to the parent
                const T up = par[rep];
                if (up == (T)NONE) break;
                rep = up;
                x = xo[rep];
                xe = xp[rep];
            }
        }
        if (j == 0) {
            ns = supno[0] = 0;
        } else {
            const I fs = xsup[ns], jp = xlsub[j], jm1p = xlsub[j - 1];
            // fundamental supernodes: |L(:,j)| = |L(:,j-1)| - 1 besides the
            // subset test (T2_SUPER, SRC/symbfact.c:39,633-635), and at most
            // maxsuper columns
            if (nextl - jp != jp - jm1p - 1) js = false;
            if (j - fs >= maxsuper) js = false;
            if (!js) {
                if (fs < j - 2) { // >= 3 columns: keep only the first and last lists
                    I to = xlsub[fs + 1];
                    xlsub[j - 1] = to;
                    const I stop = to + jp - jm1p;
                    xprune[j - 1] = stop;
                    xlsub[j] = stop;
                    for (I f = jm1p; f < nextl; ++f, ++to) lsub[to] = lsub[f];
                    nextl = to;
                }
                ++ns;
                supno[j] = (T)ns;
            }
        }
        xsup[ns + 1] = (T)(j + 1);
        supno[j + 1] = (T)ns;
        xprune[j] = nextl;
        xlsub[j + 1] = nextl;
        return nseg;
    }

    // U segments of column j, in topological order (SRC/symbfact.c:763-820)
    void set_usub(I j, I nseg) {
        const T js = supno[j];
        for (I s = nseg - 1; s >= 0; --s) {
            const T rep = segrep[s];
            if (supno[rep] == js || repfnz[rep] == (T)NONE) continue;
            if (nextu >= (I)usub.size()) usub.resize(std::max<I>(2 * usub.size(), nextu + 1024));
            usub[nextu++] = repfnz[rep];
        }
        xusub[j + 1] = nextu;
    }

    // diagonal row of column j to position j - fsupc of its supernode's
    // first list (SRC/symbfact.c:684-742)
    void pivot(I j) {
        const I fs = xsup[supno[j]], lp = xlsub[fs], nr = xlsub[fs + 1] - lp, d0 = j - fs;
        I d = NONE;
        for (I s = d0; s < nr; ++s)
            if (lsub[lp + s] == (T)j) {
                d = s;
                break;
            }
        if (d == NONE) throw Error("symbfact: zero diagonal at column " + std::to_string(j));
        if (d != d0) std::swap(lsub[lp + d], lsub[lp + d0]);
    }

    // symmetric pruning of the supernodes column j's search reached
    // (SRC/symbfact.c:824-906); rows <= j are pivoted now
    void prune(I j, I nseg) {
        const T js = supno[j], tj = (T)j;
        for (I s = 0; s < nseg; ++s) {
            const T rep = segrep[s];
            if (repfnz[rep] == (T)NONE || supno[rep] == js) continue;
            if (xprune[rep] < xlsub[rep + 1]) continue; // pruned before
            I lo = xlsub[rep], hi = xlsub[rep + 1] - 1;
            SYMB_CNT(1, hi - lo + 1);
            bool hit = false;
            for (I q = lo; q <= hi; ++q)
                if (lsub[q] == tj) {
                    hit = true;
                    break;
                }
            if (!hit) continue;
            while (lo <= hi) {
                if (lsub[hi] > tj)
                    --hi;
                else if (lsub[lo] <= tj)
                    ++lo;
                else {
                    std::swap(lsub[lo], lsub[hi]);
                    ++lo;
                    --hi;
                }
            }
            xprune[rep] = lo;
        }
    }

    // ---------------------------------------------------------------------
    // The same state machine with the current supernode's last list kept
    // virtual (the default; SLU_SYMB_CLASSIC=1 runs column() above).
    //
    // Column j's search reaches the supernode it may extend through that
    // supernode's representative j - 1, whose list is L(:, j-1), and appends
    // every row >= j of it that is not yet marked: at 100^3 that re-scan is
    // 95 % of the search (1.52e9 of 1.59e9 entries, each column of a wide
    // supernode copying the whole front).  Here L(:, j-1) lives in a linked
    // list (lnx / lpv) with membership stamps (cur[r] == its supernode), and
    // entering j - 1 only records where its rows go: L(:, j) is
    //   P ++ (L(:, j-1) minus {j-1} minus P, in its order) ++ Q
    // with P / Q the rows found before / after (Q is empty when j joins).  A
    // column that joins moves P to the front of the linked list and drops
    // j - 1; one that starts a new supernode writes the old supernode's last
    // list and its own list out in full, where the classic compaction puts
    // them (first list, last list; SRC/symbfact.c:633-671).  Every array and
    // the returned lsub size are the classic ones (tests/test_symbolic.py).
    vector<T> cur, lnx, lpv, fl, pos;
    vector<T> repc; // representative of each row's finished supernode (NONE: the current one)
    T lhead = (T)NONE, ltail = (T)NONE, cur_s = (T)-2; // cur_s: supernode of the list
    I cur_fs = 0, last_len = 0, tail_sum = 0;          // tail_sum: classic sizes past the first list
    I lbelow = 0; // rows of the list below the next column (1; a relaxed copy: its width)
    T lmin = 0;   // smallest row of the list (the representative's first nonzero row bound)
    // no current supernode: the one before column j was closed by close_at(j)
    // (a subtree task's first column, or the column after an imported task)
    bool closed = false;

    void vinit() {
        cur.assign(m, (T)-3);
        fl.assign(m, (T)-3);
        lnx.assign(m, (T)NONE);
        lpv.assign(m, (T)NONE);
        pos.assign(m, 0);
        repc.assign(m, (T)NONE);
    }
    void set_rep(I fs, I last) {
        for (I c = fs; c <= last; ++c) repc[c] = (T)last;
    }
    void l_unlink(T c) {
        const T a = lpv[c], b = lnx[c];
        if (a != (T)NONE) lnx[a] = b;
        else lhead = b;
        if (b != (T)NONE) lpv[b] = a;
        else ltail = a;
    }
    void l_push_front(T c) {
        lpv[c] = (T)NONE;
        lnx[c] = lhead;
        if (lhead != (T)NONE) lpv[lhead] = c;
        else ltail = c;
        lhead = c;
    }
    void l_build(const T *v, I cnt) {
        lhead = ltail = (T)NONE;
        for (I i = cnt - 1; i >= 0; --i) l_push_front(v[i]);
    }
    // the supernode starting at fs, whose search representative is rep:
    // its list (the rep's) into the linked list, its first list's positions
    void start_supernode(I fs, I rep) {
        const T s = supno[fs];
        const I a = xlsub[rep], b = xprune[rep];
        l_build(lsub.data() + a, b - a);
        for (I i = a; i < b; ++i) cur[lsub[i]] = s;
        const I fa = xlsub[fs], fb = xlsub[fs + 1];
        for (I i = fa; i < fb; ++i) {
            fl[lsub[i]] = s;
            pos[lsub[i]] = i - fa;
        }
        cur_s = s;
        cur_fs = fs;
        closed = false;
        last_len = b - a;
        tail_sum = rep > fs ? b - a : 0;
        lbelow = 0;
        lmin = (T)m;
        for (I i = a; i < b; ++i) {
            if (lsub[i] <= (T)rep) ++lbelow;
            lmin = std::min(lmin, lsub[i]);
        }
    }
    // write the linked list (L(:, j-1)) at `at`, skipping rows below `below`
    // and rows marked `mark`; returns the count written
    I l_write(I at, T below, T mark) {
        I o = at;
        SYMB_CNT(2, last_len);
        for (T c = lhead; c != (T)NONE; c = lnx[c])
            if (c >= below && marker[c] != mark) lsub[o++] = c;
        return o - at;
    }

    I column_v(I j) {
        const T tj = (T)j;
        I ns = supno[j];
        const bool prev = j > 0 && !closed; // a current supernode (columns cur_fs .. j-1) exists
        const T sc = prev ? cur_s : (T)-2;
        const I start = !prev ? xlsub[j] : (j - 1 > cur_fs ? xlsub[cur_fs + 1] + last_len : xlsub[cur_fs + 1]);
        I nextl = start, nseg = 0, split = -1, p_in = 0;
        bool subset = true;
        reserve(start, m + 1);
        T *const L = lsub.data(), *const mk = marker.data(), *const rf = repfnz.data(),
                 *const par = parent.data(), *const sg = segrep.data(), *const cu = cur.data();
        const T *const rc = repc.data();
        const I *const xl = xlsub.data(), *const xp = xprune.data();
        I *const xo = xplore.data();
        const T vrep = prev ? (T)(j - 1) : (T)NONE; // the representative kept virtual
        // entering the virtual representative: its rows >= j count as found
        // from here on; its rows < j (the representative's own, all of a
        // relaxed supernode's) would each lower repfnz to their index
        auto enter_virtual = [&]() {
            split = nextl - start;
            if (lmin < rf[vrep]) rf[vrep] = lmin;
        };
        for (I p = cb[j]; p < ce[j]; ++p) {
            const T r = ri[p], km = mk[r];
            if (km == tj) continue;
            if (r >= tj) {
                if (split >= 0 && cu[r] == sc) continue; // in the virtual part
                mk[r] = tj;
                L[nextl++] = r;
                if (cu[r] == sc) ++p_in;
                else subset = false;
                continue;
            }
            mk[r] = tj;
            T rep = rc[r];
            if (rep == (T)NONE) rep = vrep;
            if (rf[rep] != (T)NONE) {
                if (r < rf[rep]) rf[rep] = r;
                continue;
            }
            par[rep] = (T)NONE;
            rf[rep] = r;
            I x = xl[rep], xe = xp[rep];
            if (rep == vrep) {
                enter_virtual();
                x = xe = 0;
            }
            for (;;) {
                SYMB_CNT(0, xe - x);
                while (x < xe) {
                    const T c = L[x++], cm = mk[c];
                    if (cm == tj) continue;
                    if (c >= tj) {
                        if (split >= 0 && cu[c] == sc) continue;
                        mk[c] = tj;
                        L[nextl++] = c;
                        if (cu[c] == sc) ++p_in;
                        else subset = false;
                        continue;
                    }
                    mk[c] = tj;
                    T crep = rc[c];
                    if (crep == (T)NONE) crep = vrep;
                    if (rf[crep] != (T)NONE) {
                        if (c < rf[crep]) rf[crep] = c;
                        continue;
                    }
                    xo[rep] = x; // descend
                    par[crep] = rep;
                    rep = crep;
                    rf[rep] = c;
                    x = xl[rep];
                    xe = xp[rep];
                    if (rep == vrep) {
                        enter_virtual();
                        x = xe = 0;
                    }
                }
                sg[nseg++] = rep; // finished: back to the parent
                const T up = par[rep];
                if (up == (T)NONE) break;
                rep = up;
                x = xo[rep];
                xe = xp[rep];
            }
        }
        const I nexp = nextl - start;                                  // P and Q
        const I nvirt = split >= 0 ? last_len - lbelow - p_in : 0;     // the virtual part
        const I len = nexp + nvirt;                                    // |L(:, j)|
        if (j == 0) {
            ns = supno[0] = 0;
        } else {
            bool js = subset;
            if (len != last_len - 1) js = false;
            if (j - cur_fs >= maxsuper) js = false;
            if (js) {
                // L(:, j) = P ++ (L(:, j-1) minus j-1 minus P): P to the front
                if (split >= 0) {
                    SYMB_CNT(4, nexp);
                    for (I i = start + nexp - 1; i >= start; --i) {
                        l_unlink(L[i]);
                        l_push_front(L[i]);
                    }
                    if (lbelow == 1) {
                        l_unlink(vrep);
                    } else {
                        for (T c = lhead; c != (T)NONE;) {
                            SYMB_CNT(3, 1);
                            const T nx = lnx[c];
                            if (c < tj) l_unlink(c);
                            c = nx;
                        }
                    }
                } else {
                    l_build(L + start, nexp);
                }
                lbelow = 1; // (row j of L(:, j))
                lmin = tj;
                last_len = len;
                tail_sum += len;
                xsup[ns + 1] = (T)(j + 1);
                supno[j + 1] = (T)ns;
                xlsub[j + 1] = xlsub[cur_fs + 1] + len;
                xprune[j] = xlsub[j + 1];
                return nseg;
            }
            // the current supernode ends at j - 1: its last list where the
            // classic compaction leaves it
            if (!closed) {
                if (j - 1 > cur_fs) {
                    const I to = xlsub[cur_fs + 1];
                    l_write(to, (T)0, (T)-4); // (every row: no mark equals -4)
                    xlsub[j - 1] = to;
                    xprune[j - 1] = to + last_len;
                }
                set_rep(cur_fs, j - 1);
            }
            // L(:, j) in full: P, the virtual part, then Q
            if (split >= 0) {
                const I nq = nexp - split;
                if (nq && nvirt) memmove(L + start + split + nvirt, L + start + split, nq * sizeof(T));
                l_write(start + split, tj, tj);
            }
            ++ns;
            supno[j] = (T)ns;
        }
        xsup[ns + 1] = (T)(j + 1);
        supno[j + 1] = (T)ns;
        xlsub[j] = start;
        xprune[j] = start + len;
        xlsub[j + 1] = start + len;
        return nseg;
    }

    // pivot of a column that extends the current supernode: row j to
    // position j - fsupc of the first list, by the kept positions
    void pivot_v(I j) {
        if (j == cur_fs || supno[j] != cur_s) return pivot(j);
        const I fs = cur_fs, lp = xlsub[fs], nr = xlsub[fs + 1] - lp, d0 = j - fs;
        const T tj = (T)j;
        if (fl[tj] != cur_s || pos[tj] < d0 || pos[tj] >= nr)
            throw Error("symbfact: zero diagonal at column " + std::to_string(j));
        const I d = pos[tj];
        if (d != d0) {
            const T o = lsub[lp + d0];
            std::swap(lsub[lp + d], lsub[lp + d0]);
            pos[o] = d;
            pos[tj] = d0;
        }
    }

    // columns [a, b) with the relaxed supernode ends `rend`
    void run(I a, I b, const I *rend) {
        const char *cl = getenv("SLU_SYMB_CLASSIC");
        if (cl && atoi(cl) == 1) {
            for (I j = a; j < b;) {
                if (rend[j] != NONE) {
                    const I k = rend[j];
                    relaxed(j, k);
                    for (I i = j; i <= k; ++i) pivot(i);
                    j = k + 1;
                } else {
                    const I nseg = column(j);
                    set_usub(j, nseg);
                    pivot(j);
                    prune(j, nseg);
                    for (I s = 0; s < nseg; ++s) repfnz[segrep[s]] = (T)NONE;
                    ++j;
                }
            }
            return;
        }
        vinit();
        for (I j = a; j < b;) {
            if (sub_i < subs.size() && subs[sub_i].first == j) { // a subtree searched by its own Walker
                close_at(j, rend);
                const auto ti0 = std::chrono::steady_clock::now();
                j = import_task(*subs[sub_i].second);
                subs[sub_i].second->free();
                ++sub_i;
                t_import += std::chrono::duration<double>(std::chrono::steady_clock::now() - ti0).count();
                continue;
            }
            if (rend[j] != NONE) {
                const I k = rend[j];
                if (j > 0 && !closed) finish_current(j);
                relaxed(j, k);
                for (I i = j; i <= k; ++i) pivot(i);
                start_supernode(j, k);
                j = k + 1;
            } else {
                const I nseg = column_v(j);
                set_usub(j, nseg);
                const bool fresh = supno[j] != cur_s || j == 0;
                if (fresh) pivot(j);
                else pivot_v(j);
                prune(j, nseg);
                for (I s = 0; s < nseg; ++s) repfnz[segrep[s]] = (T)NONE;
                if (fresh) start_supernode(j, j);
                ++j;
            }
        }
        if (b > a) close_at(b, rend);
    }

    // Closes the current supernode as column j's processing would in the
    // sequential search, j being a column that cannot extend it (the first
    // column of a subtree that is not the one ending at j - 1's parent, or
    // the end): before a relaxed supernode or at the end finish_current,
    // else what column_v does for a column that does not join.  Leaves
    // xlsub[j] at where column j's list starts.
    void close_at(I j, const I *rend) {
        if (closed || j == 0) return;
        if (j >= mn_ || rend[j] != NONE) {
            finish_current(j);
        } else {
            if (j - 1 > cur_fs) {
                const I to = xlsub[cur_fs + 1];
                reserve(to, last_len);
                l_write(to, (T)0, (T)-4);
                xlsub[j - 1] = to;
                xprune[j - 1] = to + last_len;
                xlsub[j] = to + last_len;
            } else {
                xlsub[j] = xlsub[cur_fs + 1];
            }
            set_rep(cur_fs, j - 1);
        }
        cur_s = (T)-2;
        closed = true;
    }

    // ---- subtree tasks: a subtree [lo, hi] of the postordered etree whose
    // root's next column is not its parent searched by its own Walker (the
    // search of a column only reaches its descendants), then its arrays
    // imported here at the positions and supernode numbers the sequential
    // search would have given them (tests/test_symbolic.py: identical arrays)
    struct TaskOut {
        I lo = 0, hi = -1, nsup = 0, nl = 0, nu = 0;
        vector<T> supno, xsup, repc, lsub, usub; // supno: lo..hi+1; xsup: 0..nsup
        vector<I> xlsub, xprune, xusub;          // lo..hi+1 (xusub: lo+1..hi+1)
        void free() {
            *this = TaskOut();
        }
    };
    // the subtrees inside this Walker's range searched before it (first
    // column, result), in column order
    vector<std::pair<I, TaskOut *>> subs;
    size_t sub_i = 0;
    double t_import = 0;
    I mn_ = 0;

    // this Walker as a task over [lo, hi] (fresh): local supernode numbers
    // from 0, positions from 0
    std::unique_ptr<TaskOut> run_task(I lo, I hi, const I *rend) {
        supno[lo] = (T)NONE;
        xsup[0] = (T)lo;
        xlsub[lo] = 0;
        xusub[lo] = 0;
        nextu = 0;
        closed = true;
        run(lo, hi + 1, rend);
        auto o = std::make_unique<TaskOut>();
        o->lo = lo;
        o->hi = hi;
        o->nsup = (I)supno[hi + 1] + 1;
        o->nl = xlsub[hi + 1];
        o->nu = nextu;
        o->supno.assign(supno.begin() + lo, supno.begin() + hi + 2);
        o->xsup.assign(xsup.begin(), xsup.begin() + o->nsup + 1);
        o->repc.assign(repc.begin() + lo, repc.begin() + hi + 1);
        o->lsub.assign(lsub.begin(), lsub.begin() + o->nl);
        o->usub.assign(usub.begin(), usub.begin() + o->nu);
        o->xlsub.assign(xlsub.begin() + lo, xlsub.begin() + hi + 2);
        o->xprune.assign(xprune.begin() + lo, xprune.begin() + hi + 1);
        o->xusub.assign(xusub.begin() + lo, xusub.begin() + hi + 2);
        return o;
    }

    // a finished task's arrays into this (closed) Walker; returns hi + 1
    I import_task(const TaskOut &o) {
        const I lo = o.lo, hi = o.hi, off = xlsub[lo], uoff = nextu;
        const T soff = (T)(supno[lo] + 1); // (supno[0] = NONE: the first supernode is 0)
        reserve(off, o.nl);
        parallel_for((int)((o.nl + (1 << 22) - 1) >> 22), [&](int t) {
            const I a = (I)t << 22, b = std::min<I>(o.nl, (I)(t + 1) << 22);
            std::copy(o.lsub.begin() + a, o.lsub.begin() + b, lsub.begin() + off + a);
        }, 1);
        if (uoff + o.nu > (I)usub.size()) usub.resize(std::max<I>(2 * usub.size(), uoff + o.nu + 1024));
        parallel_for((int)((o.nu + (1 << 22) - 1) >> 22), [&](int t) {
            const I a = (I)t << 22, b = std::min<I>(o.nu, (I)(t + 1) << 22);
            std::copy(o.usub.begin() + a, o.usub.begin() + b, usub.begin() + uoff + a);
        }, 1);
        nextu = uoff + o.nu;
        for (I c = lo; c <= hi; ++c) {
            supno[c] = o.supno[c - lo] + soff;
            xlsub[c] = o.xlsub[c - lo] + off;
            xprune[c] = o.xprune[c - lo] + off;
            repc[c] = o.repc[c - lo];
            xusub[c + 1] = o.xusub[c + 1 - lo] + uoff;
        }
        supno[hi + 1] = o.supno[hi + 1 - lo] + soff;
        xlsub[hi + 1] = o.xlsub[hi + 1 - lo] + off;
        for (I sn = 0; sn <= o.nsup; ++sn) xsup[soff + sn] = o.xsup[sn];
        cur_s = (T)-2;
        closed = true;
        return hi + 1;
    }

    // before a relaxed supernode at column j (or at the end, j = b): the
    // current supernode's last list written out; at the end the classic
    // layout keeps every column list of the last supernode uncompacted, so
    // xlsub[b] is its classic total
    void finish_current(I j) {
        if (cur_s == supno[j - 1]) set_rep(cur_fs, j - 1);
        if (j - 1 > cur_fs && cur_s == supno[j - 1]) {
            // the classic layout: compaction happens only when a searched
            // column does not join, so here every column list past the first
            // stays in place and the last one ends at xlsub[fs+1] + tail_sum
            const I end = xlsub[cur_fs + 1] + tail_sum, at = end - last_len;
            reserve(at, last_len);
            l_write(at, (T)0, (T)-4);
            xlsub[j - 1] = at;
            xprune[j - 1] = end;
            xlsub[j] = end;
        }
    }
};

// Subtree tasks for the host threads.  The search of a column only reaches
// its descendants when every entry A(r, j), r < j, has r in j's subtree
// (checked here; if not, no tasks).  A task is a subtree of between tmin and
// tmax columns whose root is not its parent's last child -- so the column
// after it is not the root's parent and cannot extend the subtree's last
// supernode -- and that does not start inside a relaxed supernode; the
// search in column order imports its arrays when it gets there.  (Tasks
// inside tasks, to take the upper separators' siblings off the ordered
// search too, measured slower: every level waits for its slowest subtree
// and the nested imports copy the lists again, 11.2 -> 12.4 s at 100^3 in
// the build container.)  SLU_SYMB_TASKS=0: none; SLU_SYMB_TASK_MIN / _MAX:
// the bounds (default 1024 and max(4096, n / 8)).
struct SymbTask {
    I lo, hi; // the subtree's columns
};
static void plan_tasks(I n, const I *parent, const I *cb, const I *ce, const I *ri, const I *rend,
                       vector<SymbTask> &tasks) {
    tasks.clear();
    auto env = [](const char *k, I d) {
        const char *e = getenv(k);
        return e ? (I)atoll(e) : d;
    };
    if (env("SLU_SYMB_TASKS", 1) == 0) return;
    if (const char *cl = getenv("SLU_SYMB_CLASSIC"); cl && atoi(cl) == 1) return;
    const I tmin = std::max<I>(2, env("SLU_SYMB_TASK_MIN", 1024));
    // (n / 8: at 100^3 in the build container 5.5 s against 8.2 s with
    // n / 32 -- the smaller the tasks, the more of the middle separators the
    // search in column order keeps)
    const I tmax = std::max<I>(tmin, env("SLU_SYMB_TASK_MAX", std::max<I>(4096, n / 8)));
    if (n < 2 * tmin) return;
    vector<I> desc(n + 1, 0);
    for (I j = 0; j < n; ++j) {
        if (parent[j] <= j || parent[j] > n) return; // not a postordered forest
        desc[parent[j]] += desc[j] + 1;
    }
    std::atomic<bool> ok(true);
    parallel_for((int)((n + 4095) / 4096), [&](int t) {
        for (I j = (I)t * 4096; j < std::min<I>(n, (I)(t + 1) * 4096); ++j)
            for (I p = cb[j]; p < ce[j]; ++p)
                if (ri[p] < j && ri[p] < j - desc[j]) ok = false;
    }, 1);
    if (!ok) return;
    // the last column of the relaxed supernode each column lies in (NONE: none)
    vector<I> inrel(n, NONE);
    for (I f = 0; f < n; ++f)
        if (rend[f] != NONE)
            for (I c = f; c <= rend[f]; ++c) inrel[c] = rend[f];
    vector<I> head(n + 1, NONE), next(n, NONE); // children in increasing order
    for (I v = n - 1; v >= 0; --v) {
        next[v] = head[parent[v]];
        head[parent[v]] = v;
    }
    vector<I> stack;
    for (I c = head[n]; c != NONE; c = next[c]) stack.push_back(c);
    while (!stack.empty()) {
        const I v = stack.back();
        stack.pop_back();
        const I size = desc[v] + 1;
        if (size < tmin) continue;                      // small: searched in column order
        if (inrel[v] != NONE && inrel[v] != v) continue; // inside a relaxed supernode: likewise
        const bool closable = parent[v] == n || v + 1 != parent[v];
        if (size <= tmax && closable) {
            tasks.push_back({v - desc[v], v});
            continue;
        }
        for (I c = head[v]; c != NONE; c = next[c]) stack.push_back(c);
    }
    if (tasks.size() < 2) {
        tasks.clear();
        return;
    }
    std::sort(tasks.begin(), tasks.end(), [](const SymbTask &x, const SymbTask &y) { return x.lo < y.lo; });
}

// symbfact (SRC/symbfact.c:81-215).  m x n matrix, columns [cb[j], ce[j])
// of ri (A Pc', rows relabelled by perm_c); etree postordered.
template <class T>
static Result symbfact_t(I m, I n, const I *cb, const I *ce, const I *ri64, const I *etree,
                         I relax, I maxsuper, bool dev_default) {
    Result R;
    R.n = n;
    const I mn = std::min(m, n);
    I annz = 0, top = 0;
    for (I c = 0; c < n; ++c) {
        annz += ce[c] - cb[c];
        top = std::max(top, ce[c]);
    }
    vector<T> ri(top);
    for (I c = 0; c < n; ++c)
        for (I p = cb[c]; p < ce[c]; ++p) ri[p] = (T)ri64[p];
    const vector<I> rend = relaxed_ends(n, etree, relax);

    const auto t0 = std::chrono::steady_clock::now();
    auto setup = [&](Walker<T> &w) {
        w.m = m;
        w.cb = cb;
        w.ce = ce;
        w.ri = ri.data();
        w.maxsuper = maxsuper;
        w.mn_ = mn;
    };
    // the subtree tasks on the host threads, then the search in column order
    // importing their arrays (identical arrays; SLU_SYMB_TASKS=0: no tasks)
    vector<SymbTask> tasks;
    if (m == n) plan_tasks(n, etree, cb, ce, ri64, rend.data(), tasks);
    Walker<T> w(m, n, std::max<I>(4 * annz, 1024));
    setup(w);
    using Out = typename Walker<T>::TaskOut;
    vector<std::unique_ptr<Out>> outs(tasks.size());
    bool seq = tasks.empty();
    if (!seq) {
        try {
            parallel_for((int)tasks.size(), [&](int q) {
                const SymbTask &t = tasks[q];
                I nz = 0;
                for (I c = t.lo; c <= t.hi; ++c) nz += ce[c] - cb[c];
                Walker<T> tw(m, n, std::max<I>(4 * nz, 1024));
                setup(tw);
                outs[q] = tw.run_task(t.lo, t.hi, rend.data());
            }, 1);
            I total = 0, totu = 0; // room for the imported lists at once, not by doublings
            for (size_t q = 0; q < tasks.size(); ++q) {
                w.subs.push_back({tasks[q].lo, outs[q].get()});
                total += outs[q]->nl;
                totu += outs[q]->nu;
            }
            if ((I)w.lsub.size() < total + 4 * annz) w.lsub.resize(total + 4 * annz);
            if ((I)w.usub.size() < totu + 2 * annz) w.usub.resize(totu + 2 * annz);
        } catch (const std::exception &) {
            seq = true; // (the search in column order reports the first failing column)
            w.subs.clear();
        }
    }
    if (getenv("SLU_SYMB_TIME") && !seq)
        fprintf(stderr, "symbfact: %zu subtree tasks %.3f s\n", tasks.size(),
                std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count());
    w.run(0, mn, rend.data());
    const auto t1 = std::chrono::steady_clock::now();
    if (getenv("SLU_SYMB_TIME") && !seq) fprintf(stderr, "symbfact: imports %.3f s\n", w.t_import);

    g_last_epilogue = 0;
    if constexpr (std::is_same<T, int32_t>::value) {
        const I nsup1 = (I)w.supno[n] + 1;
        if (n > 1 && use_device_epilogue(m, n, nsup1, dev_default)) {
            // countnz + fixupL on the device (csrc/symbolic_dev.hip)
            std::string err;
            R.lsub_size = w.xlsub[n];
            if (!slu_symb_epilogue_dev(n, nsup1, w.lsub.data(), w.xlsub[n], w.xlsub.data(), w.xsup.data(),
                                       w.supno.data(), w.usub.data(), w.xusub[mn], R.lsub, R.xlsub, &R.nnzL,
                                       &R.nnzU, err))
                throw Error("symbfact device epilogue: " + err);
            R.nnzLU = R.nnzL + R.nnzU - mn;
            R.xsup.assign(w.xsup.begin(), w.xsup.end());
            R.supno.assign(w.supno.begin(), w.supno.end());
            R.xusub = std::move(w.xusub);
            R.usub.assign(w.usub.begin(), w.usub.begin() + R.xusub[mn]);
            g_last_epilogue = 1;
            if (getenv("SLU_SYMB_TIME"))
                fprintf(stderr, "symbfact: search %.3f s, total %.3f s (device epilogue)\n",
                        std::chrono::duration<double>(t1 - t0).count(),
                        std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count());
            return R;
        }
    }
    auto te = std::chrono::steady_clock::now();
    auto etick = [&](const char *what) {
        if (!getenv("SLU_SYMB_TIME")) return;
        fprintf(stderr, "symbfact epilogue: %-10s %.3f s\n", what,
                std::chrono::duration<double>(std::chrono::steady_clock::now() - te).count());
        te = std::chrono::steady_clock::now();
    };
    R.xsup.assign(w.xsup.begin(), w.xsup.end());
    R.supno.assign(w.supno.begin(), w.supno.end());
    R.xlsub = std::move(w.xlsub);
    R.xusub = std::move(w.xusub);
    {
        const I nu = R.xusub[mn];
        R.usub.resize(nu);
        parallel_for((int)((nu + (1 << 20) - 1) >> 20), [&](int t) {
            for (I p = (I)t << 20; p < std::min<I>(nu, (I)(t + 1) << 20); ++p) R.usub[p] = w.usub[p];
        }, 1);
    }
    etick("copies");

    // ---- counts (SRC/util.c:95-152) and the final L subscripts: the first
    // column's list of each supernode, in supernode order (SRC/util.c:163-199).
    // On the host threads: blocks of supernodes / columns, partial sums added
    // in block order (integers: the same totals as serially)
    const I nsup = R.supno[n];
    constexpr I SB = 4096;
    const int nsb = (int)((nsup + 1 + SB - 1) / SB), ncb = (int)((n + SB - 1) / SB);
    vector<I> pl(nsb, 0), pu(nsb, 0), pc(ncb, 0), flen(nsup + 1), fsrc(nsup + 1);
    parallel_for(nsb, [&](int t) {
        I a = 0, u = 0;
        for (I s = (I)t * SB; s < std::min<I>(nsup + 1, (I)(t + 1) * SB); ++s) {
            const I f = R.xsup[s];
            fsrc[s] = R.xlsub[f];
            flen[s] = R.xlsub[f + 1] - R.xlsub[f];
            I len = flen[s];
            for (I c = f; c < R.xsup[s + 1]; ++c) {
                a += len;
                u += c - f + 1;
                --len;
            }
        }
        pl[t] = a;
        pu[t] = u;
    }, 1);
    parallel_for(ncb, [&](int t) {
        I u = 0;
        for (I c = (I)t * SB; c < std::min<I>(n, (I)(t + 1) * SB); ++c)
            for (I p = R.xusub[c]; p < R.xusub[c + 1]; ++p) {
                const I f = R.usub[p];
                u += R.xsup[R.supno[f] + 1] - f;
            }
        pc[t] = u;
    }, 1);
    etick("counts");
    for (I v : pl) R.nnzL += v;
    for (I v : pu) R.nnzU += v;
    for (I v : pc) R.nnzU += v;
    R.nnzLU = R.nnzL + R.nnzU - mn;
    if (n > 1) {
        R.lsub_size = R.xlsub[n];
        vector<I> out(nsup + 2, 0);
        for (I s = 0; s <= nsup; ++s) out[s + 1] = out[s] + flen[s];
        R.lsub.resize(out[nsup + 1]);
        etick("lsub alloc");
        parallel_for(nsb, [&](int t) {
            for (I s = (I)t * SB; s < std::min<I>(nsup + 1, (I)(t + 1) * SB); ++s) {
                const I f = R.xsup[s], a = fsrc[s], o = out[s];
                // the reference applies perm_r here: the identity on pivoted
                // rows, EMPTY on rows past min(m, n)
                for (I q = 0; q < flen[s]; ++q) R.lsub[o + q] = (I)w.lsub[a + q] < mn ? (I)w.lsub[a + q] : NONE;
                R.xlsub[f] = o;
                for (I c = f + 1; c < R.xsup[s + 1]; ++c) R.xlsub[c] = o + flen[s];
            }
        }, 1);
        R.xlsub[n] = out[nsup + 1];
        etick("lsub");
    } else {
        R.lsub.assign(w.lsub.begin(), w.lsub.begin() + R.xlsub[n]);
    }
    if (getenv("SLU_SYMB_TIME"))
        fprintf(stderr, "symbfact: search %.3f s, total %.3f s\n",
                std::chrono::duration<double>(t1 - t0).count(),
                std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count());
#ifdef SLU_SYMB_COUNT
    fprintf(stderr, "symbfact counts: dfs %lld prune-scan %lld list-write %lld unlink-scan %lld p-front %lld\n",
            g_cnt[0], g_cnt[1], g_cnt[2], g_cnt[3], g_cnt[4]);
#endif
    return R;
}

static Result symbfact(I m, I n, const I *cb, const I *ce, const I *ri, const I *etree, I relax,
                       I maxsuper, bool dev_default) {
    if (std::max(m, n) + 2 < (I)INT32_MAX)
        return symbfact_t<int32_t>(m, n, cb, ce, ri, etree, relax, maxsuper, dev_default);
    return symbfact_t<int64_t>(m, n, cb, ce, ri, etree, relax, maxsuper, dev_default);
}

// sp_ienv_dist(2) / (3) (SRC/sp_ienv.c:85-112): environment first, then
// the options; relax not above maxsup
static I env_or(const char *a, const char *b, I dflt, bool cap) {
    const char *s = getenv(a);
    if (!s) s = getenv(b);
    if (!s) return dflt;
    const I k = atoi(s);
    return cap ? std::min<I>(k, 512) : k; // MAX_SUPER_SIZE, SRC/superlu_defs.h:139
}
static I maxsup_of(const superlu_dist_options_t *o) {
    return env_or("SUPERLU_MAXSUP", "NSUP", o->superlu_maxsup, true);
}
static I relax_of(const superlu_dist_options_t *o) {
    return std::min(env_or("SUPERLU_RELAX", "NREL", o->superlu_relax, false), maxsup_of(o));
}

template <class T, class V>
static T *copy_out(const V &v, size_t n) {
    T *p = (T *)malloc(std::max<size_t>(n, 1) * sizeof(T));
    if (!p) throw Error("symbfact: out of host memory");
    if (n) memcpy(p, v.data(), n * sizeof(T));
    return p;
}

} // namespace symb
} // namespace slu

using namespace slu::symb;

extern "C" {

int slu_colorder(int64_t m, int64_t n, const int64_t *colptr, const int64_t *rowind, int ata,
                 int recompute, int64_t *perm_c, int64_t *etree, int64_t *colbeg, int64_t *colend) {
    try {
        colorder(m, n, colptr, rowind, ata != 0, recompute != 0, perm_c, etree, colbeg, colend);
        return 0;
    } catch (const std::exception &e) {
        slu::set_last_error(e.what());
        return -1;
    }
}

void *slu_symbfact(int64_t m, int64_t n, const int64_t *colbeg, const int64_t *colend,
                   const int64_t *rowind, const int64_t *etree, int64_t relax, int64_t maxsuper) {
    try {
        return new Result(symbfact(m, n, colbeg, colend, rowind, etree, relax, maxsuper, true));
    } catch (const std::exception &e) {
        slu::set_last_error(e.what());
        return nullptr;
    }
}

void slu_symbfact_sizes(const void *h, int64_t *out) {
    const Result &R = *(const Result *)h;
    out[0] = R.n ? R.supno[R.n] + 1 : 0;
    out[1] = (int64_t)R.lsub.size();
    out[2] = (int64_t)R.usub.size();
    out[3] = R.nnzL;
    out[4] = R.nnzU;
    out[5] = R.nnzLU;
    out[6] = R.lsub_size;
}

void slu_symbfact_arrays(const void *h, int64_t *xsup, int64_t *supno, int64_t *xlsub,
                         int64_t *lsub, int64_t *xusub, int64_t *usub) {
    const Result &R = *(const Result *)h;
    const size_t n1 = R.n + 1;
    memcpy(xsup, R.xsup.data(), n1 * sizeof(int64_t));
    memcpy(supno, R.supno.data(), n1 * sizeof(int64_t));
    memcpy(xlsub, R.xlsub.data(), n1 * sizeof(int64_t));
    memcpy(xusub, R.xusub.data(), n1 * sizeof(int64_t));
    if (!R.lsub.empty()) memcpy(lsub, R.lsub.data(), R.lsub.size() * sizeof(int64_t));
    if (!R.usub.empty()) memcpy(usub, R.usub.data(), R.usub.size() * sizeof(int64_t));
}

void slu_symbfact_views(const void *h, const int64_t **ptrs) {
    const Result &R = *(const Result *)h;
    ptrs[0] = R.xsup.data();
    ptrs[1] = R.supno.data();
    ptrs[2] = R.xlsub.data();
    ptrs[3] = R.lsub.data();
    ptrs[4] = R.xusub.data();
    ptrs[5] = R.usub.data();
}

void slu_symbfact_free(void *h) { delete (Result *)h; }

// 1 when the last symbfact ran its countnz / fixupL epilogue on the GPU
int slu_symbfact_last_epilogue_device(void) { return g_last_epilogue; }

// ---- drop-in entry points with the reference's prototypes

// SRC/sp_colorder.c:81 (prototype SRC/superlu_defs.h).  AC's store and its
// colbeg / colend are malloc'ed as in the reference; rowind / nzval shared
// with A.
void sp_colorder(superlu_dist_options_t *options, SuperMatrix *A, int_t *perm_c, int_t *etree,
                 SuperMatrix *AC) {
    const NCformat *As = (const NCformat *)A->Store;
    const I n = A->ncol;
    NCPformat *S = (NCPformat *)malloc(sizeof(NCPformat));
    if (!S) {
        fprintf(stderr, "sp_colorder: out of host memory\n");
        abort(); // the reference ABORTs (SRC/sp_colorder.c:106)
    }
    S->nnz = As->nnz;
    S->nzval = As->nzval;
    S->rowind = As->rowind;
    S->colbeg = (int_t *)malloc(std::max<I>(n, 1) * sizeof(int_t));
    S->colend = (int_t *)malloc(std::max<I>(n, 1) * sizeof(int_t));
    if (!S->colbeg || !S->colend) {
        fprintf(stderr, "sp_colorder: out of host memory\n");
        abort();
    }
    AC->Stype = SLU_NCP;
    AC->Dtype = A->Dtype;
    AC->Mtype = A->Mtype;
    AC->nrow = A->nrow;
    AC->ncol = A->ncol;
    AC->Store = S;
    const bool recompute = options->Fact == SLU_DOFACT || options->Fact == SLU_SAMEPATTERN;
    colorder(A->nrow, n, As->colptr, As->rowind, options->ColPerm == SLU_MMD_ATA, recompute, perm_c,
             etree, S->colbeg, S->colend);
}

// SRC/symbfact.c:81: returns -(the reference's lsub size), 0 for n <= 1.
// Glu_persist->xsup / supno and the Glu_freeable arrays are malloc'ed
// (freed by the reference's symbfact_SubFree / LU destructors with free()).
int_t symbfact(superlu_dist_options_t *options, int pnum, SuperMatrix *A, int_t *perm_c,
               int_t *etree, Glu_persist_t *Glu_persist, Glu_freeable_t *Glu_freeable) {
    (void)perm_c;
    const NCPformat *S = (const NCPformat *)A->Store;
    // a device epilogue (SLU_SYMB_DEVICE=1) creates a HIP queue, which
    // reseeds libc rand(); pddistribute after this draws its solve trees'
    // seeds from rand() on every rank (abi.cpp, CallerRandState)
    char rbuf[256];
    char *rprev = initstate(1u, rbuf, sizeof rbuf);
    struct Restore {
        char *p;
        ~Restore() { setstate(p); }
    } restore{rprev};
    try {
        const Result R = symbfact(A->nrow, A->ncol, S->colbeg, S->colend, S->rowind, etree,
                                  relax_of(options), maxsup_of(options), false);
        if (!pnum && options->PrintStat == SLU_YES) { // SRC/symbfact.c:187-194
            printf("\tMatrix size min_mn  %lld\n", (long long)std::min<I>(A->nrow, A->ncol));
            printf("\tNonzeros in L       %lld\n", (long long)R.nnzL);
            printf("\tNonzeros in U       %lld\n", (long long)R.nnzU);
            printf("\tnonzeros in L+U     %lld\n", (long long)R.nnzLU);
            printf("\tnonzeros in LSUB    %lld\n", (long long)R.lsub_size);
        }
        const size_t n1 = A->ncol + 1;
        Glu_persist->xsup = copy_out<int_t>(R.xsup, n1);
        Glu_persist->supno = copy_out<int_t>(R.supno, n1);
        Glu_freeable->xlsub = copy_out<int_t>(R.xlsub, n1);
        Glu_freeable->xusub = copy_out<int_t>(R.xusub, n1);
        Glu_freeable->lsub = copy_out<int_t>(R.lsub, R.lsub.size());
        Glu_freeable->usub = copy_out<int_t>(R.usub, R.usub.size());
        Glu_freeable->nzlmax = std::max<I>((I)R.lsub.size(), 1);
        Glu_freeable->nzumax = std::max<I>((I)R.usub.size(), 1);
        Glu_freeable->MemModel = 0; // SYSTEM
        Glu_freeable->nnzLU = R.nnzLU;
        return -R.lsub_size;
    } catch (const std::exception &e) {
        // the reference ABORTs here (SRC/symbfact.c:724-727)
        fprintf(stderr, "symbfact: %s\n", e.what());
        abort();
    }
}

} // extern "C"

// Fill-reducing ordering for ColPerm = METIS_AT_PLUS_A.
//
// The reference orders A'+A with METIS when ColPerm = METIS_AT_PLUS_A, its
// default (SRC/get_perm_c.c:524-541, get_metis :33-108 calling
// METIS_NodeND(&n, xadj, adjncy, NULL, NULL, perm, iperm) with int_t
// arguments, then perm_c = iperm).  METIS is not part of the reference and
// not in this image, so a reference build here leaves METIS_NodeND
// unresolved and cannot run its default ordering.  This library exports
// METIS_NodeND with the prototype get_perm_c.c declares, computing a nested
// dissection of the graph:
//
//   * per connected part: a pseudo-peripheral vertex (repeated breadth-first
//     sweeps), its BFS level structure, and the level that best balances the
//     two sides among the levels near the median (a level set separates the
//     levels before it from those after it);
//   * the separator thinned to the vertices that touch the far side (the
//     others join the near side);
//   * near side, far side, then the separator, recursively, down to parts of
//     at most LEAF (32) vertices, which keep their BFS order;
//   * the two sides of the top splits on host threads.
//
// Not METIS's multilevel algorithm: its quality on 3D grids is measured
// against the reference's MMD and the geometric grid dissection in DESIGN §11.
#include <algorithm>
#include <cstdint>
#include <cstdlib>
#include <future>
#include <vector>

#include "common.h"
#include "slu_abi.h"

namespace slu {
namespace nd {

using I = int64_t;
using std::vector;

struct Graph {
    I n;
    const I *xadj, *adj;
};

struct Work {
    const Graph &g;
    vector<I> &order; // order[pos] = vertex
    // per-vertex scratch shared by all parts: a vertex belongs to one part at
    // a time, so concurrent parts touch disjoint entries
    vector<I> &level, &mark;
    vector<int> &part;
};

// leaf size (SLU_ND_LEAF for A/B): 32 -- 128 gave 2.5x the supernodes on the
// 3D Laplacian at the same factor time
static const I LEAF = getenv("SLU_ND_LEAF") ? atoll(getenv("SLU_ND_LEAF")) : 32;

// part[] is read for neighbours that belong to parts other threads are
// splitting: relaxed atomic accesses (the value read is never this part's id)
static inline int get_part(const Work &w, I v) { return __atomic_load_n(&w.part[v], __ATOMIC_RELAXED); }
static inline void set_part(const Work &w, I v, int p) { __atomic_store_n(&w.part[v], p, __ATOMIC_RELAXED); }

// BFS from `s` over vertices v with part[v] == p; fills lev (vertices in BFS
// order) and level[v]; returns the number of levels.
static I bfs(const Work &w, I s, int p, vector<I> &lev, vector<I> &start) {
    lev.clear();
    start.clear();
    lev.push_back(s);
    w.level[s] = 0;
    w.mark[s] = s;
    start.push_back(0);
    I cur = 0;
    for (size_t h = 0; h < lev.size(); ++h) {
        const I v = lev[h];
        if (w.level[v] != cur) {
            cur = w.level[v];
            start.push_back((I)h);
        }
        for (I q = w.g.xadj[v]; q < w.g.xadj[v + 1]; ++q) {
            const I u = w.g.adj[q];
            if (u == v || get_part(w, u) != p || w.mark[u] == s) continue;
            w.mark[u] = s;
            w.level[u] = cur + 1;
            lev.push_back(u);
        }
    }
    start.push_back((I)lev.size());
    return cur + 1;
}

// Orders the vertices of part p (listed in `verts`) into order[pos, pos+|verts|).
static void dissect(const Work &w, vector<I> verts, int p, I pos, int depth, int *next_part) {
    const I nv = (I)verts.size();
    if (nv <= LEAF) {
        // keep a BFS order inside the leaf (neighbours close together)
        vector<I> lev, start;
        I at = pos;
        for (I v : verts) w.mark[v] = -1;
        for (I v : verts) {
            if (w.mark[v] != -1) continue;
            bfs(w, v, p, lev, start);
            for (I u : lev) w.order[at++] = u;
        }
        return;
    }
    // BFS from the first vertex reaches its connected component; with
    // several components each is ordered on its own, one after the other
    vector<I> lev, start;
    for (I v : verts) w.mark[v] = -1;
    I s = verts[0];
    I nl = bfs(w, s, p, lev, start);
    if ((I)lev.size() < nv) {
        vector<vector<I>> comps;
        comps.emplace_back(lev.begin(), lev.end());
        for (I v : verts) {
            if (w.mark[v] != -1) continue;
            bfs(w, v, p, lev, start);
            comps.emplace_back(lev.begin(), lev.end());
        }
        I at = pos;
        for (auto &c : comps) {
            const int pc = __atomic_fetch_add(next_part, 1, __ATOMIC_RELAXED);
            for (I v : c) set_part(w, v, pc);
            const I nc = (I)c.size();
            dissect(w, std::move(c), pc, at, depth, next_part);
            at += nc;
        }
        return;
    }
    // pseudo-peripheral vertex: restart from a last-level vertex of
    // smallest degree while the eccentricity grows
    for (int sweep = 0; sweep < 4; ++sweep) {
        I best = -1, bd = INT64_MAX;
        for (I h = start[nl - 1]; h < start[nl]; ++h) {
            const I v = lev[h], d = w.g.xadj[v + 1] - w.g.xadj[v];
            if (d < bd) {
                bd = d;
                best = v;
            }
        }
        for (I v : verts) w.mark[v] = -1;
        vector<I> lev2, start2;
        const I nl2 = bfs(w, best, p, lev2, start2);
        if (nl2 <= nl) {
            // no longer growing: redo the BFS of the kept root (marks / levels)
            for (I v : verts) w.mark[v] = -1;
            nl = bfs(w, s, p, lev, start);
            break;
        }
        s = best;
        nl = nl2;
        lev.swap(lev2);
        start.swap(start2);
    }
    if (nl < 3) {
        // (nearly) a clique or a star: no useful separator, keep BFS order
        for (I h = 0; h < nv; ++h) w.order[pos + h] = lev[h];
        return;
    }
    // separator level: among levels whose near side holds 40-60 % (widened
    // if none), the smallest; ties to the most balanced
    I best = -1;
    for (double tol = 0.10; best < 0 && tol <= 0.5; tol += 0.10) {
        I bsz = INT64_MAX;
        double bbal = 1.0;
        for (I l = 1; l + 1 < nl; ++l) {
            const double near = (double)start[l] / nv;
            const double far = (double)(nv - start[l + 1]) / nv;
            if (near < 0.5 - tol || far < 0.5 - tol) continue;
            const I sz = start[l + 1] - start[l];
            const double bal = std::abs(near - far);
            if (sz < bsz || (sz == bsz && bal < bbal)) {
                bsz = sz;
                bbal = bal;
                best = l;
            }
        }
    }
    if (best < 0) best = nl / 2;
    // thin: a separator vertex without a neighbour on the far side joins the
    // near side
    const int pa = __atomic_fetch_add(next_part, 3, __ATOMIC_RELAXED), pb = pa + 1, ps = pa + 2;
    vector<I> A, B, S;
    A.reserve(start[best] + 16);
    for (I h = 0; h < start[best]; ++h) A.push_back(lev[h]);
    for (I h = start[best + 1]; h < nv; ++h) B.push_back(lev[h]);
    for (I h = start[best]; h < start[best + 1]; ++h) {
        const I v = lev[h];
        bool far = false;
        for (I q = w.g.xadj[v]; q < w.g.xadj[v + 1] && !far; ++q) {
            const I u = w.g.adj[q];
            far = get_part(w, u) == p && w.mark[u] == s && w.level[u] == best + 1;
        }
        (far ? S : A).push_back(v);
    }
    for (I v : A) set_part(w, v, pa);
    for (I v : B) set_part(w, v, pb);
    for (I v : S) set_part(w, v, ps);
    const I na = (I)A.size(), nb = (I)B.size();
    for (I h = 0; h < (I)S.size(); ++h) w.order[pos + na + nb + h] = S[h];
    if (depth < 3 && na > 4096 && nb > 4096) {
        auto fa = std::async(std::launch::async,
                             [&, A = std::move(A)]() mutable { dissect(w, std::move(A), pa, pos, depth + 1, next_part); });
        dissect(w, std::move(B), pb, pos + na, depth + 1, next_part);
        fa.get();
    } else {
        dissect(w, std::move(A), pa, pos, depth + 1, next_part);
        dissect(w, std::move(B), pb, pos + na, depth + 1, next_part);
    }
}

// perm[new] = old, iperm[old] = new (METIS convention)
static void order(I n, const I *xadj, const I *adj, I *perm, I *iperm) {
    Graph g{n, xadj, adj};
    vector<I> ord(n), level(n, 0), mark(n, -1);
    vector<int> part(n, 0);
    Work w{g, ord, level, mark, part};
    vector<I> all(n);
    for (I i = 0; i < n; ++i) all[i] = i;
    int next_part = 1;
    dissect(w, std::move(all), 0, 0, 0, &next_part);
    for (I i = 0; i < n; ++i) {
        perm[i] = ord[i];
        iperm[ord[i]] = i;
    }
}

} // namespace nd
} // namespace slu

extern "C" {

// METIS_NodeND as SRC/get_perm_c.c:49-50 declares it (int_t arguments;
// vwgt / options unused, as the reference passes NULL).  Returns 1
// (METIS_OK), or -4 (METIS_ERROR) on bad input.  Exported only by the
// opt-in libslu_mi355x_full.so (never by the drop-in libslu_mi355x.so),
// and weak: a METIS linked statically into the program binds first.
__attribute__((weak)) int METIS_NodeND(int_t *nvtxs, int_t *xadj, int_t *adjncy, int_t *vwgt, int_t *options,
                 int_t *perm, int_t *iperm) {
    (void)vwgt;
    (void)options;
    try {
        const int64_t n = *nvtxs;
        if (n < 0 || !xadj || !perm || !iperm || (n > 0 && xadj[0] != 0)) return -4;
        for (int64_t i = 0; i < n; ++i)
            if (xadj[i + 1] < xadj[i]) return -4;
        if (n > 0 && xadj[n] > 0 && !adjncy) return -4;
        for (int64_t i = 0; i < n; ++i)
            for (int64_t q = xadj[i]; q < xadj[i + 1]; ++q)
                if (adjncy[q] < 0 || adjncy[q] >= n) return -4;
        slu::nd::order(n, xadj, adjncy, perm, iperm);
        return 1;
    } catch (const std::exception &e) {
        slu::set_last_error(e.what());
        return -4;
    }
}

} // extern "C"

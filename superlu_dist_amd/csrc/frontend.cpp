// Front-end: stencil matrices, geometric nested dissection, supernodal symbolic
// factorization and 2D block-cyclic distribution into the SuperLU_DIST LU
// layout.  Host C++.  This is the input side of the numeric factorization
// (the reference's get_perm_c / symbfact / pddistribute stage, SURVEY §8f
// rows 1 and 3); it exists so that tests and the benchmark can build the
// LUstruct that pdgstrf consumes without the reference's front-end.
//
// Layout produced (SRC/superlu_defs.h:152-190, SRC/pddistribute.c:689-1340):
//   L block column ljb (PCOL(jb)==mycol):
//     index = [nblocks, nsupr, {gb, nrows, rows[nrows]}...]   (blocks sorted
//     by gb, diagonal block first on the diagonal process row)
//     nzval = nsupr x nsupc column-major
//   U block row lb (PROW(gb)==myrow):
//     index = [nblocks, len(nzval), len(index), {jb, nnz, fstnz[nsupc(jb)]}...,
//              -1]  (blocks sorted by jb)
//     nzval = concatenated column segments [fstnz, xsup[gb+1])
//   ToRecv / ToSendD / ToSendR / bufmax as SRC/pddistribute.c:752-801,2370.
#include "slu_mi355x.h"
#include "amalg.h"
#include "common.h"

#include <algorithm>
#include <complex>
#include <cstdlib>
#include <cstring>
#include <numeric>
#include <vector>

using std::vector;

namespace {

size_t vsize(int dtype) { return dtype == SLU_S ? 4 : dtype == SLU_Z ? 16 : 8; }

// ----------------------------------------------------------------------------
// Nested dissection of a regular grid.
struct Box { int x0, x1, y0, y1, z0, z1; };

void nd_box(const Box &b, int ny, int nz, vector<int64_t> &order) {
    int dx = b.x1 - b.x0, dy = b.y1 - b.y0, dz = b.z1 - b.z0;
    if (dx <= 0 || dy <= 0 || dz <= 0) return;
    long vol = (long)dx * dy * dz;
    int mx = std::max(dx, std::max(dy, dz));
    if (vol <= 32 || mx <= 2) {
        for (int i = b.x0; i < b.x1; ++i)
            for (int j = b.y0; j < b.y1; ++j)
                for (int l = b.z0; l < b.z1; ++l)
                    order.push_back(((int64_t)i * ny + j) * nz + l);
        return;
    }
    Box lo = b, hi = b, sep = b;
    if (dx == mx) {
        int m = b.x0 + dx / 2;
        lo.x1 = m; hi.x0 = m + 1; sep.x0 = m; sep.x1 = m + 1;
    } else if (dy == mx) {
        int m = b.y0 + dy / 2;
        lo.y1 = m; hi.y0 = m + 1; sep.y0 = m; sep.y1 = m + 1;
    } else {
        int m = b.z0 + dz / 2;
        lo.z1 = m; hi.z0 = m + 1; sep.z0 = m; sep.z1 = m + 1;
    }
    nd_box(lo, ny, nz, order);
    nd_box(hi, ny, nz, order);
    for (int i = sep.x0; i < sep.x1; ++i)
        for (int j = sep.y0; j < sep.y1; ++j)
            for (int l = sep.z0; l < sep.z1; ++l)
                order.push_back(((int64_t)i * ny + j) * nz + l);
}

// Symmetric adjacency (no diagonal), CSC-like, sorted rows.
struct Graph {
    int64_t n = 0;
    vector<int64_t> ptr, idx;
};

Graph sym_pattern(const slu_csc *A, const vector<int64_t> &perm) {
    int64_t n = A->n;
    vector<int64_t> cnt(n + 1, 0);
    for (int64_t j = 0; j < n; ++j)
        for (int64_t p = A->colptr[j]; p < A->colptr[j + 1]; ++p) {
            int64_t i = A->rowind[p];
            if (i == j) continue;
            cnt[perm[i] + 1]++;
            cnt[perm[j] + 1]++;
        }
    Graph g;
    g.n = n;
    g.ptr.assign(n + 1, 0);
    for (int64_t j = 0; j < n; ++j) g.ptr[j + 1] = g.ptr[j] + cnt[j + 1];
    g.idx.resize(g.ptr[n]);
    vector<int64_t> pos(g.ptr.begin(), g.ptr.end() - 1);
    for (int64_t j = 0; j < n; ++j)
        for (int64_t p = A->colptr[j]; p < A->colptr[j + 1]; ++p) {
            int64_t i = A->rowind[p];
            if (i == j) continue;
            int64_t pi = perm[i], pj = perm[j];
            g.idx[pos[pj]++] = pi;
            g.idx[pos[pi]++] = pj;
        }
    // sort + dedupe each column
    vector<int64_t> nptr(n + 1, 0);
    int64_t w = 0;
    for (int64_t j = 0; j < n; ++j) {
        int64_t b = g.ptr[j], e = g.ptr[j + 1];
        std::sort(g.idx.begin() + b, g.idx.begin() + e);
        nptr[j] = w;
        int64_t last = -1;
        for (int64_t p = b; p < e; ++p)
            if (g.idx[p] != last) { last = g.idx[p]; g.idx[w++] = last; }
    }
    nptr[n] = w;
    g.idx.resize(w);
    g.ptr.swap(nptr);
    return g;
}

vector<int64_t> etree_of(const Graph &g) {
    int64_t n = g.n;
    vector<int64_t> parent(n, -1), anc(n, -1);
    for (int64_t k = 0; k < n; ++k) {
        for (int64_t p = g.ptr[k]; p < g.ptr[k + 1]; ++p) {
            int64_t i = g.idx[p];
            if (i >= k) break; // sorted
            while (true) {
                int64_t a = anc[i];
                if (a == k) break;
                anc[i] = k;
                if (a == -1) { parent[i] = k; break; }
                i = a;
            }
        }
    }
    return parent;
}

vector<int64_t> postorder(const vector<int64_t> &parent) {
    int64_t n = parent.size();
    vector<int64_t> head(n, -1), next(n, -1);
    // children in increasing order: insert in reverse
    for (int64_t j = n - 1; j >= 0; --j) {
        int64_t p = parent[j];
        if (p >= 0) { next[j] = head[p]; head[p] = j; }
    }
    vector<int64_t> post;
    post.reserve(n);
    vector<int64_t> stack;
    for (int64_t r = 0; r < n; ++r) {
        if (parent[r] != -1) continue;
        stack.push_back(r);
        while (!stack.empty()) {
            int64_t v = stack.back();
            int64_t c = head[v];
            if (c != -1) {
                head[v] = next[c];
                stack.push_back(c);
            } else {
                stack.pop_back();
                post.push_back(v);
            }
        }
    }
    return post; // post[k] = node visited k-th
}

} // namespace

struct slu_symb {
    int64_t n = 0, nsupers = 0;
    vector<int64_t> perm;       // final perm_c
    vector<int64_t> xsup, supno;
    vector<int64_t> sptr, srows; // struct(L_s) incl. diagonal rows, sorted
    vector<int64_t> sparent;     // supernodal etree
    double nnzL = 0, nnzU = 0;
    // SLU_SYMB_REFERENCE: the reference's own symbolic factorization
    // (sp_colorder + symbfact, csrc/symbolic.cpp) -- Glu_freeable's arrays,
    // distributed by the reference's pddistribute (csrc/distribute.cpp)
    bool ref = false;
    vector<int64_t> xlsub, lsub, xusub, usub;
    // SLU_SYMB_COARSE: the partition and Glu above are the engine's coarse
    // partition of the reference's (csrc/amalg.h); the reference's own
    // partition size and algorithmic work (real-flop sums) are kept here
    int64_t nsupers_fine = 0;
    double fl[6] = {0, 0, 0, 0, 0, 0}; // schur, trsm, trsv, s1, s2, w
};

extern "C" {

slu_csc *slu_csc_create(int64_t n, int64_t nnz, const int64_t *colptr,
                        const int64_t *rowind, const void *val, int dtype) {
    slu_csc *A = (slu_csc *)calloc(1, sizeof(slu_csc));
    A->n = n;
    A->nnz = nnz;
    A->dtype = dtype;
    A->colptr = (int64_t *)malloc((n + 1) * sizeof(int64_t));
    A->rowind = (int64_t *)malloc(std::max<int64_t>(nnz, 1) * sizeof(int64_t));
    A->val = malloc(std::max<int64_t>(nnz, 1) * vsize(dtype));
    memcpy(A->colptr, colptr, (n + 1) * sizeof(int64_t));
    if (nnz) {
        memcpy(A->rowind, rowind, nnz * sizeof(int64_t));
        memcpy(A->val, val, nnz * vsize(dtype));
    }
    return A;
}

void slu_csc_free(slu_csc *A) {
    if (!A) return;
    free(A->colptr);
    free(A->rowind);
    free(A->val);
    free(A);
}

slu_csc *slu_gen_stencil(int kind, int nx, int ny, int nz, double diag,
                         double diag_im, double off, int dtype) {
    if (kind == 0) nz = 1;
    int64_t n = (int64_t)nx * ny * nz;
    int maxnb = kind == 2 ? 27 : kind == 1 ? 7 : 5;
    slu_csc *A = (slu_csc *)calloc(1, sizeof(slu_csc));
    A->n = n;
    A->dtype = dtype;
    A->colptr = (int64_t *)malloc((n + 1) * sizeof(int64_t));
    A->rowind = (int64_t *)malloc(n * maxnb * sizeof(int64_t));
    A->val = malloc(n * maxnb * vsize(dtype));
    int64_t w = 0;
    auto put = [&](int64_t r, bool isdiag) {
        A->rowind[w] = r;
        if (dtype == SLU_D) ((double *)A->val)[w] = isdiag ? diag : off;
        else if (dtype == SLU_S) ((float *)A->val)[w] = (float)(isdiag ? diag : off);
        else {
            ((double *)A->val)[2 * w] = isdiag ? diag : off;
            ((double *)A->val)[2 * w + 1] = isdiag ? diag_im : 0.0;
        }
        ++w;
    };
    int dmin = -1, dmax = 1;
    for (int i = 0; i < nx; ++i)
        for (int j = 0; j < ny; ++j)
            for (int l = 0; l < nz; ++l) {
                int64_t c = ((int64_t)i * ny + j) * nz + l;
                A->colptr[c] = w;
                // neighbours in lexicographic (sorted) order
                for (int di = dmin; di <= dmax; ++di)
                    for (int dj = dmin; dj <= dmax; ++dj)
                        for (int dl = dmin; dl <= dmax; ++dl) {
                            int nd = (di != 0) + (dj != 0) + (dl != 0);
                            if (kind == 0 && (dl != 0 || nd > 1)) continue;
                            if (kind == 1 && nd > 1) continue;
                            int ii = i + di, jj = j + dj, ll = l + dl;
                            if (ii < 0 || ii >= nx || jj < 0 || jj >= ny ||
                                ll < 0 || ll >= nz)
                                continue;
                            int64_t r = ((int64_t)ii * ny + jj) * nz + ll;
                            put(r, nd == 0);
                        }
            }
    A->colptr[n] = w;
    A->nnz = w;
    return A;
}

int slu_order_nd_grid(int nx, int ny, int nz, int64_t *perm_c) {
    if (nz < 1) nz = 1;
    vector<int64_t> order;
    order.reserve((size_t)nx * ny * nz);
    nd_box(Box{0, nx, 0, ny, 0, nz}, ny, nz, order);
    int64_t n = (int64_t)nx * ny * nz;
    if ((int64_t)order.size() != n) return -1;
    for (int64_t k = 0; k < n; ++k) perm_c[order[k]] = k;
    return 0;
}

// pdgssvx's symbolic stage for a square A with perm_r = I
// (SRC/pdgssvx.c:1046-1076): sp_colorder's etree postorder folded into perm_c,
// A Pc''s rows relabelled by perm_c, symbfact with relax / maxsup.  The
// supernode partition and L / U structure are then exactly what the
// reference's pdgssvx would hand pddistribute and pdgstrf for this perm_c.
static void coarsen(slu_symb *S);
static void glu_work(slu_symb *S);

static slu_symb *symbolic_reference(const slu_csc *A, vector<int64_t> perm, int relax,
                                    int maxsup, bool coarse) {
    const int64_t n = A->n;
    vector<int64_t> etree(n), cb(n), ce(n);
    if (slu_colorder(n, n, A->colptr, A->rowind, 0, 1, perm.data(), etree.data(), cb.data(),
                     ce.data()))
        return nullptr;
    vector<int64_t> ri(A->nnz);
    for (int64_t p = 0; p < A->nnz; ++p) ri[p] = perm[A->rowind[p]];
    void *h = slu_symbfact(n, n, cb.data(), ce.data(), ri.data(), etree.data(), relax, maxsup);
    if (!h) return nullptr;
    int64_t sz[7];
    slu_symbfact_sizes(h, sz);
    slu_symb *S = new slu_symb;
    S->ref = true;
    S->n = n;
    S->perm = perm;
    S->nsupers = sz[0];
    S->xsup.assign(n + 1, 0);
    S->supno.assign(n + 1, 0);
    S->xlsub.assign(n + 1, 0);
    S->xusub.assign(n + 1, 0);
    S->lsub.assign(std::max<int64_t>(sz[1], 1), 0);
    S->usub.assign(std::max<int64_t>(sz[2], 1), 0);
    slu_symbfact_arrays(h, S->xsup.data(), S->supno.data(), S->xlsub.data(), S->lsub.data(),
                        S->xusub.data(), S->usub.data());
    slu_symbfact_free(h);
    S->xsup.resize(S->nsupers + 1);
    S->supno.resize(n);
    // |struct(L_s)| (diagonal block rows included): the subscripts of a
    // supernode are stored once, at its first column (SRC/symbfact.c:81-215)
    S->sptr.assign(S->nsupers + 1, 0);
    for (int64_t k = 0; k < S->nsupers; ++k) {
        const int64_t f = S->xsup[k];
        S->sptr[k + 1] = S->sptr[k] + (S->xlsub[f + 1] - S->xlsub[f]);
    }
    S->nnzL = (double)sz[3];
    S->nnzU = (double)sz[4];
    S->nsupers_fine = S->nsupers;
    glu_work(S);
    if (coarse) coarsen(S);
    return S;
}

// The reference partition's algorithmic work from the Glu arrays (the
// accounting of the plan and of csrc/amalg.h): per supernode the
// diagonal LU, the L-panel TRSM over its rows below the diagonal block, and
// per U segment (a usub entry is the first row of a column's segment in its
// block row) the TRSV and the Schur update.
static void glu_work(slu_symb *S) {
    const int64_t ns = S->nsupers, n = S->n;
    vector<int64_t> b(ns, 0);
    double fl[6] = {0, 0, 0, 0, 0, 0};
    for (int64_t s = 0; s < ns; ++s) {
        const double w = (double)(S->xsup[s + 1] - S->xsup[s]);
        const int64_t f = S->xsup[s];
        b[s] = (S->xlsub[f + 1] - S->xlsub[f]) - (int64_t)w;
        fl[5] += w;
        fl[3] += w * (w - 1) / 2;
        fl[4] += (w - 1) * w * (2 * w - 1) / 6;
        fl[1] += w * (w + 1) * (double)b[s];
    }
    for (int64_t j = 0; j < n; ++j)
        for (int64_t i = S->xusub[j]; i < S->xusub[j + 1]; ++i) {
            const int64_t irow = S->usub[i], s = S->supno[irow];
            const double seg = (double)(S->xsup[s + 1] - irow);
            fl[2] += seg * (seg + 1);
            fl[0] += 2.0 * (double)b[s] * seg;
        }
    for (int i = 0; i < 6; ++i) S->fl[i] = fl[i];
}

// Replace the reference's partition by the engine's coarse one (csrc/amalg.h):
// the 1x1 index arrays of the reference's pddistribute (no values), their
// amalgamation, and the coarse Glu, so that slu_distribute lays the coarse
// partition out on any grid with the reference's own rules.
static void coarsen(slu_symb *S) {
    void *LU = slu_distribute_glu(SLU_D, S->n, S->xsup.data(), S->supno.data(), S->xlsub.data(),
                                  S->lsub.data(), S->xusub.data(), S->usub.data(), nullptr, nullptr,
                                  nullptr, 1, 1, 0, 0);
    if (!LU) throw slu::Error(slu_last_error());
    slu_lu_view v;
    slu_lu_get_view(LU, SLU_D, &v);
    const int ns = (int)S->nsupers;
    vector<const int_t *> li(ns, nullptr), ui(ns, nullptr);
    for (int s = 0; s < ns; ++s) {
        if (v.Lidx_off[s] >= 0) li[s] = v.Lidx + v.Lidx_off[s];
        if (v.Uidx_off[s] >= 0) ui[s] = v.Uidx + v.Uidx_off[s];
    }
    slu::Amalg A;
    A.programs = false; // the structure is all the coarse symbolic needs
    const bool merged = A.build(S->n, ns, S->xsup.data(), li.data(), ui.data(), 0.10, 256);
    slu_lustruct_free(LU, SLU_D);
    S->fl[0] = A.fl_schur; S->fl[1] = A.fl_trsm; S->fl[2] = A.fl_trsv;
    S->fl[3] = A.fl_s1; S->fl[4] = A.fl_s2; S->fl[5] = A.fl_w;
    if (!merged) return;
    A.coarse_glu(S->xlsub, S->lsub, S->xusub, S->usub);
    S->nsupers = A.ns2;
    S->xsup.assign(A.xsup2.begin(), A.xsup2.end());
    S->supno.assign(A.supno2.begin(), A.supno2.end());
    S->sptr.assign(S->nsupers + 1, 0);
    for (int64_t k = 0; k < S->nsupers; ++k) {
        const int64_t f = S->xsup[k];
        S->sptr[k + 1] = S->sptr[k] + (S->xlsub[f + 1] - S->xlsub[f]);
    }
}

slu_symb *slu_symbolic(const slu_csc *A, const int64_t *perm_c_in, int relax,
                       int maxsup, int flags) {
    int64_t n = A->n;
    if (maxsup < 1) maxsup = 256;
    if (relax > maxsup) relax = maxsup;
    vector<int64_t> perm(n);
    if (perm_c_in) std::copy(perm_c_in, perm_c_in + n, perm.begin());
    else std::iota(perm.begin(), perm.end(), 0);
    if (flags & SLU_SYMB_REFERENCE) {
        try {
            return symbolic_reference(A, std::move(perm), relax, maxsup, (flags & SLU_SYMB_COARSE) != 0);
        } catch (const std::exception &e) {
            slu::set_last_error(e.what());
            return nullptr;
        }
    }

    // etree of P(A+A^T)P^T, then compose perm with its postorder
    Graph g = sym_pattern(A, perm);
    vector<int64_t> parent = etree_of(g);
    vector<int64_t> post = postorder(parent);
    vector<int64_t> pinv(n);
    for (int64_t k = 0; k < n; ++k) pinv[post[k]] = k;
    for (int64_t i = 0; i < n; ++i) perm[i] = pinv[perm[i]];
    g = sym_pattern(A, perm);
    parent = etree_of(g);

    // column counts (off-diagonal) by row subtrees: O(nnz(L))
    vector<int64_t> cc(n, 0), mark(n, -1), nchild(n, 0), size(n, 1);
    for (int64_t i = 0; i < n; ++i) {
        mark[i] = i;
        for (int64_t p = g.ptr[i]; p < g.ptr[i + 1]; ++p) {
            int64_t k = g.idx[p];
            if (k >= i) break;
            while (k != -1 && k < i && mark[k] != i) {
                mark[k] = i;
                cc[k]++;
                k = parent[k];
            }
        }
    }
    for (int64_t j = 0; j < n; ++j)
        if (parent[j] >= 0) { nchild[parent[j]]++; size[parent[j]] += size[j]; }

    // supernode partition: relaxed subtrees, then fundamental chains.
    // SLU_SYMB_MULTICHILD: a chain may also continue through a column with
    // several children (their structures are nested in it)
    const bool multichild = (flags & SLU_SYMB_MULTICHILD) != 0;
    static const double AMALG_ZERO_FRAC =
        getenv("SLU_AMALG_ZERO") ? atof(getenv("SLU_AMALG_ZERO")) : 0.10;
    vector<int64_t> xsup;
    xsup.reserve(n / 4 + 2);
    int64_t j = 0;
    while (j < n) {
        // is j the first node of a relaxed subtree?  (postorder: the subtree
        // rooted at r occupies [r-size[r]+1, r])
        int64_t r = j;
        while (parent[r] != -1 && size[parent[r]] <= relax &&
               parent[r] - size[parent[r]] + 1 == j)
            r = parent[r];
        if (size[r] <= relax && r - size[r] + 1 == j) {
            for (int64_t s = j; s <= r; s += maxsup) xsup.push_back(s);
            j = r + 1;
            continue;
        }
        // Chain supernode starting at j.  A fundamental supernode needs
        // cc[c] == cc[c+1]+1 along the chain; separator planes of a nested
        // dissection break that at every border column, so (as in relaxed
        // amalgamation) a chain is extended while the explicit zeros it
        // introduces stay below AMALG_ZERO_FRAC of the stored entries.  Along
        // a chain struct(L_c)\{c} is contained in struct(L_{c+1}), so the
        // supernode's structure is [f..l] u struct(L_l): exact bookkeeping.
        xsup.push_back(j);
        int64_t f = j, len = 1;
        double sumcc = (double)cc[j];
        while (j + 1 < n && len < maxsup && parent[j] == j + 1 &&
               (nchild[j + 1] == 1 || multichild) && size[j + 1] > relax) {
            double w = (double)(len + 1), c1 = (double)cc[j + 1];
            double zeros = w * (w - 1) / 2 + w * c1 - (sumcc + c1);
            double stored = w * (w + 1) / 2 + w * c1;
            bool fundamental = cc[j] == cc[j + 1] + 1;
            if (!fundamental && zeros > AMALG_ZERO_FRAC * stored) break;
            ++j;
            ++len;
            sumcc += c1;
        }
        (void)f;
        ++j;
    }
    xsup.push_back(n);

    slu_symb *S = new slu_symb;
    S->n = n;
    S->perm = perm;
    S->nsupers = (int64_t)xsup.size() - 1;
    S->xsup = xsup;
    S->supno.resize(n);
    for (int64_t s = 0; s < S->nsupers; ++s)
        for (int64_t c = xsup[s]; c < xsup[s + 1]; ++c) S->supno[c] = s;

    // supernodal structures
    int64_t ns = S->nsupers;
    S->sparent.assign(ns, -1);
    vector<vector<int64_t>> kids(ns);
    S->sptr.assign(ns + 1, 0);
    S->srows.clear();
    vector<int64_t> mk(n, -1), below;
    for (int64_t s = 0; s < ns; ++s) {
        int64_t f = xsup[s], l = xsup[s + 1] - 1;
        below.clear();
        for (int64_t c = f; c <= l; ++c)
            for (int64_t p = g.ptr[c]; p < g.ptr[c + 1]; ++p) {
                int64_t i = g.idx[p];
                if (i > l && mk[i] != s) { mk[i] = s; below.push_back(i); }
            }
        for (int64_t c : kids[s]) {
            for (int64_t p = S->sptr[c]; p < S->sptr[c + 1]; ++p) {
                int64_t i = S->srows[p];
                if (i > l && mk[i] != s) { mk[i] = s; below.push_back(i); }
            }
        }
        std::sort(below.begin(), below.end());
        for (int64_t c = f; c <= l; ++c) S->srows.push_back(c);
        S->srows.insert(S->srows.end(), below.begin(), below.end());
        S->sptr[s + 1] = S->srows.size();
        int64_t w = l - f + 1;
        S->nnzL += (double)w * (w + 1) / 2 + (double)w * below.size();
        S->nnzU += (double)w * (w - 1) / 2 + (double)w * below.size();
        if (!below.empty()) {
            int64_t ps = S->supno[below[0]];
            S->sparent[s] = ps;
            kids[ps].push_back(s);
        }
    }
    return S;
}

void slu_symb_free(slu_symb *s) { delete s; }
int64_t slu_symb_nsupers(const slu_symb *s) { return s->nsupers; }
void slu_symb_arrays(const slu_symb *s, int64_t *xsup, int64_t *supno,
                     int64_t *perm_c) {
    if (xsup) std::copy(s->xsup.begin(), s->xsup.end(), xsup);
    if (supno) std::copy(s->supno.begin(), s->supno.end(), supno);
    if (perm_c) std::copy(s->perm.begin(), s->perm.end(), perm_c);
}
void slu_symb_struct_sizes(const slu_symb *s, int64_t *sizes) {
    // (for SLU_SYMB_REFERENCE: |struct(L_s)| from symbfact's lsub)
    for (int64_t k = 0; k < s->nsupers; ++k) sizes[k] = s->sptr[k + 1] - s->sptr[k];
}
// SLU_SYMB_REFERENCE: [nsupers of the reference's partition, then its
// algorithmic-work sums schur, trsm, trsv, s1, s2, w] (csrc/amalg.h)
void slu_symb_ref_info(const slu_symb *s, double *out) {
    out[0] = (double)s->nsupers_fine;
    for (int i = 0; i < 6; ++i) out[1 + i] = s->fl[i];
}
void slu_symb_counts(const slu_symb *s, double *nnzL, double *nnzU) {
    if (nnzL) *nnzL = s->nnzL;
    if (nnzU) *nnzU = s->nnzU;
}

slu_csc *slu_permute(const slu_csc *A, const int64_t *perm) {
    int64_t n = A->n;
    size_t vs = vsize(A->dtype);
    vector<int64_t> iperm(n);
    for (int64_t i = 0; i < n; ++i) iperm[perm[i]] = i;
    slu_csc *B = (slu_csc *)calloc(1, sizeof(slu_csc));
    B->n = n;
    B->nnz = A->nnz;
    B->dtype = A->dtype;
    B->colptr = (int64_t *)malloc((n + 1) * sizeof(int64_t));
    B->rowind = (int64_t *)malloc(std::max<int64_t>(A->nnz, 1) * sizeof(int64_t));
    B->val = malloc(std::max<int64_t>(A->nnz, 1) * vs);
    int64_t w = 0;
    vector<std::pair<int64_t, int64_t>> col;
    for (int64_t jn = 0; jn < n; ++jn) {
        B->colptr[jn] = w;
        int64_t jo = iperm[jn];
        col.clear();
        for (int64_t p = A->colptr[jo]; p < A->colptr[jo + 1]; ++p)
            col.push_back({perm[A->rowind[p]], p});
        std::sort(col.begin(), col.end());
        for (auto &e : col) {
            B->rowind[w] = e.first;
            memcpy((char *)B->val + w * vs, (char *)A->val + e.second * vs, vs);
            ++w;
        }
    }
    B->colptr[n] = w;
    return B;
}

} // extern "C"

// ----------------------------------------------------------------------------
// Distribution.
namespace {

template <typename T, typename LocalLU, typename LUstruct>
void *distribute_t(const slu_symb *S, const slu_csc *A, int Pr, int Pc,
                   int myrow, int mycol) {
    const int64_t n = S->n, ns = S->nsupers;
    const vector<int64_t> &xsup = S->xsup, &supno = S->supno;
    slu_csc *B = slu_permute(A, S->perm.data());
    const T *bval = (const T *)B->val;

    LUstruct *LU = (LUstruct *)calloc(1, sizeof(LUstruct));
    LU->Glu_persist = (Glu_persist_t *)calloc(1, sizeof(Glu_persist_t));
    LU->Glu_persist->xsup = (int_t *)malloc((ns + 1) * sizeof(int_t));
    LU->Glu_persist->supno = (int_t *)malloc(n * sizeof(int_t));
    std::copy(xsup.begin(), xsup.end(), LU->Glu_persist->xsup);
    std::copy(supno.begin(), supno.end(), LU->Glu_persist->supno);
    LocalLU *Llu = (LocalLU *)calloc(1, sizeof(LocalLU));
    LU->Llu = Llu;
    LU->dt = sizeof(T) == 4 ? 's' : sizeof(T) == 8 ? 'd' : 'z';

    auto W = [&](int64_t s) { return xsup[s + 1] - xsup[s]; };
    const int64_t nlc = (ns + Pc - 1) / Pc; // local block columns
    const int64_t nlr = (ns + Pr - 1) / Pr; // local block rows

    // ---- global buffer maxima (every rank computes the same numbers) ----
    int_t bufmax[SLU_NBUFFERS] = {0, 0, 0, 0, 0};
    {
        vector<int64_t> rowsin(Pr), blksin(Pr);
        for (int64_t s = 0; s < ns; ++s) {
            std::fill(rowsin.begin(), rowsin.end(), 0);
            std::fill(blksin.begin(), blksin.end(), 0);
            int64_t last = -1;
            for (int64_t p = S->sptr[s]; p < S->sptr[s + 1]; ++p) {
                int64_t gb = supno[S->srows[p]];
                rowsin[gb % Pr]++;
                if (gb != last) { blksin[gb % Pr]++; last = gb; }
            }
            for (int pr = 0; pr < Pr; ++pr)
                if (rowsin[pr]) {
                    int64_t len = rowsin[pr];
                    int64_t len1 = len + SLU_BC_HEADER + blksin[pr] * SLU_LB_DESCRIPTOR;
                    bufmax[0] = std::max<int64_t>(bufmax[0], len1);
                    bufmax[1] = std::max<int64_t>(bufmax[1], len * W(s));
                    bufmax[4] = std::max<int64_t>(bufmax[4], len);
                }
            // U block row s: blocks jb (struct rows below diag), per column
            // process: nnz and index length
            vector<int64_t> ulen(Pc, 0), uidx(Pc, 0), ublk(Pc, 0);
            int64_t w = W(s);
            last = -1;
            for (int64_t p = S->sptr[s] + w; p < S->sptr[s + 1]; ++p) {
                int64_t jb = supno[S->srows[p]];
                ulen[jb % Pc] += w;
                if (jb != last) { ublk[jb % Pc]++; uidx[jb % Pc] += W(jb); last = jb; }
            }
            for (int pc = 0; pc < Pc; ++pc)
                if (ulen[pc]) {
                    int64_t len1 = uidx[pc] + SLU_BR_HEADER + ublk[pc] * SLU_UB_DESCRIPTOR;
                    bufmax[2] = std::max<int64_t>(bufmax[2], len1);
                    bufmax[3] = std::max<int64_t>(bufmax[3], ulen[pc]);
                }
        }
    }
    for (int i = 0; i < SLU_NBUFFERS; ++i) Llu->bufmax[i] = bufmax[i];

    // ---- L block columns ----
    Llu->Lrowind_bc_ptr = (int_t **)calloc(nlc, sizeof(int_t *));
    Llu->Lnzval_bc_ptr = (T **)calloc(nlc, sizeof(T *));
    Llu->Lrowind_bc_offset = (long *)malloc(nlc * sizeof(long));
    Llu->Lnzval_bc_offset = (long *)malloc(nlc * sizeof(long));
    // sizes first
    vector<int64_t> lidx_len(nlc, 0), lval_len(nlc, 0);
    int64_t lidx_tot = 0, lval_tot = 0;
    for (int64_t jb = mycol; jb < ns; jb += Pc) {
        int64_t ljb = jb / Pc, len = 0, nb = 0, last = -1;
        for (int64_t p = S->sptr[jb]; p < S->sptr[jb + 1]; ++p) {
            int64_t gb = supno[S->srows[p]];
            if (gb % Pr != myrow) continue;
            ++len;
            if (gb != last) { ++nb; last = gb; }
        }
        if (len) {
            lidx_len[ljb] = len + SLU_BC_HEADER + nb * SLU_LB_DESCRIPTOR;
            lval_len[ljb] = len * W(jb);
        }
    }
    for (int64_t ljb = 0; ljb < nlc; ++ljb) {
        if (lidx_len[ljb]) {
            Llu->Lrowind_bc_offset[ljb] = lidx_tot;
            Llu->Lnzval_bc_offset[ljb] = lval_tot;
            lidx_tot += lidx_len[ljb];
            lval_tot += lval_len[ljb];
        } else {
            Llu->Lrowind_bc_offset[ljb] = -1;
            Llu->Lnzval_bc_offset[ljb] = -1;
        }
    }
    Llu->Lrowind_bc_dat = (int_t *)calloc(lidx_tot + 1, sizeof(int_t));
    Llu->Lnzval_bc_dat = (T *)calloc(lval_tot + 1, sizeof(T));
    Llu->Lrowind_bc_cnt = lidx_tot + 1;
    Llu->Lnzval_bc_cnt = lval_tot + 1;

    vector<int64_t> rowpos(n, -1);
    for (int64_t jb = mycol; jb < ns; jb += Pc) {
        int64_t ljb = jb / Pc;
        if (!lidx_len[ljb]) continue;
        int_t *index = Llu->Lrowind_bc_dat + Llu->Lrowind_bc_offset[ljb];
        T *lusup = Llu->Lnzval_bc_dat + Llu->Lnzval_bc_offset[ljb];
        Llu->Lrowind_bc_ptr[ljb] = index;
        Llu->Lnzval_bc_ptr[ljb] = lusup;
        int64_t nsupr = lval_len[ljb] / W(jb);
        index[0] = 0;
        index[1] = nsupr;
        int64_t w = SLU_BC_HEADER, r = 0, last = -1, desc = -1;
        for (int64_t p = S->sptr[jb]; p < S->sptr[jb + 1]; ++p) {
            int64_t gr = S->srows[p], gb = supno[gr];
            if (gb % Pr != myrow) continue;
            if (gb != last) {
                index[0]++;
                desc = w;
                index[w++] = gb;
                index[w++] = 0;
                last = gb;
            }
            index[desc + 1]++;
            index[w++] = gr;
            rowpos[gr] = r++;
        }
        // values of B in the block column
        for (int64_t c = xsup[jb]; c < xsup[jb + 1]; ++c) {
            int64_t cc = c - xsup[jb];
            for (int64_t p = B->colptr[c]; p < B->colptr[c + 1]; ++p) {
                int64_t gr = B->rowind[p];
                if (gr < xsup[jb]) continue;       // U part
                if (supno[gr] % Pr != myrow) continue;
                lusup[rowpos[gr] + cc * nsupr] = bval[p];
            }
        }
        for (int64_t p = S->sptr[jb]; p < S->sptr[jb + 1]; ++p) rowpos[S->srows[p]] = -1;
    }

    // ---- U block rows ----
    Llu->Ufstnz_br_ptr = (int_t **)calloc(nlr, sizeof(int_t *));
    Llu->Unzval_br_ptr = (T **)calloc(nlr, sizeof(T *));
    Llu->Ufstnz_br_offset = (long *)malloc(nlr * sizeof(long));
    Llu->Unzval_br_offset = (long *)malloc(nlr * sizeof(long));
    vector<int64_t> uidx_len(nlr, 0), uval_len(nlr, 0);
    int64_t uidx_tot = 0, uval_tot = 0;
    for (int64_t gb = myrow; gb < ns; gb += Pr) {
        int64_t lb = gb / Pr, w = W(gb), len = 0, idx = 0, nb = 0, last = -1;
        for (int64_t p = S->sptr[gb] + w; p < S->sptr[gb + 1]; ++p) {
            int64_t jb = supno[S->srows[p]];
            if (jb % Pc != mycol) continue;
            len += w;
            if (jb != last) { ++nb; idx += W(jb); last = jb; }
        }
        if (len) {
            uidx_len[lb] = idx + SLU_BR_HEADER + nb * SLU_UB_DESCRIPTOR + 1;
            uval_len[lb] = len;
        }
    }
    for (int64_t lb = 0; lb < nlr; ++lb) {
        if (uidx_len[lb]) {
            Llu->Ufstnz_br_offset[lb] = uidx_tot;
            Llu->Unzval_br_offset[lb] = uval_tot;
            uidx_tot += uidx_len[lb];
            uval_tot += uval_len[lb];
        } else {
            Llu->Ufstnz_br_offset[lb] = -1;
            Llu->Unzval_br_offset[lb] = -1;
        }
    }
    Llu->Ufstnz_br_dat = (int_t *)calloc(uidx_tot + 1, sizeof(int_t));
    Llu->Unzval_br_dat = (T *)calloc(uval_tot + 1, sizeof(T));
    Llu->Ufstnz_br_cnt = uidx_tot + 1;
    Llu->Unzval_br_cnt = uval_tot + 1;
    // per U block row: value offset of column gc's segment (full segments)
    vector<int64_t> ucoloff(n, -1);
    for (int64_t gb = myrow; gb < ns; gb += Pr) {
        int64_t lb = gb / Pr, w = W(gb);
        if (!uidx_len[lb]) continue;
        int_t *index = Llu->Ufstnz_br_dat + Llu->Ufstnz_br_offset[lb];
        T *uval = Llu->Unzval_br_dat + Llu->Unzval_br_offset[lb];
        Llu->Ufstnz_br_ptr[lb] = index;
        Llu->Unzval_br_ptr[lb] = uval;
        int64_t len1 = uidx_len[lb] - 1;
        index[0] = 0;
        index[1] = uval_len[lb];
        index[2] = len1;
        index[len1] = -1;
        int64_t iw = SLU_BR_HEADER, voff = 0, last = -1, desc = -1;
        for (int64_t p = S->sptr[gb] + w; p < S->sptr[gb + 1]; ++p) {
            int64_t gc = S->srows[p], jb = supno[gc];
            if (jb % Pc != mycol) continue;
            if (jb != last) {
                index[0]++;
                desc = iw;
                index[iw++] = jb;
                index[iw++] = 0;
                for (int64_t c = 0; c < W(jb); ++c) index[iw + c] = xsup[gb + 1];
                iw += W(jb);
                last = jb;
            }
            index[desc + 1] += w;
            index[desc + 2 + (gc - xsup[jb])] = xsup[gb];
            ucoloff[gc] = voff;
            voff += w;
        }
        // values: U(gb, gc) for gc in my process column
        for (int64_t p = S->sptr[gb] + w; p < S->sptr[gb + 1]; ++p) {
            int64_t gc = S->srows[p];
            if (supno[gc] % Pc != mycol) continue;
            for (int64_t q = B->colptr[gc]; q < B->colptr[gc + 1]; ++q) {
                int64_t gr = B->rowind[q];
                if (gr < xsup[gb] || gr >= xsup[gb + 1]) continue;
                uval[ucoloff[gc] + gr - xsup[gb]] = bval[q];
            }
        }
        for (int64_t p = S->sptr[gb] + w; p < S->sptr[gb + 1]; ++p) ucoloff[S->srows[p]] = -1;
    }

    // ---- communication schedule (SRC/pddistribute.c:752-801) ----
    Llu->ToRecv = (int *)calloc(ns, sizeof(int));
    Llu->ToSendD = (int *)calloc(nlr, sizeof(int));
    Llu->ToSendR = (int **)malloc(nlc * sizeof(int *));
    int *tsr = (int *)malloc(std::max<int64_t>(nlc * Pc, 1) * sizeof(int));
    for (int64_t i = 0; i < nlc * Pc; ++i) tsr[i] = SLU_EMPTY;
    for (int64_t i = 0; i < nlc; ++i) Llu->ToSendR[i] = tsr + i * Pc;
    for (int64_t gb = 0; gb < ns; ++gb) {
        int64_t w = W(gb);
        int kcol = gb % Pc;
        for (int64_t p = S->sptr[gb] + w; p < S->sptr[gb + 1]; ++p) {
            int64_t jb = supno[S->srows[p]];
            int pc = jb % Pc;
            if (mycol == kcol && mycol != pc) Llu->ToSendR[gb / Pc][pc] = 1;
            if (mycol == pc) {
                if (myrow == gb % Pr) {
                    Llu->ToSendD[gb / Pr] = 1;
                    Llu->ToRecv[gb] = 1;
                } else
                    Llu->ToRecv[gb] = 2;
            }
        }
    }
    slu_csc_free(B);
    return LU;
}

// An LUstruct holding arrays made elsewhere (e.g. dumped from the reference's
// own pddistribute, tests/golden/refdump_*): the flat index / value arrays
// with per local block column / row offsets (-1 = empty), laid out as
// SRC/pddistribute.c:1283-1340, 1465-1493 lays out its *_dat arrays.
template <typename T, typename LocalLU, typename LUstruct>
void *build_t(int64_t n, int64_t ns, const int_t *xsup, const int_t *supno, int Pr, int Pc,
              const int_t *Lidx, int64_t Lidx_cnt, const int64_t *Loff, const void *Lval,
              int64_t Lval_cnt, const int64_t *Lvoff, const int_t *Uidx, int64_t Uidx_cnt,
              const int64_t *Uoff, const void *Uval, int64_t Uval_cnt, const int64_t *Uvoff,
              const int *ToRecv, const int *ToSendD, const int *ToSendR, const int_t *bufmax) {
    LUstruct *LU = (LUstruct *)calloc(1, sizeof(LUstruct));
    LU->Glu_persist = (Glu_persist_t *)calloc(1, sizeof(Glu_persist_t));
    LU->Glu_persist->xsup = (int_t *)malloc((ns + 1) * sizeof(int_t));
    LU->Glu_persist->supno = (int_t *)malloc(n * sizeof(int_t));
    std::copy(xsup, xsup + ns + 1, LU->Glu_persist->xsup);
    std::copy(supno, supno + n, LU->Glu_persist->supno);
    LocalLU *Llu = (LocalLU *)calloc(1, sizeof(LocalLU));
    LU->Llu = Llu;
    LU->dt = sizeof(T) == 4 ? 's' : sizeof(T) == 8 ? 'd' : 'z';
    const int64_t nlc = (ns + Pc - 1) / Pc, nlr = (ns + Pr - 1) / Pr;
    for (int i = 0; i < SLU_NBUFFERS; ++i) Llu->bufmax[i] = bufmax[i];
    Llu->Lrowind_bc_dat = (int_t *)calloc(Lidx_cnt + 1, sizeof(int_t));
    Llu->Lnzval_bc_dat = (T *)calloc(Lval_cnt + 1, sizeof(T));
    Llu->Lrowind_bc_cnt = Lidx_cnt + 1;
    Llu->Lnzval_bc_cnt = Lval_cnt + 1;
    if (Lidx_cnt) memcpy(Llu->Lrowind_bc_dat, Lidx, Lidx_cnt * sizeof(int_t));
    if (Lval_cnt) memcpy(Llu->Lnzval_bc_dat, Lval, Lval_cnt * sizeof(T));
    Llu->Lrowind_bc_ptr = (int_t **)calloc(std::max<int64_t>(nlc, 1), sizeof(int_t *));
    Llu->Lnzval_bc_ptr = (T **)calloc(std::max<int64_t>(nlc, 1), sizeof(T *));
    Llu->Lrowind_bc_offset = (long *)malloc(std::max<int64_t>(nlc, 1) * sizeof(long));
    Llu->Lnzval_bc_offset = (long *)malloc(std::max<int64_t>(nlc, 1) * sizeof(long));
    for (int64_t j = 0; j < nlc; ++j) {
        Llu->Lrowind_bc_offset[j] = Loff[j];
        Llu->Lnzval_bc_offset[j] = Lvoff[j];
        if (Loff[j] >= 0) {
            Llu->Lrowind_bc_ptr[j] = Llu->Lrowind_bc_dat + Loff[j];
            Llu->Lnzval_bc_ptr[j] = Llu->Lnzval_bc_dat + Lvoff[j];
        }
    }
    Llu->Ufstnz_br_dat = (int_t *)calloc(Uidx_cnt + 1, sizeof(int_t));
    Llu->Unzval_br_dat = (T *)calloc(Uval_cnt + 1, sizeof(T));
    Llu->Ufstnz_br_cnt = Uidx_cnt + 1;
    Llu->Unzval_br_cnt = Uval_cnt + 1;
    if (Uidx_cnt) memcpy(Llu->Ufstnz_br_dat, Uidx, Uidx_cnt * sizeof(int_t));
    if (Uval_cnt) memcpy(Llu->Unzval_br_dat, Uval, Uval_cnt * sizeof(T));
    Llu->Ufstnz_br_ptr = (int_t **)calloc(std::max<int64_t>(nlr, 1), sizeof(int_t *));
    Llu->Unzval_br_ptr = (T **)calloc(std::max<int64_t>(nlr, 1), sizeof(T *));
    Llu->Ufstnz_br_offset = (long *)malloc(std::max<int64_t>(nlr, 1) * sizeof(long));
    Llu->Unzval_br_offset = (long *)malloc(std::max<int64_t>(nlr, 1) * sizeof(long));
    for (int64_t j = 0; j < nlr; ++j) {
        Llu->Ufstnz_br_offset[j] = Uoff[j];
        Llu->Unzval_br_offset[j] = Uvoff[j];
        if (Uoff[j] >= 0) {
            Llu->Ufstnz_br_ptr[j] = Llu->Ufstnz_br_dat + Uoff[j];
            Llu->Unzval_br_ptr[j] = Llu->Unzval_br_dat + Uvoff[j];
        }
    }
    Llu->ToRecv = (int *)calloc(std::max<int64_t>(ns, 1), sizeof(int));
    Llu->ToSendD = (int *)calloc(std::max<int64_t>(nlr, 1), sizeof(int));
    Llu->ToSendR = (int **)malloc(std::max<int64_t>(nlc, 1) * sizeof(int *));
    int *tsr = (int *)malloc(std::max<int64_t>(nlc * Pc, 1) * sizeof(int));
    if (ToRecv) memcpy(Llu->ToRecv, ToRecv, ns * sizeof(int));
    if (ToSendD) memcpy(Llu->ToSendD, ToSendD, nlr * sizeof(int));
    for (int64_t i = 0; i < nlc * Pc; ++i) tsr[i] = ToSendR ? ToSendR[i] : SLU_EMPTY;
    for (int64_t i = 0; i < nlc; ++i) Llu->ToSendR[i] = tsr + i * Pc;
    return LU;
}

template <typename LocalLU, typename LUstruct>
void free_t(void *p) {
    LUstruct *LU = (LUstruct *)p;
    if (!LU) return;
    LocalLU *Llu = LU->Llu;
    if (Llu) {
        free(Llu->Lrowind_bc_ptr);
        free(Llu->Lnzval_bc_ptr);
        free(Llu->Lrowind_bc_offset);
        free(Llu->Lnzval_bc_offset);
        free(Llu->Lrowind_bc_dat);
        free(Llu->Lnzval_bc_dat);
        free(Llu->Ufstnz_br_ptr);
        free(Llu->Unzval_br_ptr);
        free(Llu->Ufstnz_br_offset);
        free(Llu->Unzval_br_offset);
        free(Llu->Ufstnz_br_dat);
        free(Llu->Unzval_br_dat);
        free(Llu->ToRecv);
        free(Llu->ToSendD);
        if (Llu->ToSendR) free(Llu->ToSendR[0]);
        free(Llu->ToSendR);
        free(Llu);
    }
    if (LU->Glu_persist) {
        free(LU->Glu_persist->xsup);
        free(LU->Glu_persist->supno);
        free(LU->Glu_persist);
    }
    free(LU);
}

} // namespace

namespace {
template <typename LocalLU, typename LUstruct>
int view_t(void *p, slu_lu_view *v) {
    LUstruct *LU = (LUstruct *)p;
    LocalLU *L = LU->Llu;
    memset(v, 0, sizeof(*v));
    v->xsup = LU->Glu_persist->xsup;
    v->supno = LU->Glu_persist->supno;
    v->Lidx = L->Lrowind_bc_dat; v->Lidx_cnt = L->Lrowind_bc_cnt; v->Lidx_off = L->Lrowind_bc_offset;
    v->Lval = L->Lnzval_bc_dat; v->Lval_cnt = L->Lnzval_bc_cnt; v->Lval_off = L->Lnzval_bc_offset;
    v->Uidx = L->Ufstnz_br_dat; v->Uidx_cnt = L->Ufstnz_br_cnt; v->Uidx_off = L->Ufstnz_br_offset;
    v->Uval = L->Unzval_br_dat; v->Uval_cnt = L->Unzval_br_cnt; v->Uval_off = L->Unzval_br_offset;
    v->ToRecv = L->ToRecv; v->ToSendD = L->ToSendD; v->ToSendR = L->ToSendR;
    for (int i = 0; i < SLU_NBUFFERS; ++i) v->bufmax[i] = L->bufmax[i];
    return 0;
}

} // namespace

extern "C" {

void *slu_distribute(const slu_symb *s, const slu_csc *A, int nprow,
                     int npcol, int myrow, int mycol) {
    if (s->ref) {
        // the reference's pddistribute on Pc A Pc^T (csrc/distribute.cpp)
        slu_csc *B = slu_permute(A, s->perm.data());
        void *LU = slu_distribute_glu(A->dtype, s->n, s->xsup.data(), s->supno.data(),
                                      s->xlsub.data(), s->lsub.data(), s->xusub.data(),
                                      s->usub.data(), B->colptr, B->rowind, B->val, nprow, npcol,
                                      myrow, mycol);
        slu_csc_free(B);
        return LU;
    }
    switch (A->dtype) {
    case SLU_D: return distribute_t<double, dLocalLU_t, dLUstruct_t>(s, A, nprow, npcol, myrow, mycol);
    case SLU_S: return distribute_t<float, sLocalLU_t, sLUstruct_t>(s, A, nprow, npcol, myrow, mycol);
    case SLU_Z: return distribute_t<doublecomplex, zLocalLU_t, zLUstruct_t>(s, A, nprow, npcol, myrow, mycol);
    }
    return nullptr;
}

void *slu_lustruct_build(int dtype, int64_t n, int64_t nsupers, const int_t *xsup,
                         const int_t *supno, int nprow, int npcol, const int_t *Lidx,
                         int64_t Lidx_cnt, const int64_t *Loff, const void *Lval, int64_t Lval_cnt,
                         const int64_t *Lvoff, const int_t *Uidx, int64_t Uidx_cnt,
                         const int64_t *Uoff, const void *Uval, int64_t Uval_cnt,
                         const int64_t *Uvoff, const int *ToRecv, const int *ToSendD,
                         const int *ToSendR, const int_t *bufmax) {
#define SLU_BUILD_ARGS                                                                             \
    n, nsupers, xsup, supno, nprow, npcol, Lidx, Lidx_cnt, Loff, Lval, Lval_cnt, Lvoff, Uidx,      \
        Uidx_cnt, Uoff, Uval, Uval_cnt, Uvoff, ToRecv, ToSendD, ToSendR, bufmax
    switch (dtype) {
    case SLU_D: return build_t<double, dLocalLU_t, dLUstruct_t>(SLU_BUILD_ARGS);
    case SLU_S: return build_t<float, sLocalLU_t, sLUstruct_t>(SLU_BUILD_ARGS);
    case SLU_Z: return build_t<doublecomplex, zLocalLU_t, zLUstruct_t>(SLU_BUILD_ARGS);
    }
#undef SLU_BUILD_ARGS
    return nullptr;
}

int slu_lu_get_view(void *LU, int dtype, slu_lu_view *v) {
    switch (dtype) {
    case SLU_D: return view_t<dLocalLU_t, dLUstruct_t>(LU, v);
    case SLU_S: return view_t<sLocalLU_t, sLUstruct_t>(LU, v);
    case SLU_Z: return view_t<zLocalLU_t, zLUstruct_t>(LU, v);
    }
    return -1;
}

void slu_lustruct_free(void *LU, int dtype) {
    switch (dtype) {
    case SLU_D: free_t<dLocalLU_t, dLUstruct_t>(LU); break;
    case SLU_S: free_t<sLocalLU_t, sLUstruct_t>(LU); break;
    case SLU_Z: free_t<zLocalLU_t, zLUstruct_t>(LU); break;
    }
}

} // extern "C"

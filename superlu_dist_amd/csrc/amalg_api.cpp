// C API of the engine-side amalgamation (csrc/amalg.h) for the CPU tests:
// opt-in library only (full.map exports slu_*).
#include <algorithm>
#include <complex>
#include <memory>

#include "amalg.h"
#include "common.h"
#include "slu_mi355x.h"

// ---- C API for the tests (opt-in library only, full.map)
using slu::Amalg;

extern "C" {

// amalgamation of a 1x1 LUstruct (dtype d/s/z); NULL when nothing merges
// or on error (slu_last_error)
void *slu_amalg_create(int dtype, void *LU, int64_t n, double zero_frac, int maxw) {
    try {
        slu_lu_view v;
        if (slu_lu_get_view(LU, dtype, &v)) throw slu::Error("bad dtype");
        const int ns = (int)(v.supno[n - 1] + 1);
        std::vector<const int_t *> li(ns, nullptr), ui(ns, nullptr);
        for (int s = 0; s < ns; ++s) {
            if (v.Lidx_off[s] >= 0) li[s] = v.Lidx + v.Lidx_off[s];
            if (v.Uidx_off[s] >= 0) ui[s] = v.Uidx + v.Uidx_off[s];
        }
        auto *A = new Amalg;
        if (!A->build(n, ns, v.xsup, li.data(), ui.data(), zero_frac, maxw)) {
            delete A;
            slu::set_last_error("amalgamation: nothing merges");
            return nullptr;
        }
        return A;
    } catch (const std::exception &e) {
        slu::set_last_error(e.what());
        return nullptr;
    }
}

// sizes: [ns1, ns2, |Lidx2|, |Uidx2|, lval2, uval2, merged groups, explicit zeros]
void slu_amalg_sizes(const void *h, int64_t *out) {
    const Amalg *A = (const Amalg *)h;
    out[0] = A->ns1;
    out[1] = A->ns2;
    out[2] = (int64_t)A->Lidx2.size();
    out[3] = (int64_t)A->Uidx2.size();
    out[4] = A->lval2;
    out[5] = A->uval2;
    out[6] = A->n_merged_groups;
    out[7] = A->zeros;
}

void slu_amalg_arrays(const void *h, int64_t *xsup2, int64_t *supno2, int64_t *Lidx2,
                      int64_t *Loff2, int64_t *Lvoff2, int64_t *Uidx2, int64_t *Uoff2,
                      int64_t *Uvoff2) {
    const Amalg *A = (const Amalg *)h;
    std::copy(A->xsup2.begin(), A->xsup2.end(), xsup2);
    std::copy(A->supno2.begin(), A->supno2.end(), supno2);
    std::copy(A->Lidx2.data(), A->Lidx2.data() + A->Lidx2.size(), Lidx2);
    std::copy(A->Loff2.begin(), A->Loff2.end(), Loff2);
    std::copy(A->Lvoff2.begin(), A->Lvoff2.end(), Lvoff2);
    std::copy(A->Uidx2.data(), A->Uidx2.data() + A->Uidx2.size(), Uidx2);
    std::copy(A->Uoff2.begin(), A->Uoff2.end(), Uoff2);
    std::copy(A->Uvoff2.begin(), A->Uvoff2.end(), Uvoff2);
}

// host expand (dir 0: original -> zeroed merged) / compress (dir 1)
int slu_amalg_apply(const void *h, int dtype, void *oL, void *oU, void *mL, void *mU, int dir) {
    const Amalg *A = (const Amalg *)h;
    switch (dtype) {
    case SLU_D: A->apply((double *)oL, (double *)oU, (double *)mL, (double *)mU, dir); return 0;
    case SLU_S: A->apply((float *)oL, (float *)oU, (float *)mL, (float *)mU, dir); return 0;
    case SLU_Z:
        A->apply((std::complex<double> *)oL, (std::complex<double> *)oU, (std::complex<double> *)mL,
                 (std::complex<double> *)mU, dir);
        return 0;
    }
    return -1;
}

// the original partition's algorithmic flops for value type dtype (as the
// plan reports them): [schur, panel]
void slu_amalg_flops(const void *h, int dtype, double *out) {
    const Amalg *A = (const Amalg *)h;
    const bool cp = dtype == SLU_Z;
    out[0] = A->fl_schur * (cp ? 4.0 : 1.0);
    out[1] = (cp ? 6 * A->fl_s1 + 10 * A->fl_w + 8 * A->fl_s2 : A->fl_s1 + 2 * A->fl_s2) +
             (cp ? 4.0 : 1.0) * A->fl_trsm + A->fl_trsv;
}

void slu_amalg_free(void *h) { delete (Amalg *)h; }

} // extern "C"

// ---- grids: every rank of a Pr x Pc grid in one process (amalg.h
// "grids"), the phases run rank by rank with the streams handed over in
// memory -- what the engine's GridAmalgPlan does with its transport.
struct GaSim {
    int Pr = 1, Pc = 1, dtype = 0;
    int64_t n = 0;
    std::vector<slu::GaFine> f;
    std::vector<std::vector<const int_t *>> li, ui;
    slu::GaPartition g;
    std::vector<slu::GaChains> ch;
    std::vector<slu::GaRelay> r;
};

template <typename T>
static void gamalg_apply(const GaSim *S, void **oL, void **oU, void **mL, void **mU, int dir);

extern "C" {

// lus[r * Pc + c] = rank (r, c)'s LUstruct; NULL on error (slu_last_error)
void *slu_gamalg_create(int dtype, int nranks, void **lus, int64_t n, int pr, int pc, double zero_frac,
                        int maxw) {
    try {
        SLU_REQUIRE(nranks == pr * pc && nranks >= 1, "grid amalgamation: %d LUstructs for %dx%d", nranks, pr, pc);
        auto *S = new GaSim;
        std::unique_ptr<GaSim> own(S);
        S->Pr = pr;
        S->Pc = pc;
        S->dtype = dtype;
        S->n = n;
        S->f.resize(nranks);
        S->li.resize(nranks);
        S->ui.resize(nranks);
        for (int k = 0; k < nranks; ++k) {
            slu_lu_view v;
            if (slu_lu_get_view(lus[k], dtype, &v)) throw slu::Error("bad dtype");
            slu::GaFine &F = S->f[k];
            F.n = n;
            F.ns = (int)(v.supno[n - 1] + 1);
            F.Pr = pr;
            F.Pc = pc;
            F.myrow = k / pc;
            F.mycol = k % pc;
            F.xsup = v.xsup;
            S->li[k].assign(F.nlc(), nullptr);
            S->ui[k].assign(F.nlr(), nullptr);
            for (int j = 0; j < F.nlc(); ++j)
                if (v.Lidx_off[j] >= 0) S->li[k][j] = v.Lidx + v.Lidx_off[j];
            for (int j = 0; j < F.nlr(); ++j)
                if (v.Uidx_off[j] >= 0) S->ui[k][j] = v.Uidx + v.Uidx_off[j];
            F.lidx = S->li[k].data();
            F.uidx = S->ui[k].data();
        }
        // phase 1: structure to the analysis owners, chains per range
        std::vector<slu::GaStreams> out(nranks);
        for (int k = 0; k < nranks; ++k) out[k] = slu::ga_structure_out(S->f[k]);
        std::vector<std::vector<int64_t>> gst(nranks);
        S->ch.resize(nranks);
        for (int k = 0; k < nranks; ++k) {
            slu::GaStreams in(nranks);
            for (int src = 0; src < nranks; ++src) in[src] = out[src][k];
            S->ch[k] = slu::ga_analyse(S->f[k], in, zero_frac, maxw);
            gst[k] = S->ch[k].gstart;
        }
        // phase 2 + 3
        S->g = slu::ga_partition(S->f[0], gst);
        S->r.resize(nranks);
        for (int k = 0; k < nranks; ++k) slu::ga_send_side(S->f[k], S->g, S->r[k]);
        for (int k = 0; k < nranks; ++k) {
            slu::GaStreams in(nranks);
            for (int src = 0; src < nranks; ++src) in[src] = S->r[src].sstruct[k];
            slu::ga_receive_side(S->f[k], S->g, in, S->r[k]);
        }
        for (int k = 0; k < nranks; ++k)
            for (int src = 0; src < nranks; ++src)
                SLU_REQUIRE(S->r[src].scount[k] == S->r[k].rcount[src], "grid amalgamation: %d -> %d counts", src, k);
        return own.release();
    } catch (const std::exception &e) {
        slu::set_last_error(e.what());
        return nullptr;
    }
}

// sizes of rank k: [ns1, ns2, |Lidx2|, |Uidx2|, lval2, uval2, nlc2, nlr2]
void slu_gamalg_sizes(const void *h, int k, int64_t *out) {
    const GaSim *S = (const GaSim *)h;
    const slu::GaRelay &r = S->r[k];
    int64_t nli = 0, nui = 0;
    for (auto &v : r.Lidx2) nli += (int64_t)v.size();
    for (auto &v : r.Uidx2) nui += (int64_t)v.size();
    out[0] = S->f[k].ns;
    out[1] = S->g.ns2;
    out[2] = nli;
    out[3] = nui;
    out[4] = r.lval2;
    out[5] = r.uval2;
    out[6] = r.nlc2;
    out[7] = r.nlr2;
}

// rank k's coarse LUstruct in slu_lustruct_build's flat form
void slu_gamalg_arrays(const void *h, int k, int64_t *xsup2, int64_t *supno2, int64_t *Lidx2,
                       int64_t *Loff2, int64_t *Lvoff2, int64_t *Uidx2, int64_t *Uoff2, int64_t *Uvoff2) {
    const GaSim *S = (const GaSim *)h;
    const slu::GaRelay &r = S->r[k];
    std::copy(S->g.xsup2.begin(), S->g.xsup2.end(), xsup2);
    std::copy(S->g.supno2.begin(), S->g.supno2.end(), supno2);
    int64_t o = 0;
    for (int j = 0; j < r.nlc2; ++j) {
        Loff2[j] = r.Lidx2[j].empty() ? -1 : o;
        Lvoff2[j] = r.Lvoff2[j];
        std::copy(r.Lidx2[j].begin(), r.Lidx2[j].end(), Lidx2 + o);
        o += (int64_t)r.Lidx2[j].size();
    }
    o = 0;
    for (int j = 0; j < r.nlr2; ++j) {
        Uoff2[j] = r.Uidx2[j].empty() ? -1 : o;
        Uvoff2[j] = r.Uvoff2[j];
        std::copy(r.Uidx2[j].begin(), r.Uidx2[j].end(), Uidx2 + o);
        o += (int64_t)r.Uidx2[j].size();
    }
}

// [schur, panel] flops of the original partition summed over the ranks'
// analysis ranges (each rank's plan reports its range's share)
void slu_gamalg_flops(const void *h, int dtype, double *out) {
    const GaSim *S = (const GaSim *)h;
    const bool cp = dtype == SLU_Z;
    out[0] = out[1] = 0;
    for (const slu::GaChains &c : S->ch) {
        const slu::AmalgFlops &F = c.fl;
        out[0] += F.schur * (cp ? 4.0 : 1.0);
        out[1] += (cp ? 6 * F.s1 + 10 * F.w + 8 * F.s2 : F.s1 + 2 * F.s2) + (cp ? 4.0 : 1.0) * F.trsm + F.trsv;
    }
}

// dir 0: every rank's caller values -> its (zeroed) coarse values; dir 1 back
int slu_gamalg_apply(const void *h, int dtype, void **oL, void **oU, void **mL, void **mU, int dir) {
    const GaSim *S = (const GaSim *)h;
    switch (dtype) {
    case SLU_D: gamalg_apply<double>(S, oL, oU, mL, mU, dir); return 0;
    case SLU_S: gamalg_apply<float>(S, oL, oU, mL, mU, dir); return 0;
    case SLU_Z: gamalg_apply<std::complex<double>>(S, oL, oU, mL, mU, dir); return 0;
    }
    return -1;
}

void slu_gamalg_free(void *h) { delete (GaSim *)h; }

} // extern "C"

template <typename T>
static void gamalg_apply(const GaSim *S, void **oL, void **oU, void **mL, void **mU, int dir) {
    const int P = S->Pr * S->Pc;
    std::vector<std::vector<T>> send(P), recv(P);
    for (int k = 0; k < P; ++k) {
        send[k].assign(S->r[k].soff[P], T{});
        recv[k].assign(S->r[k].received, T{});
    }
    auto exchange = [&](bool forward) { // the all-to-all: region (p -> q) of p's send = region p of q's recv
        for (int p = 0; p < P; ++p)
            for (int q = 0; q < P; ++q) {
                const int64_t cnt = S->r[p].scount[q];
                T *a = send[p].data() + S->r[p].soff[q], *b = recv[q].data() + S->r[q].roff[p];
                if (forward) std::copy(a, a + cnt, b);
                else std::copy(b, b + cnt, a);
            }
    };
    if (dir == 0) {
        for (int k = 0; k < P; ++k) slu::ga_pack<T>(S->r[k], (T *)oL[k], (T *)oU[k], send[k].data(), 0);
        exchange(true);
        for (int k = 0; k < P; ++k) slu::ga_unpack<T>(S->r[k], recv[k].data(), (T *)mL[k], (T *)mU[k], 0);
    } else {
        for (int k = 0; k < P; ++k) slu::ga_unpack<T>(S->r[k], recv[k].data(), (T *)mL[k], (T *)mU[k], 1);
        exchange(false);
        for (int k = 0; k < P; ++k) slu::ga_pack<T>(S->r[k], (T *)oL[k], (T *)oU[k], send[k].data(), 1);
    }
}



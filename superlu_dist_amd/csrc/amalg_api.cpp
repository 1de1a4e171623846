// C API of the engine-side amalgamation (csrc/amalg.h) for the CPU tests:
// opt-in library only (full.map exports slu_*).
#include <algorithm>
#include <complex>

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
    std::copy(A->Lidx2.begin(), A->Lidx2.end(), Lidx2);
    std::copy(A->Loff2.begin(), A->Loff2.end(), Loff2);
    std::copy(A->Lvoff2.begin(), A->Lvoff2.end(), Lvoff2);
    std::copy(A->Uidx2.begin(), A->Uidx2.end(), Uidx2);
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

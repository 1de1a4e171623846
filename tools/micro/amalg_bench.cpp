// Host timing harness for the 1x1 amalgamation analysis (csrc/amalg.cpp) on
// dumped index arrays (xsup / Lidx / Loff / Uidx / Uoff as raw int64 files,
// e.g. from a Symbolic(reference=True).distribute() of the 100^3 stencil).
// usage: amalg_bench PREFIX [reps]   (reads PREFIX_xsup.bin etc.)
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <string>
#include <vector>

#include "../../superlu_dist_amd/csrc/amalg.h"

static std::vector<int64_t> load(const std::string &f) {
    FILE *fp = fopen(f.c_str(), "rb");
    if (!fp) { perror(f.c_str()); exit(1); }
    fseek(fp, 0, SEEK_END);
    const long sz = ftell(fp);
    fseek(fp, 0, SEEK_SET);
    std::vector<int64_t> v(sz / 8);
    if (fread(v.data(), 8, v.size(), fp) != v.size()) { perror("read"); exit(1); }
    fclose(fp);
    return v;
}

int main(int argc, char **argv) {
    const std::string p = argv[1];
    const int reps = argc > 2 ? atoi(argv[2]) : 2;
    auto xsup = load(p + "_xsup.bin"), Lidx = load(p + "_Lidx.bin"), Loff = load(p + "_Loff.bin"),
         Uidx = load(p + "_Uidx.bin"), Uoff = load(p + "_Uoff.bin");
    const int ns = (int)xsup.size() - 1;
    const int64_t n = xsup[ns];
    std::vector<const int_t *> li(ns, nullptr), ui(ns, nullptr);
    for (int s = 0; s < ns; ++s) {
        if (Loff[s] >= 0) li[s] = Lidx.data() + Loff[s];
        if (Uoff[s] >= 0) ui[s] = Uidx.data() + Uoff[s];
    }
    for (int r = 0; r < reps; ++r) {
        const auto t0 = std::chrono::steady_clock::now();
        slu::Amalg A;
        A.build(n, ns, xsup.data(), li.data(), ui.data(), 0.10, 256);
        const double ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
        printf("build %.1f ms: ns %d -> %d, Lidx2 %zu Uidx2 %zu lrow %zu U columns %zu D %zu\n", ms, ns, A.ns2,
               A.Lidx2.size(), A.Uidx2.size(), A.lrow.size(), A.ucd.size(), A.D.size());
    }
}

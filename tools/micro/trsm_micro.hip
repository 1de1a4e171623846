// Microbenchmark (not product code): k_trsm_reg<double, 0> (the L-panel
// TRSM) and its latency form (PF) on nslab 64-row slabs of a 256-wide panel,
// ld = rows; best of reps launch times, and an empty launch for reference.
// usage: trsm_micro [nslab reps]
// build: hipcc --offload-arch=gfx950 -O3 -std=c++17 -I superlu_dist_amd/csrc -I include
//        -I /opt/conda/include tools/micro/trsm_micro.hip -o tools/micro/trsm_micro
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define SLU_TR_PROBE 1
#include "kernels.h"

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); exit(1); } } while (0)
using namespace slu;

__global__ void k_empty(int *p) {
    if (threadIdx.x == 0 && blockIdx.x == 0 && p) p[0] = 1;
}

int main(int argc, char **argv) {
    const int nslab = argc > 1 ? atoi(argv[1]) : 4, reps = argc > 2 ? atoi(argv[2]) : 20;
    const int w = 256, m = 64 * nslab, ld = m + w;
    // panel: rows 0..w-1 the diagonal block (upper part used), rows w.. the L rows
    std::vector<double> h((size_t)ld * w);
    for (int j = 0; j < w; ++j)
        for (int i = 0; i < ld; ++i) h[i + (size_t)j * ld] = (i == j) ? 2.0 * w : ((i * 7 + j * 13) % 17) / 17.0 - 0.5;
    std::vector<double> dinv((size_t)2 * 8 * 1024, 0.0);
    for (int b = 0; b < 8; ++b)
        for (int i = 0; i < 32; ++i) dinv[(size_t)b * 1024 + i * 32 + i] = 1.0 / (2.0 * w);
    double *dA, *dA0, *dD;
    CK(hipMalloc(&dA, h.size() * 8));
    CK(hipMalloc(&dA0, h.size() * 8));
    CK(hipMalloc(&dD, dinv.size() * 8));
    CK(hipMemcpy(dA0, h.data(), h.size() * 8, hipMemcpyHostToDevice));
    CK(hipMemcpy(dD, dinv.data(), dinv.size() * 8, hipMemcpyHostToDevice));
    std::vector<TrsmItemF<double>> it(nslab);
    for (int s = 0; s < nslab; ++s) {
        it[s] = {};
        it[s].x = dA + w + 64 * s;
        it[s].t = dA;
        it[s].dinv = dD;
        it[s].ldx = ld;
        it[s].ldt = ld;
        it[s].w = w;
        it[s].nrows = 64;
    }
    TrsmItemF<double> *di;
    CK(hipMalloc(&di, nslab * sizeof(it[0])));
    CK(hipMemcpy(di, it.data(), nslab * sizeof(it[0]), hipMemcpyHostToDevice));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    auto timeit = [&](auto launch) {
        float best = 1e30f;
        for (int r = 0; r < reps; ++r) {
            CK(hipMemcpy(dA, dA0, h.size() * 8, hipMemcpyDeviceToDevice));
            CK(hipDeviceSynchronize());
            CK(hipEventRecord(e0));
            launch();
            CK(hipEventRecord(e1));
            CK(hipEventSynchronize(e1));
            float ms;
            CK(hipEventElapsedTime(&ms, e0, e1));
            best = std::min(best, ms);
        }
        CK(hipGetLastError());
        return best * 1e3f;
    };
    const float te = timeit([&] { hipLaunchKernelGGL(k_empty, dim3(nslab), dim3(256), 0, 0, nullptr); });
    long long zz[8] = {};
    CK(hipMemcpyToSymbol(HIP_SYMBOL(slu_tr_tp), zz, sizeof(zz)));
    const float tr = timeit([&] {
        hipLaunchKernelGGL((k_trsm_reg<double, 0>), dim3(nslab), dim3(64 * TR_WAVES), 0, 0, di);
    });
    long long tp[8];
    CK(hipMemcpyFromSymbol(tp, HIP_SYMBOL(slu_tr_tp), sizeof(tp)));
    const double nwg = (double)reps * nslab;
    printf("  k_trsm_reg phases (cycles per workgroup, mean): X load %.0f  staging %.0f  acc MFMAs %.0f  Z Dinv %.0f  store %.0f\n",
           tp[0] / nwg, tp[1] / nwg, tp[2] / nwg, tp[3] / nwg, tp[4] / nwg);
    std::vector<double> r1(h.size()), r2(h.size());
    CK(hipMemcpy(r1.data(), dA, h.size() * 8, hipMemcpyDeviceToHost));
    CK(hipMemcpyToSymbol(HIP_SYMBOL(slu_tr_tp), zz, sizeof(zz)));
    const float tl = timeit([&] {
        hipLaunchKernelGGL((k_trsm_reg<double, 0, FAST_MAXW, true>), dim3(nslab), dim3(64 * TR_WAVES), 0, 0, di);
    });
    CK(hipMemcpyFromSymbol(tp, HIP_SYMBOL(slu_tr_tp), sizeof(tp)));
    printf("  k_trsm_reg PF phases (cycles per workgroup, mean): X load %.0f  staging %.0f  acc MFMAs %.0f  Z Dinv %.0f  store %.0f\n",
           tp[0] / nwg, tp[1] / nwg, tp[2] / nwg, tp[3] / nwg, tp[4] / nwg);
    CK(hipMemcpy(r2.data(), dA, h.size() * 8, hipMemcpyDeviceToHost));
    double d = 0;
    for (size_t i = 0; i < h.size(); ++i) d = std::max(d, std::abs(r1[i] - r2[i]));
    const double fl = 64.0 * nslab * w * (w + 1.0);
    printf("slabs %4d  empty %6.1f us  k_trsm_reg %7.1f us (%.2f TF/s)  k_trsm_reg PF %7.1f us (%.2f TF/s)  max diff %.1e\n",
           nslab, te, tr, fl / tr * 1e-6, tl, fl / tl * 1e-6, d);
    return 0;
}

// Diagonal-block LU microbenchmark (not product code): k_diag_lu_f on nb
// blocks of w x w (ld = w), phase split by clock64 probes (kernels.h built
// with SLU_DIAG_PROBE), LU residual.
// usage: diag_micro [w nb]   build: hipcc --offload-arch=gfx950 -O3 -std=c++17
//   -I superlu_dist_amd/csrc -I include -I /opt/conda/include tools/micro/diag_micro.hip
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define SLU_DIAG_PROBE 1
#include "kernels.h"

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); exit(1); } } while (0)
using namespace slu;

template <typename K>
float timeit(K launch, double *dA, const double *dA0, size_t bytes, int reps) {
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    float best = 1e30f;
    for (int r = 0; r < reps; ++r) {
        CK(hipMemcpy(dA, dA0, bytes, hipMemcpyDeviceToDevice));
        CK(hipEventRecord(e0));
        launch();
        CK(hipEventRecord(e1));
        CK(hipEventSynchronize(e1));
        float ms;
        CK(hipEventElapsedTime(&ms, e0, e1));
        if (r) best = std::min(best, ms);
    }
    CK(hipGetLastError());
    return best * 1e3f;
}

int main(int argc, char **argv) {
    const int w = argc > 1 ? atoi(argv[1]) : 256, nb = argc > 2 ? atoi(argv[2]) : 1;
    const size_t bytes = (size_t)w * w * nb * 8;
    std::vector<double> h((size_t)w * w * nb);
    for (int b = 0; b < nb; ++b)
        for (int j = 0; j < w; ++j)
            for (int i = 0; i < w; ++i)
                h[(size_t)b * w * w + i + (size_t)j * w] =
                    (i == j) ? 2.0 * w : ((i * 7 + j * 13 + b) % 17) / 17.0 - 0.5;
    double *dA, *dA0, *dinv;
    CK(hipMalloc(&dA, bytes));
    CK(hipMalloc(&dA0, bytes));
    CK(hipMemcpy(dA0, h.data(), bytes, hipMemcpyHostToDevice));
    const int nbk = (w + 31) / 32;
    const size_t dl = (size_t)2 * nbk * 1024;
    CK(hipMalloc(&dinv, nb * dl * 8));
    std::vector<DiagItemF<double>> items(nb);
    for (int b = 0; b < nb; ++b) {
        items[b].a = dA + (size_t)b * w * w;
        items[b].dinv = dinv + (size_t)b * dl;
        items[b].ld = w;
        items[b].w = w;
        items[b].k = b;
        items[b].fcol = 0;
    }
    DiagItemF<double> *di;
    CK(hipMalloc(&di, nb * sizeof(DiagItemF<double>)));
    CK(hipMemcpy(di, items.data(), nb * sizeof(DiagItemF<double>), hipMemcpyHostToDevice));
    int *cnt, *zp;
    CK(hipMalloc(&cnt, 16));
    CK(hipMalloc(&zp, nb * 4));
    CK(hipMemset(zp, 0, nb * 4));
    auto fst = [&] { hipLaunchKernelGGL(k_diag_lu_f<double>, dim3(nb), dim3(DF_THREADS), 0, 0, di, 0.0, 0, cnt, zp); };
    std::vector<double> f2(h.size());
    const float t2 = timeit(fst, dA, dA0, bytes, 4);
    CK(hipMemcpy(f2.data(), dA, bytes, hipMemcpyDeviceToHost));
    double err = 0, nrm = 0; // sampled residual of block 0: L U - A
    for (int j = 0; j < w; j += 3)
        for (int i = 0; i < w; i += 5) {
            double s = 0;
            for (int k = 0; k <= std::min(i, j); ++k) s += (k == i ? 1.0 : f2[i + (size_t)k * w]) * f2[k + (size_t)j * w];
            err = std::max(err, fabs(s - h[i + (size_t)j * w]));
            nrm = std::max(nrm, fabs(h[i + (size_t)j * w]));
        }
    {
        long long z[8] = {0};
        CK(hipMemcpyToSymbol(HIP_SYMBOL(slu_diag_tp), z, sizeof z));
        CK(hipMemcpy(dA, dA0, bytes, hipMemcpyDeviceToDevice));
        fst();
        CK(hipDeviceSynchronize());
        long long h_tp[8];
        CK(hipMemcpyFromSymbol(h_tp, HIP_SYMBOL(slu_diag_tp), sizeof h_tp));
        printf("  phases (cycles per block, all panels): staging %lld  A11 LU %lld  inverses %lld  "
               "L21/U12 %lld  writeback+trailing %lld\n", h_tp[0] / nb, h_tp[1] / nb, h_tp[2] / nb,
               h_tp[3] / nb, h_tp[4] / nb);
    }
    printf("w=%3d blocks=%5d  k_diag_lu_f %8.1f us  LU resid %.2e\n", w, nb, t2, err / nrm);
    return 0;
}

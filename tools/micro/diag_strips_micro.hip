// Microbenchmark (not product code): k_diag_strips (multi-workgroup, one
// 32-column strip per workgroup) against k_diag_lu_f (one workgroup per
// block) on nb blocks of w x w, ld = w + pad.  Prints both times, the LU
// residual of each and the largest difference between their factors and
// dinv blocks.
// usage: diag_strips_micro [w nb reps]
// build: hipcc --offload-arch=gfx950 -O3 -std=c++17 -I superlu_dist_amd/csrc -I include
//        -I /opt/conda/include tools/micro/diag_strips_micro.hip -o tools/micro/diag_strips_micro
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define SLU_DS_PROBE 1
#include "diag_strips.h"

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); exit(1); } } while (0)
using namespace slu;

template <typename T> double resid(const std::vector<T> &f, const std::vector<T> &h, int w, int ld) {
    double err = 0, nrm = 0;
    for (int j = 0; j < w; j += 3)
        for (int i = 0; i < w; i += 5) {
            double s = 0;
            for (int k = 0; k <= std::min(i, j); ++k)
                s += (k == i ? 1.0 : (double)f[i + (size_t)k * ld]) * (double)f[k + (size_t)j * ld];
            err = std::max(err, fabs(s - (double)h[i + (size_t)j * ld]));
            nrm = std::max(nrm, fabs((double)h[i + (size_t)j * ld]));
        }
    return err / nrm;
}

template <typename T> int run(int w, int nb, int reps) {
    const int ld = w + 7;
    const size_t per = (size_t)ld * w, bytes = per * nb * sizeof(T);
    std::vector<T> h(per * nb, T(0));
    for (int b = 0; b < nb; ++b)
        for (int j = 0; j < w; ++j)
            for (int i = 0; i < w; ++i)
                h[(size_t)b * per + i + (size_t)j * ld] =
                    (i == j) ? T(2.0 * w) : T(((i * 7 + j * 13 + b) % 17) / 17.0 - 0.5);
    T *dA, *dA0, *dinv;
    CK(hipMalloc(&dA, bytes));
    CK(hipMalloc(&dA0, bytes));
    CK(hipMemcpy(dA0, h.data(), bytes, hipMemcpyHostToDevice));
    const int nbk = (w + 31) / 32;
    const size_t dl = (size_t)2 * nbk * 1024;
    CK(hipMalloc(&dinv, nb * dl * sizeof(T) * 2));
    T *dinv2 = dinv + nb * dl;
    std::vector<DiagItemF<T>> items(nb), items2(nb);
    for (int b = 0; b < nb; ++b) {
        items[b] = {dA + (size_t)b * per, dinv + (size_t)b * dl, ld, w, b, 0};
        items2[b] = {dA + (size_t)b * per, dinv2 + (size_t)b * dl, ld, w, b, 0};
    }
    DiagItemF<T> *di, *di2;
    CK(hipMalloc(&di, nb * sizeof(DiagItemF<T>)));
    CK(hipMalloc(&di2, nb * sizeof(DiagItemF<T>)));
    CK(hipMemcpy(di, items.data(), nb * sizeof(DiagItemF<T>), hipMemcpyHostToDevice));
    CK(hipMemcpy(di2, items2.data(), nb * sizeof(DiagItemF<T>), hipMemcpyHostToDevice));
    int *cnt, *zp, *err;
    unsigned *flags;
    CK(hipMalloc(&cnt, 16));
    CK(hipMalloc(&zp, nb * 4));
    CK(hipMalloc(&err, 4));
    CK(hipMalloc(&flags, nb * DS_NFLAGS * 4));
    CK(hipMemset(zp, 0, nb * 4));
    CK(hipMemset(err, 0, 4));
    CK(hipMemset(flags, 0, nb * DS_NFLAGS * 4));
    unsigned epoch = 0;
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    auto timeit = [&](auto launch) {
        float best = 1e30f;
        for (int r = 0; r < reps; ++r) {
            CK(hipMemcpy(dA, dA0, bytes, hipMemcpyDeviceToDevice));
            CK(hipDeviceSynchronize());
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
    };
    std::vector<T> f1(h.size()), f2(h.size()), v1(nb * dl), v2(nb * dl);
    const float t1 = timeit([&] {
        if (w <= 64)
            hipLaunchKernelGGL((k_diag_lu_f<T, DF_SMALLW, DF_SMALL_THREADS>), dim3(nb), dim3(DF_SMALL_THREADS), 0, 0, di, 0.0, 0, cnt, zp);
        else
            hipLaunchKernelGGL(k_diag_lu_f<T>, dim3(nb), dim3(DF_THREADS), 0, 0, di, 0.0, 0, cnt, zp);
    });
    CK(hipMemcpy(f1.data(), dA, bytes, hipMemcpyDeviceToHost));
    CK(hipMemcpy(v1.data(), dinv, nb * dl * sizeof(T), hipMemcpyDeviceToHost));
    const float t2 = timeit([&] {
        ++epoch;
        hipLaunchKernelGGL(k_diag_strips<T>, dim3(ds_grid(nb)), dim3(DS_THREADS), 0, 0, di2, nb, flags, epoch,
                           err, 0.0, 0, cnt, zp);
    });
    CK(hipMemcpy(f2.data(), dA, bytes, hipMemcpyDeviceToHost));
    CK(hipMemcpy(v2.data(), dinv2, nb * dl * sizeof(T), hipMemcpyDeviceToHost));
    {
        long long z[8] = {0}, tp[8];
        CK(hipMemcpyToSymbol(HIP_SYMBOL(slu_ds_tp), z, sizeof z));
        CK(hipMemcpy(dA, dA0, bytes, hipMemcpyDeviceToDevice));
        ++epoch;
        hipLaunchKernelGGL(k_diag_strips<T>, dim3(ds_grid(nb)), dim3(DS_THREADS), 0, 0, di2, nb, flags, epoch,
                           err, 0.0, 0, cnt, zp);
        CK(hipDeviceSynchronize());
        CK(hipMemcpyFromSymbol(tp, HIP_SYMBOL(slu_ds_tp), sizeof tp));
        const int nsb = (w + 31) / 32;
        printf("  strips phases (cycles per strip, mean): load+wait %lld  panel read %lld  panel update %lld  "
               "own LU %lld  inverses %lld  publish %lld\n", tp[0] / (nb * nsb), tp[1] / (nb * nsb),
               tp[2] / (nb * nsb), tp[3] / (nb * nsb), tp[4] / (nb * nsb), tp[5] / (nb * nsb));
    }
    int herr = 0;
    CK(hipMemcpy(&herr, err, 4, hipMemcpyDeviceToHost));
    double df = 0, dv = 0, mf = 0, mv = 0;
    for (size_t i = 0; i < f1.size(); ++i) {
        df = std::max(df, fabs((double)f1[i] - (double)f2[i]));
        mf = std::max(mf, fabs((double)f1[i]));
    }
    for (size_t i = 0; i < v1.size(); ++i) {
        dv = std::max(dv, fabs((double)v1[i] - (double)v2[i]));
        mv = std::max(mv, fabs((double)v1[i]));
    }
    printf("%s w=%3d blocks=%4d  k_diag_lu_f %8.1f us  k_diag_strips %8.1f us  resid %.1e / %.1e  "
           "factor diff %.1e  dinv diff %.1e  err %d\n",
           sizeof(T) == 8 ? "f64" : "f32", w, nb, t1, t2, resid(f1, h, w, ld), resid(f2, h, w, ld), df / mf,
           dv / mv, herr);
    return herr;
}

int main(int argc, char **argv) {
    const int w = argc > 1 ? atoi(argv[1]) : 256, nb = argc > 2 ? atoi(argv[2]) : 1;
    const int reps = argc > 3 ? atoi(argv[3]) : 5;
    int bad = run<double>(w, nb, reps);
    bad |= run<float>(w, nb, reps);
    return bad;
}

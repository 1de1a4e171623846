// Microbenchmarks for the Schur-update kernel (not part of the product).
//   1. peak: independent v_mfma_f64_16x16x4f64 chains from registers
//   2. k_schur_big on one synthetic dense supernode update: C(m x n) -= A(m x kw) B(kw x n)
//      with an identity destination map (one L block), i.e. GEMM + fused scatter
// usage: schur_micro [m n kw reps]
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

#include <rocblas/rocblas.h>

#include "kernels.h"

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); exit(1); } } while (0)

using namespace slu;

template <int NACC>
__global__ void __launch_bounds__(256) k_peak(double *out, int iters) {
    typedef __attribute__((ext_vector_type(4))) double v4;
    v4 acc[NACC];
    for (int i = 0; i < NACC; ++i) acc[i] = v4{0, 0, 0, 0};
    double a = threadIdx.x * 1e-3, b = blockIdx.x * 1e-3;
    for (int it = 0; it < iters; ++it) {
#pragma unroll
        for (int i = 0; i < NACC; ++i) acc[i] = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, acc[i], 0, 0, 0);
    }
    double s = 0;
    for (int i = 0; i < NACC; ++i) s += acc[i][0] + acc[i][1] + acc[i][2] + acc[i][3];
    if (s == 123.456) out[0] = s;
}
template <int NACC>
void peak(double *dout, int wg, int iters) {
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    hipLaunchKernelGGL(k_peak<NACC>, dim3(wg), dim3(256), 0, 0, dout, iters);
    hipEventRecord(e0);
    hipLaunchKernelGGL(k_peak<NACC>, dim3(wg), dim3(256), 0, 0, dout, iters);
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    float ms;
    hipEventElapsedTime(&ms, e0, e1);
    double fl = (double)wg * 4 * iters * NACC * 2048.0;
    printf("peak f64 mfma 16x16x4: %5d WGs x 4 waves (%.1f waves/SIMD), %2d acc: %7.3f ms %.2f TFLOP/s\n",
           wg, wg * 4.0 / 1024, NACC, ms, fl / ms / 1e9);
}

int main(int argc, char **argv) {
    int m = argc > 1 ? atoi(argv[1]) : 8192, n = argc > 2 ? atoi(argv[2]) : 8192;
    int kw = argc > 3 ? atoi(argv[3]) : 256, reps = argc > 4 ? atoi(argv[4]) : 5;
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    float ms;
    double *dout;
    CK(hipMalloc(&dout, 8));
    if (getenv("PEAK")) {
        for (int wg : {256, 512, 1024, 2048, 4096}) {
            peak<1>(dout, wg, 20000);
            peak<4>(dout, wg, 5000);
            peak<8>(dout, wg, 2500);
            peak<16>(dout, wg, 1250);
        }
    }
    if (getenv("BLAS")) {
        rocblas_handle h;
        rocblas_create_handle(&h);
        for (int sz : {8192, 4096}) {
            for (int kk : {256, 8192}) {
                if (kk > sz) continue;
                double *A, *B, *C;
                CK(hipMalloc(&A, (size_t)sz * kk * 8));
                CK(hipMalloc(&B, (size_t)sz * kk * 8));
                CK(hipMalloc(&C, (size_t)sz * sz * 8));
                CK(hipMemset(A, 0, (size_t)sz * kk * 8));
                CK(hipMemset(B, 0, (size_t)sz * kk * 8));
                double al = -1, be = 1;
                for (int r = 0; r < 3; ++r) {
                    CK(hipEventRecord(e0));
                    rocblas_dgemm(h, rocblas_operation_none, rocblas_operation_none, sz, sz, kk, &al, A, sz, B, kk, &be, C, sz);
                    CK(hipEventRecord(e1));
                    CK(hipEventSynchronize(e1));
                    CK(hipEventElapsedTime(&ms, e0, e1));
                }
                printf("rocblas_dgemm %d x %d x %d: %.3f ms %.2f TFLOP/s\n", sz, sz, kk, ms, 2.0 * sz * sz * kk / ms / 1e9);
                hipFree(A); hipFree(B); hipFree(C);
            }
        }
    }
    // ---- synthetic supernode update
    std::vector<double> hA((size_t)m * kw), hB((size_t)kw * n);
    for (size_t i = 0; i < hA.size(); ++i) hA[i] = (double)((i * 2654435761u) % 1000) / 1000.0;
    for (size_t i = 0; i < hB.size(); ++i) hB[i] = (double)((i * 40503u) % 1000) / 1000.0;
    double *dA, *dB, *dC;
    CK(hipMalloc(&dA, hA.size() * 8));
    CK(hipMalloc(&dB, hB.size() * 8));
    CK(hipMalloc(&dC, (size_t)m * n * 8));
    CK(hipMemcpy(dA, hA.data(), hA.size() * 8, hipMemcpyHostToDevice));
    CK(hipMemcpy(dB, hB.data(), hB.size() * 8, hipMemcpyHostToDevice));
    CK(hipMemset(dC, 0, (size_t)m * n * 8));
    std::vector<int64_t> cvoff(n);
    std::vector<int> ct0(n, 0), cg(n), cb(n, 0), rg(m), ra(m, 0), pair(1, 0), lmap(m);
    for (int c = 0; c < n; ++c) { cvoff[c] = (int64_t)c * kw; cg[c] = c; }
    for (int r = 0; r < m; ++r) { rg[r] = r; lmap[r] = r; }
    auto up = [](const void *h, size_t bytes) { void *d; CK(hipMalloc(&d, bytes)); CK(hipMemcpy(d, h, bytes, hipMemcpyHostToDevice)); return d; };
    KInfo<double> ki{};
    ki.a = dA; ki.lda = m; ki.m = m; ki.n = n; ki.kmin = 0; ki.kw = kw; ki.nub = 1; ki.atomic = getenv("ATOMIC") ? 1 : 0;
    ki.ubase = dB;
    ki.cvoff = (const int64_t *)up(cvoff.data(), n * 8);
    ki.ct0 = (const int *)up(ct0.data(), n * 4);
    ki.cg = (const int *)up(cg.data(), n * 4);
    ki.cb = (const int *)up(cb.data(), n * 4);
    ki.rg = (const int *)up(rg.data(), m * 4);
    ki.ra = (const int *)up(ra.data(), m * 4);
    ki.pair = (const int *)up(pair.data(), 4);
    LBlk L{};
    L.colvoff = 0; L.mapoff = 0; L.ld = m; L.fcol = 0; L.frow = 0;
    DRec rec{0, 0, m, 0}; // the one destination: L block (0,0), identity row map, ld = m
    ki.prec = (const DRec *)up(&rec, sizeof rec);
    auto *dk = (KInfo<double> *)up(&ki, sizeof ki);
    auto *dl = (LBlk *)up(&L, sizeof L);
    auto *dmap = (int *)up(lmap.data(), m * 4);
    int tm = (m + SB_BM - 1) / SB_BM, tn = (n + SB_BN - 1) / SB_BN;
    std::vector<TileItem> tiles0, tiles;
    const int order = getenv("ORDER") ? atoi(getenv("ORDER")) : 0;
    const int G = getenv("GROUP") ? atoi(getenv("GROUP")) : 8;
    if (order == 0 || order == 2) {
        for (int i = 0; i < tm; ++i)
            for (int j = 0; j < tn; ++j) tiles0.push_back(TileItem{0, i, j});
    } else { // groups of G tile rows, column-major inside a group
        for (int i0 = 0; i0 < tm; i0 += G)
            for (int j = 0; j < tn; ++j)
                for (int i = i0; i < std::min(tm, i0 + G); ++i) tiles0.push_back(TileItem{0, i, j});
    }
    if (order == 2 || order == 3) { // XCD x takes the x-th contiguous chunk of the order
        const size_t T = tiles0.size(), ch = (T + 7) / 8;
        tiles.resize(T);
        std::vector<size_t> pos;
        for (size_t j = 0; j < ch; ++j)
            for (size_t x = 0; x < 8; ++x) pos.push_back(x * ch + j);
        size_t p = 0;
        for (size_t q : pos) if (q < T) tiles[p++] = tiles0[q];
    } else tiles = tiles0;
    if (order == 9) // timing only: every tile reads the same A rows / B columns (L2-resident operands)
        for (auto &t : tiles) { t.tm = 0; t.tn = 0; }
    auto *dt = (TileItem *)up(tiles.data(), tiles.size() * sizeof(TileItem));
    double fl = 2.0 * m * n * kw;
    for (int r = 0; r < reps; ++r) {
        CK(hipEventRecord(e0));
        hipLaunchKernelGGL(k_schur_big<double>, dim3(tiles.size()), dim3(BigCfg<double>::THREADS), 0, 0, dt, dk, dC,
                           (double *)nullptr, dl, dmap, (const UBlk *)nullptr, (const int64_t *)nullptr,
                           (const int *)nullptr);
        CK(hipEventRecord(e1));
        CK(hipEventSynchronize(e1));
        CK(hipEventElapsedTime(&ms, e0, e1));
        printf("k_schur_big m=%d n=%d kw=%d tiles=%zu: %.3f ms  %.2f TFLOP/s\n", m, n, kw,
               tiles.size(), ms, fl / ms / 1e9);
    }
    // check one entry of C after reps updates
    std::vector<double> hC(4);
    CK(hipMemcpy(hC.data(), dC + (size_t)5 + (size_t)7 * m, 8, hipMemcpyDeviceToHost));
    double ref = 0;
    for (int k = 0; k < kw; ++k) ref += hA[5 + (size_t)k * m] * hB[(size_t)7 * kw + k];
    printf("check C(5,7) = %.12g expected %.12g\n", hC[0], -ref * reps);
    return 0;
}

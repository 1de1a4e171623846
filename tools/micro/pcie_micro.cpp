// Host<->device copy rates that bound utime[FACT] of the drop-in pdgstrf
// (SRC/pdgssvx.c:1174-1180 times upload + factor + download):
//   pageable hipMemcpy H2D / D2H, hipHostRegister cost, registered H2D / D2H,
//   and staging through a pinned ring with several host threads.
// build: hipcc -O2 -std=c++17 --offload-arch=gfx950 pcie_micro.cpp -o pcie_micro -lpthread
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <thread>
#include <vector>

#define CK(x)                                                                           \
    do {                                                                                \
        hipError_t e_ = (x);                                                            \
        if (e_ != hipSuccess) {                                                         \
            fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_));    \
            exit(1);                                                                    \
        }                                                                               \
    } while (0)

static double now() {
    return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

// pageable host <-> device through a ring of pinned chunks, nthr threads
// doing the host memcpy while the DMA engine moves the previous chunks
static void staged(char *host, char *dev, size_t bytes, bool h2d, int nthr, size_t chunk) {
    const int NB = 4;
    char *pin[NB];
    hipStream_t s;
    hipEvent_t ev[NB];
    CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    for (int i = 0; i < NB; ++i) {
        CK(hipHostMalloc((void **)&pin[i], chunk));
        CK(hipEventCreateWithFlags(&ev[i], hipEventDisableTiming));
    }
    auto pmemcpy = [&](char *d, const char *src, size_t n) {
        std::vector<std::thread> th;
        size_t per = (n + nthr - 1) / nthr;
        for (int t = 0; t < nthr; ++t) {
            size_t a = t * per, b = std::min(n, a + per);
            if (a < b) th.emplace_back([=] { memcpy(d + a, src + a, b - a); });
        }
        for (auto &x : th) x.join();
    };
    size_t nchunks = (bytes + chunk - 1) / chunk;
    if (h2d) {
        for (size_t c = 0; c < nchunks; ++c) {
            int b = c % NB;
            size_t off = c * chunk, n = std::min(chunk, bytes - off);
            if (c >= NB) CK(hipEventSynchronize(ev[b]));
            pmemcpy(pin[b], host + off, n);
            CK(hipMemcpyAsync(dev + off, pin[b], n, hipMemcpyHostToDevice, s));
            CK(hipEventRecord(ev[b], s));
        }
    } else {
        for (size_t c = 0; c < nchunks + NB; ++c) {
            if (c < nchunks) {
                int b = c % NB;
                size_t off = c * chunk, n = std::min(chunk, bytes - off);
                CK(hipMemcpyAsync(pin[b], dev + off, n, hipMemcpyDeviceToHost, s));
                CK(hipEventRecord(ev[b], s));
            }
            if (c >= NB - 1 && c - (NB - 1) < nchunks) {
                size_t d = c - (NB - 1);
                int b = d % NB;
                size_t off = d * chunk, n = std::min(chunk, bytes - off);
                CK(hipEventSynchronize(ev[b]));
                pmemcpy(host + off, pin[b], n);
            }
        }
    }
    CK(hipStreamSynchronize(s));
    for (int i = 0; i < NB; ++i) {
        CK(hipHostFree(pin[i]));
        CK(hipEventDestroy(ev[i]));
    }
    CK(hipStreamDestroy(s));
}

// GPU stores straight into pinned host memory (zero-copy), nwg workgroups
__global__ void k_push(const double *__restrict__ src, double *__restrict__ dst, size_t n) {
    for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n;
         i += (size_t)gridDim.x * blockDim.x)
        __builtin_nontemporal_store(src[i], dst + i);
}

int main(int argc, char **argv) {
    size_t gb = argc > 1 ? atol(argv[1]) : 4;
    size_t bytes = gb << 30;
    char *host = (char *)malloc(bytes);
    memset(host, 1, bytes); // fault the pages in, as a filled LUstruct would be
    char *dev;
    CK(hipMalloc(&dev, bytes));
    CK(hipMemset(dev, 0, bytes));
    CK(hipDeviceSynchronize());
    double t;
    auto rate = [&](double s) { return bytes / s / 1e9; };
    t = now();
    CK(hipMemcpy(dev, host, bytes, hipMemcpyHostToDevice));
    double h2d_page = now() - t;
    t = now();
    CK(hipMemcpy(host, dev, bytes, hipMemcpyDeviceToHost));
    double d2h_page = now() - t;
    for (int nthr : {4, 8, 16}) {
        t = now();
        staged(host, dev, bytes, true, nthr, 64 << 20);
        double a = now() - t;
        t = now();
        staged(host, dev, bytes, false, nthr, 64 << 20);
        double b = now() - t;
        printf("{\"staged_threads\": %d, \"h2d_gbs\": %.1f, \"d2h_gbs\": %.1f}\n", nthr, rate(a), rate(b));
    }
    // many pageable D2H copies (the per-level write-back of the factors)
    for (size_t piece : {(size_t)64 << 10, (size_t)512 << 10, (size_t)4 << 20}) {
        hipStream_t s;
        CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
        t = now();
        for (size_t o = 0; o < bytes; o += piece)
            CK(hipMemcpyAsync(host + o, dev + o, std::min(piece, bytes - o), hipMemcpyDeviceToHost, s));
        CK(hipStreamSynchronize(s));
        double a = now() - t;
        printf("{\"d2h_pageable_pieces_kb\": %zu, \"gbs\": %.1f, \"us_per_copy\": %.1f}\n", piece >> 10,
               rate(a), a / (bytes / piece) * 1e6);
        CK(hipStreamDestroy(s));
    }
    // GPU stores into pinned host memory
    {
        size_t pb = std::min(bytes, (size_t)1 << 30);
        double *pin;
        CK(hipHostMalloc((void **)&pin, pb));
        for (int nwg : {32, 128, 512}) {
            hipLaunchKernelGGL(k_push, dim3(nwg), dim3(256), 0, 0, (const double *)dev, pin, pb / 8);
            CK(hipDeviceSynchronize());
            t = now();
            hipLaunchKernelGGL(k_push, dim3(nwg), dim3(256), 0, 0, (const double *)dev, pin, pb / 8);
            CK(hipDeviceSynchronize());
            double a = now() - t;
            printf("{\"gpu_store_to_pinned_wg\": %d, \"gbs\": %.1f}\n", nwg, pb / a / 1e9);
        }
        // pinned -> pageable host memcpy with threads (the unpack side)
        for (int nthr : {1, 4, 8}) {
            t = now();
            std::vector<std::thread> th;
            size_t per = pb / nthr;
            for (int i = 0; i < nthr; ++i)
                th.emplace_back([=] { memcpy(host + i * per, (char *)pin + i * per, per); });
            for (auto &x : th) x.join();
            double a = now() - t;
            printf("{\"memcpy_pinned_to_pageable_threads\": %d, \"gbs\": %.1f}\n", nthr, pb / a / 1e9);
        }
        CK(hipHostFree(pin));
    }
    t = now();
    CK(hipHostRegister(host, bytes, hipHostRegisterDefault));
    double reg = now() - t;
    t = now();
    CK(hipMemcpy(dev, host, bytes, hipMemcpyHostToDevice));
    double h2d_pin = now() - t;
    t = now();
    CK(hipMemcpy(host, dev, bytes, hipMemcpyDeviceToHost));
    double d2h_pin = now() - t;
    t = now();
    CK(hipHostUnregister(host));
    double unreg = now() - t;
    printf("{\"bytes\": %zu, \"h2d_pageable_gbs\": %.1f, \"d2h_pageable_gbs\": %.1f, "
           "\"register_s\": %.3f, \"register_gbs\": %.1f, \"unregister_s\": %.3f, "
           "\"h2d_registered_gbs\": %.1f, \"d2h_registered_gbs\": %.1f}\n",
           bytes, rate(h2d_page), rate(d2h_page), reg, rate(reg), unreg, rate(h2d_pin), rate(d2h_pin));
    return 0;
}

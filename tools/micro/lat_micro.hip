// Dependent-latency microbenchmark (not product code): one wave runs chains of
// dependent fp64 FMAs, fp64 divisions, LDS round trips and v_readlane ->
// v_fma pairs; cycles per link from clock64.
#include <hip/hip_runtime.h>
#include <cstdio>

__global__ void k_lat(double *out, long long *cyc, double seed) {
    __shared__ double lds[256];
    const int l = threadIdx.x;
    lds[l] = seed + l;
    __syncthreads();
    double x = seed + l * 1e-9, y = 1.0 + 1e-12 * l;
    long long t0 = clock64();
#pragma unroll 1
    for (int i = 0; i < 1024; ++i) x = fma(x, y, 1e-9);
    long long t1 = clock64();
#pragma unroll 1
    for (int i = 0; i < 256; ++i) x = 1.0 / (x + 3.0);
    long long t2 = clock64();
    int idx = l;
#pragma unroll 1
    for (int i = 0; i < 256; ++i) {
        const double v = lds[idx & 255];
        idx = (int)v & 255;
        x += v;
    }
    long long t3 = clock64();
#pragma unroll 1
    for (int i = 0; i < 256; ++i) {
        const long long b = __double_as_longlong(x);
        const int lo = __builtin_amdgcn_readlane((int)b, 0), hi = __builtin_amdgcn_readlane((int)(b >> 32), 0);
        x = fma(__longlong_as_double(((long long)hi << 32) | (unsigned)lo), y, 1e-9);
    }
    long long t4 = clock64();
    out[l] = x + idx;
    if (l == 0) {
        cyc[0] = (t1 - t0) / 1024;
        cyc[1] = (t2 - t1) / 256;
        cyc[2] = (t3 - t2) / 256;
        cyc[3] = (t4 - t3) / 256;
    }
}

int main() {
    double *d;
    long long *c, h[4];
    (void)hipMalloc(&d, 64 * 8);
    (void)hipMalloc(&c, 4 * 8);
    for (int r = 0; r < 2; ++r) {
        hipLaunchKernelGGL(k_lat, dim3(1), dim3(64), 0, 0, d, c, 0.5);
        (void)hipDeviceSynchronize();
    }
    (void)hipMemcpy(h, c, 32, hipMemcpyDeviceToHost);
    printf("cycles per dependent link: fp64 fma %lld, fp64 div %lld, LDS load %lld, readlane+fma %lld\n",
           h[0], h[1], h[2], h[3]);
    return 0;
}

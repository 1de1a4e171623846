// FP64 MFMA issue-rate microbenchmark (not product code): NACC independent
// v_mfma_f64_16x16x4_f64 chains per wave, accumulators pinned in VGPRs by
// inline asm (the builtin version lets the compiler shuffle VGPR<->AGPR
// copies into the loop), WPS waves per SIMD.
#include <hip/hip_runtime.h>
#include <cstdio>
typedef __attribute__((ext_vector_type(4))) double v4d;

template <int NACC>
__global__ void __launch_bounds__(256) k_peak(double *out, int iters) {
    v4d acc[NACC];
#pragma unroll
    for (int i = 0; i < NACC; ++i) acc[i] = v4d{0, 0, 0, 0};
    double a = threadIdx.x * 1e-3, b = blockIdx.x * 1e-3;
    for (int it = 0; it < iters; ++it) {
#pragma unroll
        for (int i = 0; i < NACC; ++i)
            asm volatile("v_mfma_f64_16x16x4_f64 %0, %1, %2, %0" : "+v"(acc[i]) : "v"(a), "v"(b));
    }
    double s = 0;
#pragma unroll
    for (int i = 0; i < NACC; ++i) s += acc[i][0] + acc[i][1] + acc[i][2] + acc[i][3];
    if (s == 123.456) out[0] = s;
}

template <int NACC>
void peak(double *dout, int wg, int iters) {
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    hipLaunchKernelGGL(k_peak<NACC>, dim3(wg), dim3(256), 0, 0, dout, iters);
    (void)hipEventRecord(e0);
    hipLaunchKernelGGL(k_peak<NACC>, dim3(wg), dim3(256), 0, 0, dout, iters);
    (void)hipEventRecord(e1);
    (void)hipEventSynchronize(e1);
    float ms;
    (void)hipEventElapsedTime(&ms, e0, e1);
    double fl = (double)wg * 4 * iters * NACC * 2048.0;
    printf("f64 16x16x4: %5d WGs x 4 waves (%.1f waves/SIMD), %2d chains: %7.3f ms %6.2f TFLOP/s\n",
           wg, wg * 4.0 / 1024, NACC, ms, fl / ms / 1e9);
}

int main() {
    double *d;
    (void)hipMalloc(&d, 8);
    for (int wg : {256, 512, 1024}) {
        peak<1>(d, wg, 8000);
        peak<2>(d, wg, 4000);
        peak<4>(d, wg, 2000);
        peak<8>(d, wg, 1000);
    }
    return 0;
}

// K-loop anatomy experiments for the fp64 Schur tile (not product code): the
// k_schur_big main loop (128x128 tile, 8 waves 4x2, BK=16, double-buffered
// LDS, 1-stage register prefetch) with parts switched off, to see which part
// keeps the MFMA pipe idle.  No epilogue (acc sunk into one store).
//   V=0 full loop   V=1 no LDS operand reads (constant operands)
//   V=2 no barrier  V=3 no global loads (LDS written from registers)
//   V=4 no MFMA (loads + LDS + barrier only)
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <vector>
#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); exit(1); } } while (0)
typedef __attribute__((ext_vector_type(4))) double v4d;
template <typename T> __device__ __forceinline__ T gld(const T *p) { return *(const __attribute__((address_space(1))) T *)p; }

template <int V>
__global__ void __launch_bounds__(512, 2) k_loop(const double *A, const double *B, double *C, int m, int n, int kw) {
    constexpr int BM = 128, BN = 128, BK = 16, NT = 512, WN = 2, FM = 2, FN = 4;
    constexpr int LA = BM + 4, LB = BN + 4, STAGE = BK * (LA + LB);
    __shared__ double smem[2 * STAGE];
    const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6, wr = wid / WN, wc = wid % WN;
    const int tn = n / BN, row0 = (blockIdx.x / tn) * BM, col0 = (blockIdx.x % tn) * BN;
    const int ar = tid & 127, ak = tid >> 7;
    const int bc = tid >> 2, bk = (tid & 3) * 4;
    const double *ap = A + row0 + ar, *bp = B + (size_t)(col0 + bc) * kw;
    double ra[4], rb[4];
    auto gload = [&](int k0) {
        if (V == 3) return;
#pragma unroll
        for (int s = 0; s < 4; ++s) ra[s] = gld(ap + (size_t)(k0 + ak + 4 * s) * m);
#pragma unroll
        for (int s = 0; s < 4; ++s) rb[s] = gld(bp + k0 + bk + s);
    };
    auto lstore = [&](int buf) {
        double *sA = smem + buf * STAGE, *sB = sA + BK * LA;
#pragma unroll
        for (int s = 0; s < 4; ++s) sA[(ak + 4 * s) * LA + ar] = ra[s];
#pragma unroll
        for (int s = 0; s < 4; ++s) sB[(bk + s) * LB + bc] = rb[s];
    };
    for (int s = 0; s < 4; ++s) ra[s] = rb[s] = 1e-3 * (tid + s);
    v4d acc[FM][FN];
    for (int a = 0; a < FM; ++a) for (int b = 0; b < FN; ++b) acc[a][b] = v4d{0, 0, 0, 0};
    const int nst = kw / BK;
    gload(0);
    lstore(0);
    __syncthreads();
    for (int st = 0; st < nst; ++st) {
        const bool more = st + 1 < nst;
        if (more) gload((st + 1) * BK);
        const double *sA = smem + (st & 1) * STAGE, *sB = sA + BK * LA;
        if (V != 4) {
#pragma unroll
            for (int ks = 0; ks < BK; ks += 4) {
                const int kl = ks + (lane >> 4);
                double av[FM], bv[FN];
#pragma unroll
                for (int f = 0; f < FM; ++f)
                    av[f] = V == 1 ? 1e-3 * (f + ks) : sA[kl * LA + wr * 32 + f * 16 + (lane & 15)];
#pragma unroll
                for (int f = 0; f < FN; ++f)
                    bv[f] = V == 1 ? 2e-3 * (f + ks) : sB[kl * LB + wc * 64 + f * 16 + (lane & 15)];
#pragma unroll
                for (int fm = 0; fm < FM; ++fm)
#pragma unroll
                    for (int fn = 0; fn < FN; ++fn)
                        acc[fm][fn] = __builtin_amdgcn_mfma_f64_16x16x4f64(av[fm], bv[fn], acc[fm][fn], 0, 0, 0);
            }
        }
        if (more) lstore((st + 1) & 1);
        if (V != 2) __syncthreads();
    }
    double sum = 0;
    for (int a = 0; a < FM; ++a) for (int b = 0; b < FN; ++b) sum += acc[a][b][0] + acc[a][b][1] + acc[a][b][2] + acc[a][b][3];
    if (V == 4) sum += smem[tid];
    C[(size_t)blockIdx.x * 512 + tid] = sum;
}

template <int V> void run(const char *name, const double *A, const double *B, double *C, int m, int n, int kw) {
    const int nb = (m / 128) * (n / 128);
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
    float best = 1e30f;
    for (int r = 0; r < 4; ++r) {
        CK(hipEventRecord(e0));
        hipLaunchKernelGGL(k_loop<V>, dim3(nb), dim3(512), 0, 0, A, B, C, m, n, kw);
        CK(hipEventRecord(e1)); CK(hipEventSynchronize(e1));
        float ms; CK(hipEventElapsedTime(&ms, e0, e1));
        if (r) best = ms < best ? ms : best;
    }
    printf("%-40s %8.3f ms %7.2f TFLOP/s\n", name, best, 2.0 * m * n * kw / best / 1e9);
}

int main(int argc, char **argv) {
    const int kw = argc > 1 ? atoi(argv[1]) : 256, m = argc > 2 ? atoi(argv[2]) : 8192, n = argc > 3 ? atoi(argv[3]) : 8192;
    std::vector<double> h((size_t)m * kw);
    for (size_t i = 0; i < h.size(); ++i) h[i] = (double)((i * 2654435761u) % 1000) / 1000.0 - 0.5;
    double *A, *B, *C;
    CK(hipMalloc(&A, (size_t)m * kw * 8)); CK(hipMalloc(&B, (size_t)n * kw * 8)); CK(hipMalloc(&C, (size_t)m * n * 8));
    CK(hipMemcpy(A, h.data(), (size_t)m * kw * 8, hipMemcpyHostToDevice));
    CK(hipMemcpy(B, h.data(), (size_t)n * kw * 8, hipMemcpyHostToDevice));
    if (getenv("ONLY0")) { run<0>("full K loop", A, B, C, m, n, kw); return 0; }
    run<0>("full K loop", A, B, C, m, n, kw);
    run<1>("no LDS operand reads", A, B, C, m, n, kw);
    run<2>("no barrier", A, B, C, m, n, kw);
    run<3>("no global loads", A, B, C, m, n, kw);
    run<4>("no MFMA", A, B, C, m, n, kw);
    return 0;
}

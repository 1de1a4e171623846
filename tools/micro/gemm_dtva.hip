// GEMM main-loop experiment (not product code): A straight from global
// memory into the MFMA operand registers ("direct to VGPR"), B through LDS,
// one workgroup of 4 waves per 128x128 tile, each wave 128 rows x 32 columns
// (8 x 2 v_mfma_f64_16x16x4 fragments, accumulators in AGPRs).  Compared
// with rocBLAS dgemm and the product's register-staged loop (gemm_exp.hip)
// on C(m x n) += A(m x kw) B(kw x n), col-major, kw = 256.
//
// A fragments: lane l (i = l & 15, q = l >> 4) of fragment pair (2j, 2j+1)
// loads rows 32j + 2i, 32j + 2i + 1 at k + q as one 16-byte load: fragment
// 2j + h holds row 32j + 2i + h in lane-row i (a row permutation inside each
// 32-row block, undone when C is written).
#include <hip/hip_runtime.h>
#include <rocblas/rocblas.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); exit(1); } } while (0)
typedef __attribute__((ext_vector_type(4))) double v4d;
typedef __attribute__((ext_vector_type(2))) double v2d;

template <typename T> __device__ __forceinline__ T gld(const T *p) {
    return *(const __attribute__((address_space(1))) T *)p;
}

// WAVES waves along N, each 128 x (128 / WAVES); MINW waves per SIMD
template <int WAVES, int MINW, bool SCHED>
__global__ void __launch_bounds__(64 * WAVES, MINW)
k_dtva(const double *A, const double *B, double *C, int m, int n, int kw) {
    constexpr int BM = 128, BN = 128, BK = 16, NT = 64 * WAVES;
    constexpr int WNC = BN / WAVES, FN = WNC / 16, FP = BM / 32; // fragment pairs along M
    constexpr int LB = BN + 4;
    constexpr int BE = BN * BK / NT; // B elements per thread per stage
    static_assert(BE == 4 || BE == 8 || BE == 16, "");
    __shared__ double sB[2][BK * LB];
    const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
    const int i = lane & 15, q = lane >> 4;
    const int tn = n / BN;
    const int row0 = (blockIdx.x / tn) * BM, col0 = (blockIdx.x % tn) * BN;
    // B staging: thread -> column bc, k = bk .. bk + BE - 1
    constexpr int TPC = BK / BE;
    const int bc = tid / TPC, bk = (tid % TPC) * BE;
    const double *bp = B + (size_t)(col0 + bc) * kw + bk;
    const double *ap = A + row0 + 2 * i + (size_t)q * m;
    v2d ra[2][4][FP]; // [buffer][k-step][pair]
    double rb[BE];
    auto aload = [&](int buf, int k0) {
#pragma unroll
        for (int s = 0; s < 4; ++s)
#pragma unroll
            for (int j = 0; j < FP; ++j) ra[buf][s][j] = gld((const v2d *)(ap + (size_t)(k0 + 4 * s) * m + 32 * j));
    };
    auto bload = [&](int k0) {
#pragma unroll
        for (int s = 0; s < BE; s += 2) {
            v2d v = gld((const v2d *)(bp + k0 + s));
            rb[s] = v[0];
            rb[s + 1] = v[1];
        }
    };
    auto bstore = [&](int buf) {
#pragma unroll
        for (int s = 0; s < BE; ++s) sB[buf][(bk + s) * LB + bc] = rb[s];
    };
    v4d acc[2 * FP][FN];
#pragma unroll
    for (int a = 0; a < 2 * FP; ++a)
#pragma unroll
        for (int b = 0; b < FN; ++b) acc[a][b] = v4d{0, 0, 0, 0};
    const int nst = kw / BK;
    aload(0, 0);
    bload(0);
    bstore(0);
    __syncthreads();
    auto stage = [&](int st, int cur) {
        const bool more = st + 1 < nst;
        if (more) {
            aload(cur ^ 1, (st + 1) * BK);
            bload((st + 1) * BK);
        }
        const double *b = sB[st & 1];
#pragma unroll
        for (int s = 0; s < 4; ++s) {
            double bv[FN];
#pragma unroll
            for (int f = 0; f < FN; ++f) bv[f] = b[(4 * s + q) * LB + wid * WNC + f * 16 + i];
#pragma unroll
            for (int j = 0; j < FP; ++j)
#pragma unroll
                for (int f = 0; f < FN; ++f) {
                    acc[2 * j][f] = __builtin_amdgcn_mfma_f64_16x16x4f64(ra[cur][s][j][0], bv[f], acc[2 * j][f], 0, 0, 0);
                    acc[2 * j + 1][f] =
                        __builtin_amdgcn_mfma_f64_16x16x4f64(ra[cur][s][j][1], bv[f], acc[2 * j + 1][f], 0, 0, 0);
                }
            if (SCHED) {
                // interleave: per k-step 2*FP*FN MFMAs, FN LDS reads, the loads
                __builtin_amdgcn_sched_group_barrier(0x008, 2, 0); // MFMA
                __builtin_amdgcn_sched_group_barrier(0x100, 1, 0); // DS read
                __builtin_amdgcn_sched_group_barrier(0x008, 2, 0);
                __builtin_amdgcn_sched_group_barrier(0x020, 2, 0); // VMEM read
            }
        }
        if (more) bstore((st + 1) & 1);
        __syncthreads();
    };
    for (int st = 0; st < nst; st += 2) {
        stage(st, 0);
        if (st + 1 < nst) stage(st + 1, 1);
    }
#pragma unroll
    for (int f2 = 0; f2 < 2 * FP; ++f2)
#pragma unroll
        for (int f = 0; f < FN; ++f)
#pragma unroll
            for (int e = 0; e < 4; ++e) {
                const int lr = q + 4 * e; // lane-row of the accumulator element
                const int r = row0 + 32 * (f2 >> 1) + 2 * lr + (f2 & 1);
                const int c = col0 + wid * WNC + f * 16 + i;
                C[r + (size_t)c * m] += acc[f2][f][e];
            }
}

template <int WAVES, int MINW, bool SCHED>
void run(const char *name, const double *A, const double *B, double *C, int m, int n, int kw, const double *Cref,
         double *Chost) {
    int nb = (m / 128) * (n / 128);
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    float best = 1e30f;
    for (int r = 0; r < 5; ++r) {
        if (r == 0) CK(hipMemset(C, 0, (size_t)m * n * 8));
        hipEventRecord(e0);
        hipLaunchKernelGGL((k_dtva<WAVES, MINW, SCHED>), dim3(nb), dim3(64 * WAVES), 0, 0, A, B, C, m, n, kw);
        hipEventRecord(e1);
        hipEventSynchronize(e1);
        float ms;
        hipEventElapsedTime(&ms, e0, e1);
        if (r == 0) { // check the first run against rocBLAS
            CK(hipMemcpy(Chost, C, (size_t)m * n * 8, hipMemcpyDeviceToHost));
            double err = 0;
            for (size_t x = 0; x < (size_t)m * n; x += 997) err = fmax(err, fabs(Chost[x] - Cref[x]));
            printf("%-44s maxerr %.2e  ", name, err);
        } else {
            best = ms < best ? ms : best;
        }
    }
    CK(hipGetLastError());
    printf("%8.3f ms %7.2f TFLOP/s\n", best, 2.0 * m * n * kw / best / 1e9);
}

int main(int argc, char **argv) {
    int m = argc > 1 ? atoi(argv[1]) : 8192, n = argc > 2 ? atoi(argv[2]) : 8192;
    int kw = argc > 3 ? atoi(argv[3]) : 256;
    std::vector<double> h((size_t)std::max(m, n) * kw);
    for (size_t x = 0; x < h.size(); ++x) h[x] = (double)((x * 2654435761u) % 1000) / 1000.0 - 0.5;
    double *A, *B, *C;
    CK(hipMalloc(&A, (size_t)m * kw * 8));
    CK(hipMalloc(&B, (size_t)n * kw * 8));
    CK(hipMalloc(&C, (size_t)m * n * 8));
    CK(hipMemcpy(A, h.data(), (size_t)m * kw * 8, hipMemcpyHostToDevice));
    CK(hipMemcpy(B, h.data(), (size_t)n * kw * 8, hipMemcpyHostToDevice));
    CK(hipMemset(C, 0, (size_t)m * n * 8));
    rocblas_handle hd;
    rocblas_create_handle(&hd);
    const double one = 1.0, zero = 0.0;
    rocblas_dgemm(hd, rocblas_operation_none, rocblas_operation_none, m, n, kw, &one, A, m, B, kw, &zero, C, m);
    CK(hipDeviceSynchronize());
    std::vector<double> ref((size_t)m * n), hc((size_t)m * n);
    CK(hipMemcpy(ref.data(), C, (size_t)m * n * 8, hipMemcpyDeviceToHost));
    {
        hipEvent_t e0, e1;
        hipEventCreate(&e0);
        hipEventCreate(&e1);
        float best = 1e30f;
        for (int r = 0; r < 5; ++r) {
            hipEventRecord(e0);
            rocblas_dgemm(hd, rocblas_operation_none, rocblas_operation_none, m, n, kw, &one, A, m, B, kw, &one, C, m);
            hipEventRecord(e1);
            hipEventSynchronize(e1);
            float ms;
            hipEventElapsedTime(&ms, e0, e1);
            if (r) best = ms < best ? ms : best;
        }
        printf("%-44s %8.3f ms %7.2f TFLOP/s\n", "rocBLAS dgemm (beta=1)", best, 2.0 * m * n * kw / best / 1e9);
    }
    run<4, 1, false>("dtva 4 waves (128x32/wave)", A, B, C, m, n, kw, ref.data(), hc.data());
    run<4, 1, true>("dtva 4 waves, sched groups", A, B, C, m, n, kw, ref.data(), hc.data());

    run<8, 1, false>("dtva 8 waves (128x16/wave)", A, B, C, m, n, kw, ref.data(), hc.data());

    return 0;
}

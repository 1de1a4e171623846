// fp64 GEMM main loop with LDS-DMA staging (global_load_lds_dwordx4) for the
// Schur kernel (not product code).
//   C(m x n) += A(m x kw, col-major, ld m) * B(kw x n, col-major, ld ldb)
// B is the dense zero-padded U panel ("bigU", SRC/dSchCompUdt-2Ddynamic.c:245-289),
// so neither operand needs a per-element mask and both go global -> LDS by DMA.
//
// Tile 128 x 128, 512 threads = 8 waves as 4 (M) x 2 (N), each wave 32 x 64 =
// 2 x 4 v_mfma_f64_16x16x4 fragments.  A ring of NS stages of BK k each;
// stage st+NS-1 is issued right after the barrier that retires stage st, so
// NS-1 stages are in flight while stage st is multiplied; one raw s_barrier
// per stage, counted vmcnt, never __syncthreads() inside the loop.
//
// LDS images (both lane-linear per DMA instruction, swizzled through the
// source address):
//   A: [BK][128] doubles, one 1 KB row per instruction; row k holds tile row
//      p ^ 16*(k&1) at position p, so the two 16-lane groups of a
//      ds_read_b64 half-wave (k, k+1) hit opposite bank halves.
//   B: [128][BK] doubles (a column's BK k contiguous); 16-byte chunk j of
//      column c holds k-pair j ^ sw(c), conflict-free fragment reads.
#include <hip/hip_runtime.h>
#include <rocblas/rocblas.h>

#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); exit(1); } } while (0)
typedef __attribute__((ext_vector_type(4))) double v4d;

template <int BK> __device__ __forceinline__ int bsw(int c) {
    if constexpr (BK == 8) return (c >> 2) & 3;
    else return (c >> 1) & 7;
}

__device__ __forceinline__ void glds16(const double *g, double *l) {
    __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void *)g,
                                     (__attribute__((address_space(3))) void *)l, 16, 0, 0);
}

template <int N> __device__ __forceinline__ void wait_vm() {
    if constexpr (N == 0) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    else if constexpr (N == 2) asm volatile("s_waitcnt vmcnt(2)" ::: "memory");
    else if constexpr (N == 4) asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
    else if constexpr (N == 6) asm volatile("s_waitcnt vmcnt(6)" ::: "memory");
    else if constexpr (N == 8) asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
    else if constexpr (N == 12) asm volatile("s_waitcnt vmcnt(12)" ::: "memory");
    else static_assert(N < 0, "vmcnt");
}

__device__ __forceinline__ void bar() {
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
}

template <int BK, int NS, int MINW>
__global__ void __launch_bounds__(512, MINW)
k_glds(const double *A, const double *B, double *C, int m, int n, int kw, int ldb) {
    constexpr int BM = 128, BN = 128, STAGE = BK * BM + BN * BK;
    constexpr int G = BK / 4; // DMA instructions per wave per stage (A: BK/8, B: BK/8)
    __shared__ __attribute__((aligned(16))) double smem[NS * STAGE];
    const int tid = threadIdx.x, lane = tid & 63;
    const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int wr = wid >> 1, wc = wid & 1;
    const int tn = n / BN;
    const int row0 = (blockIdx.x / tn) * BM, col0 = (blockIdx.x % tn) * BN;
    const int nst = kw / BK;
    // per-lane source offsets of this wave's DMA pieces (k0 added per stage)
    // A piece i (row ka = wid + 8*i of the stage): tile rows (2*lane) ^ 16*(ka&1)
    // B piece i (columns (wid + 8*i) * 128/BK ...): column c, k-pair j ^ sw(c)
    constexpr int CPI = 128 / BK; // columns per B piece
    constexpr int LPC = BK / 2;   // lanes per column
    const double *asrc[BK / 8];
    const double *bsrc[BK / 8];
#pragma unroll
    for (int i = 0; i < BK / 8; ++i) {
        const int ka = wid + 8 * i;
        asrc[i] = A + (size_t)ka * m + row0 + ((2 * lane) ^ (16 * (ka & 1)));
        const int c = (wid + 8 * i) * CPI + lane / LPC, j = lane % LPC;
        bsrc[i] = B + (size_t)(col0 + c) * ldb + 2 * (j ^ bsw<BK>(c));
    }
    auto issue = [&](int st) {
        double *sA = smem + (st % NS) * STAGE, *sB = sA + BK * BM;
        const int k0 = st * BK;
#pragma unroll
        for (int i = 0; i < BK / 8; ++i) glds16(asrc[i] + (size_t)k0 * m, sA + (wid + 8 * i) * BM);
#pragma unroll
        for (int i = 0; i < BK / 8; ++i) glds16(bsrc[i] + k0, sB + (wid + 8 * i) * CPI * BK);
    };
    v4d acc[2][4];
#pragma unroll
    for (int a = 0; a < 2; ++a)
#pragma unroll
        for (int b = 0; b < 4; ++b) acc[a][b] = v4d{0, 0, 0, 0};
#pragma unroll
    for (int s = 0; s < NS - 1; ++s)
        if (s < nst) issue(s);
    for (int st = 0; st < nst; ++st) {
        const int left = nst - 1 - st; // stages issued after st
        if (left >= NS - 2) wait_vm<G * (NS - 2)>();
        else if (NS > 3 && left == 1) wait_vm<G>();
        else wait_vm<0>();
        bar();
        if (st + NS - 1 < nst) issue(st + NS - 1);
        const double *sA = smem + (st % NS) * STAGE, *sB = sA + BK * BM;
#pragma unroll
        for (int ks = 0; ks < BK; ks += 4) {
            const int kl = ks + (lane >> 4);
            double av[2], bv[4];
#pragma unroll
            for (int f = 0; f < 2; ++f) av[f] = sA[kl * BM + ((wr * 32 + f * 16 + (lane & 15)) ^ (16 * (kl & 1)))];
#pragma unroll
            for (int f = 0; f < 4; ++f) {
                const int c = wc * 64 + f * 16 + (lane & 15);
                bv[f] = sB[c * BK + 2 * ((kl >> 1) ^ bsw<BK>(c)) + (kl & 1)];
            }
#pragma unroll
            for (int fm = 0; fm < 2; ++fm)
#pragma unroll
                for (int fn = 0; fn < 4; ++fn)
                    acc[fm][fn] = __builtin_amdgcn_mfma_f64_16x16x4f64(av[fm], bv[fn], acc[fm][fn], 0, 0, 0);
        }
    }
#pragma unroll
    for (int fm = 0; fm < 2; ++fm)
#pragma unroll
        for (int fn = 0; fn < 4; ++fn)
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                const int r = row0 + wr * 32 + fm * 16 + (lane >> 4) + 4 * i;
                const int c = col0 + wc * 64 + fn * 16 + (lane & 15);
                C[r + (size_t)c * m] += acc[fm][fn][i];
            }
}

template <int BK, int NS, int MINW>
void run(const char *name, const double *A, const double *B, double *C, int m, int n, int kw,
         const std::vector<double> &ref, double *hC) {
    const int nb = (m / 128) * (n / 128);
    CK(hipMemset(C, 0, (size_t)m * n * 8));
    hipLaunchKernelGGL((k_glds<BK, NS, MINW>), dim3(nb), dim3(512), 0, 0, A, B, C, m, n, kw, kw);
    CK(hipDeviceSynchronize());
    CK(hipMemcpy(hC, C, (size_t)m * n * 8, hipMemcpyDeviceToHost));
    double err = 0;
    for (size_t i = 0; i < ref.size(); ++i) err = fmax(err, fabs(hC[i] - ref[i]));
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    float best = 1e30f;
    for (int r = 0; r < 6; ++r) {
        hipEventRecord(e0);
        hipLaunchKernelGGL((k_glds<BK, NS, MINW>), dim3(nb), dim3(512), 0, 0, A, B, C, m, n, kw, kw);
        hipEventRecord(e1);
        hipEventSynchronize(e1);
        float ms;
        hipEventElapsedTime(&ms, e0, e1);
        best = ms < best ? ms : best;
    }
    CK(hipGetLastError());
    printf("%-40s %8.3f ms %7.2f TFLOP/s  maxerr %.2e\n", name, best, 2.0 * m * n * kw / best / 1e9, err);
}

int main(int argc, char **argv) {
    const int m = argc > 1 ? atoi(argv[1]) : 8192, n = argc > 2 ? atoi(argv[2]) : 8192;
    const int kw = argc > 3 ? atoi(argv[3]) : 256;
    std::vector<double> hA((size_t)m * kw), hB((size_t)n * kw);
    for (size_t i = 0; i < hA.size(); ++i) hA[i] = (double)((i * 2654435761u) % 1000) / 1000.0 - 0.5;
    for (size_t i = 0; i < hB.size(); ++i) hB[i] = (double)((i * 40503u + 7) % 997) / 997.0 - 0.5;
    double *A, *B, *C;
    CK(hipMalloc(&A, (size_t)m * kw * 8 + 4096));
    CK(hipMalloc(&B, (size_t)n * kw * 8 + 4096));
    CK(hipMalloc(&C, (size_t)m * n * 8));
    CK(hipMemcpy(A, hA.data(), hA.size() * 8, hipMemcpyHostToDevice));
    CK(hipMemcpy(B, hB.data(), hB.size() * 8, hipMemcpyHostToDevice));
    // reference: rocBLAS dgemm (timed too)
    rocblas_handle h;
    rocblas_create_handle(&h);
    const double one = 1.0, zero = 0.0;
    CK(hipMemset(C, 0, (size_t)m * n * 8));
    rocblas_dgemm(h, rocblas_operation_none, rocblas_operation_none, m, n, kw, &one, A, m, B, kw, &zero, C, m);
    CK(hipDeviceSynchronize());
    std::vector<double> ref((size_t)m * n), hC((size_t)m * n);
    CK(hipMemcpy(ref.data(), C, ref.size() * 8, hipMemcpyDeviceToHost));
    {
        hipEvent_t e0, e1;
        hipEventCreate(&e0);
        hipEventCreate(&e1);
        float best = 1e30f;
        for (int r = 0; r < 6; ++r) {
            hipEventRecord(e0);
            rocblas_dgemm(h, rocblas_operation_none, rocblas_operation_none, m, n, kw, &one, A, m, B, kw, &one, C, m);
            hipEventRecord(e1);
            hipEventSynchronize(e1);
            float ms;
            hipEventElapsedTime(&ms, e0, e1);
            best = ms < best ? ms : best;
        }
        printf("%-40s %8.3f ms %7.2f TFLOP/s\n", "rocBLAS dgemm (beta=1)", best, 2.0 * m * n * kw / best / 1e9);
    }
    run<8, 4, 4>("glds BK8 x4 stages, 2 WG/CU", A, B, C, m, n, kw, ref, hC.data());
    run<8, 3, 4>("glds BK8 x3 stages, 2 WG/CU", A, B, C, m, n, kw, ref, hC.data());
    run<8, 8, 2>("glds BK8 x8 stages, 1 WG/CU", A, B, C, m, n, kw, ref, hC.data());
    run<16, 3, 2>("glds BK16 x3 stages, 1 WG/CU", A, B, C, m, n, kw, ref, hC.data());
    run<16, 4, 2>("glds BK16 x4 stages, 1 WG/CU", A, B, C, m, n, kw, ref, hC.data());
    run<16, 2, 4>("glds BK16 x2 stages, 2 WG/CU", A, B, C, m, n, kw, ref, hC.data());
    return 0;
}

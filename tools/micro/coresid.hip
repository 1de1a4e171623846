// Which workgroups share a CU (not product code): each WG of a 512-thread,
// 66 KB-LDS kernel (2 per CU, like k_schur_big) records its hardware ids.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <map>
#include <vector>
__global__ void __launch_bounds__(512, 2) k_id(unsigned *out, long long *t) {
    __shared__ double pad[8448];
    unsigned hw, xcc;
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_HW_ID)" : "=s"(hw));
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(xcc));
    pad[threadIdx.x] = threadIdx.x;
    __syncthreads();
    long long t0 = wall_clock64();
    while (wall_clock64() - t0 < 20000) {}
    if (threadIdx.x == 0) {
        out[2 * blockIdx.x] = hw;
        out[2 * blockIdx.x + 1] = xcc + (unsigned)pad[5];
        t[blockIdx.x] = t0;
    }
}
int main() {
    const int nb = 1024;
    unsigned *d;
    long long *dt;
    (void)hipMalloc(&d, nb * 8);
    (void)hipMalloc(&dt, nb * 8);
    hipLaunchKernelGGL(k_id, dim3(nb), dim3(512), 0, 0, d, dt);
    (void)hipDeviceSynchronize();
    std::vector<unsigned> h(nb * 2);
    std::vector<long long> ht(nb);
    (void)hipMemcpy(h.data(), d, nb * 8, hipMemcpyDeviceToHost);
    (void)hipMemcpy(ht.data(), dt, nb * 8, hipMemcpyDeviceToHost);
    std::map<unsigned, std::vector<int>> cu;
    for (int b = 0; b < nb; ++b) {
        unsigned hw = h[2 * b], xcc = h[2 * b + 1] - 5;
        unsigned key = ((xcc & 0xf) << 16) | (((hw >> 13) & 0x7) << 8) | (((hw >> 12) & 1) << 4) |
                       ((hw >> 8) & 0xf);
        cu[key].push_back(b);
    }
    printf("%zu distinct CUs\n", cu.size());
    int shown = 0;
    for (auto &kv : cu) {
        if (shown++ < 12) {
            printf("xcc %u se %u sh %u cu %2u:", kv.first >> 16, (kv.first >> 8) & 7,
                   (kv.first >> 4) & 1, kv.first & 15);
            for (int b : kv.second) printf(" %d", b);
            printf("\n");
        }
    }
    return 0;
}

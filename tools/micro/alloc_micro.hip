// Fresh-HBM allocation cost on the box (what the drop-in's first pdgstrf of a
// process pays for its ~34 GB of factor + caller-layout storage): hipMalloc
// of 8.5 GB buffers sequentially, from two threads at once, and beside a
// pageable H2D copy on another thread.  Prints one line per experiment.
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <thread>
#include <vector>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); exit(1); } } while (0)
using clk = std::chrono::steady_clock;
static double ms(clk::time_point a) { return std::chrono::duration<double, std::milli>(clk::now() - a).count(); }

int main() {
    auto t0 = clk::now();
    CK(hipSetDevice(0));
    CK(hipFree(nullptr));
    printf("init %.1f ms\n", ms(t0));
    const size_t GB = 1ull << 30, SZ = 8 * GB + GB / 2;
    void *a = nullptr, *b = nullptr, *c = nullptr, *d = nullptr;
    t0 = clk::now();
    CK(hipMalloc(&a, SZ));
    printf("hipMalloc 8.5 GB #1: %.1f ms\n", ms(t0));
    t0 = clk::now();
    CK(hipMemset(a, 0, 4096));
    CK(hipDeviceSynchronize());
    printf("first memset on it: %.1f ms\n", ms(t0));
    t0 = clk::now();
    CK(hipMalloc(&b, SZ));
    printf("hipMalloc 8.5 GB #2: %.1f ms\n", ms(t0));
    CK(hipFree(a));
    CK(hipFree(b));
    t0 = clk::now();
    CK(hipMalloc(&a, SZ));
    printf("hipMalloc 8.5 GB after free (reuse): %.1f ms\n", ms(t0));
    CK(hipFree(a));
    // two threads at once (fresh sizes so nothing is cached)
    t0 = clk::now();
    std::thread t1([&] { CK(hipSetDevice(0)); auto s = clk::now(); CK(hipMalloc(&c, SZ + GB)); printf("  thread A %.1f ms\n", ms(s)); });
    std::thread t2([&] { CK(hipSetDevice(0)); auto s = clk::now(); CK(hipMalloc(&d, SZ + GB)); printf("  thread B %.1f ms\n", ms(s)); });
    t1.join();
    t2.join();
    printf("two concurrent 9.5 GB hipMallocs: %.1f ms\n", ms(t0));
    // allocation beside an H2D copy
    const size_t H = 2 * GB;
    char *h = (char *)malloc(H);
    memset(h, 1, H);
    void *dst = nullptr, *eb = nullptr;
    CK(hipMalloc(&dst, H));
    CK(hipMemcpy(dst, h, H, hipMemcpyHostToDevice));
    t0 = clk::now();
    CK(hipMemcpy(dst, h, H, hipMemcpyHostToDevice));
    const double alone = ms(t0);
    t0 = clk::now();
    double tc = 0;
    std::thread t3([&] { CK(hipSetDevice(0)); auto s = clk::now(); CK(hipMemcpy(dst, h, H, hipMemcpyHostToDevice)); tc = ms(s); });
    auto s = clk::now();
    CK(hipMalloc(&eb, SZ + 2 * GB));
    const double ta = ms(s);
    t3.join();
    printf("2 GB pageable H2D alone %.1f ms; beside a 10.5 GB hipMalloc: copy %.1f ms, malloc %.1f ms\n", alone, tc, ta);
    // hipExtMallocWithFlags fine-grained? no: coarse default only; hipMallocAsync from the default pool
    void *f = nullptr;
    t0 = clk::now();
    CK(hipMallocAsync(&f, SZ + 3 * GB, 0));
    CK(hipStreamSynchronize(0));
    printf("hipMallocAsync 11.5 GB: %.1f ms\n", ms(t0));
    CK(hipFreeAsync(f, 0));
    CK(hipStreamSynchronize(0));
    t0 = clk::now();
    CK(hipMallocAsync(&f, SZ + 3 * GB, 0));
    CK(hipStreamSynchronize(0));
    printf("hipMallocAsync 11.5 GB again (pool): %.1f ms\n", ms(t0));
    return 0;
}

// First-touch cost of fresh host memory, 4 KB pages vs transparent huge
// pages (aligned_alloc + MADV_HUGEPAGE), from 1 and T threads: what the plan
// build's large tables pay (csrc/common.h big_alloc).  usage: thp_micro [T]
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <sys/mman.h>
#include <thread>
#include <vector>
int main(int argc, char **argv) {
    const int T = argc > 1 ? atoi(argv[1]) : 16;
    const size_t B = size_t(1) << 30;
    for (int th : {1, T})
        for (int mode = 0; mode < 2; ++mode) {
            auto t0 = std::chrono::steady_clock::now();
            char *p;
            if (mode) {
                p = (char *)aligned_alloc(2 << 20, B);
                madvise(p, B, MADV_HUGEPAGE);
            } else
                p = (char *)malloc(B);
            std::vector<std::thread> v;
            for (int t = 0; t < th; ++t)
                v.emplace_back([=] {
                    for (size_t i = B / th * t; i < B / th * (t + 1); i += 4096) p[i] = 1;
                });
            for (auto &x : v) x.join();
            double ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
            char l[256], hp[64] = "?";
            FILE *f = fopen("/proc/meminfo", "r");
            while (fgets(l, 256, f))
                if (!strncmp(l, "AnonHugePages", 13)) sscanf(l + 14, "%63s", hp);
            fclose(f);
            printf("%-5s %2d threads: %7.1f ms per GB first touch (AnonHugePages %s kB)\n", mode ? "thp" : "4k", th, ms, hp);
            free(p);
        }
    char l[256];
    FILE *f = fopen("/sys/kernel/mm/transparent_hugepage/enabled", "r");
    if (f && fgets(l, 256, f)) printf("thp enabled: %s", l);
}

// Exercises csrc/common.h's parallel_for workers (tests/test_pool.py):
// every index once, a nested call, two submitting threads at once, an
// exception rethrown after all workers stopped, and a forked child.
#include <atomic>
#include <cstdio>
#include <sys/wait.h>
#include <thread>
#include <unistd.h>
#include <vector>

#include "common.h"

using slu::parallel_for;

static int check_cover(int n, int chunk) {
    std::vector<std::atomic<int>> hit(n);
    for (auto &h : hit) h = 0;
    parallel_for(n, [&](int i) { hit[i]++; }, chunk);
    for (int i = 0; i < n; ++i)
        if (hit[i] != 1) return 1;
    return 0;
}

int main() {
    int bad = 0;
    for (int rep = 0; rep < 50; ++rep) bad += check_cover(1000 + rep, 1 + rep % 7);
    // nested: the inner call runs while the outer job holds the workers
    std::atomic<long> sum{0};
    parallel_for(64, [&](int i) { parallel_for(100, [&](int j) { sum += i * 100 + j; }, 3); }, 1);
    const long n = 64 * 100;
    bad += sum != n * (n - 1) / 2;
    // two submitters at once
    std::atomic<int> a{0}, b{0};
    std::thread t1([&] { for (int r = 0; r < 20; ++r) parallel_for(5000, [&](int) { a++; }, 16); });
    std::thread t2([&] { for (int r = 0; r < 20; ++r) parallel_for(5000, [&](int) { b++; }, 16); });
    t1.join();
    t2.join();
    bad += a != 100000 || b != 100000;
    // an exception from one index
    bool caught = false;
    try {
        parallel_for(10000, [&](int i) { if (i == 7777) throw slu::Error("boom"); }, 8);
    } catch (const slu::Error &) {
        caught = true;
    }
    bad += !caught;
    bad += check_cover(20000, 5); // the workers are usable after it
    // a forked child has none of the parent's workers: it must still finish
    const pid_t pid = fork();
    if (pid == 0) _exit(check_cover(20000, 5));
    int st = 0;
    waitpid(pid, &st, 0);
    bad += !(WIFEXITED(st) && WEXITSTATUS(st) == 0);
    printf("%s\n", bad ? "FAIL" : "OK");
    return bad ? 1 : 0;
}

// Error plumbing shared by the host files.  No exception leaves the C ABI:
// every extern "C" entry point catches slu::Error and stores the message
// for slu_last_error().
#pragma once
#include <algorithm>
#include <atomic>
#include <cstdarg>
#include <cstdio>
#include <cstdlib>
#include <exception>
#include <memory>
#include <mutex>
#include <stdexcept>
#include <string>
#include <thread>
#include <vector>

namespace slu {

struct Error : std::runtime_error {
    using std::runtime_error::runtime_error;
};

inline std::string fmt(const char *f, ...) {
    char buf[1024];
    va_list ap;
    va_start(ap, f);
    vsnprintf(buf, sizeof buf, f, ap);
    va_end(ap);
    return buf;
}

void set_last_error(const std::string &s);

// Host array without value-initialisation: large plan tables are filled by
// parallel passes, so the first touch (page faults) is spread over threads.
template <typename T> struct RawVec {
    std::unique_ptr<T[]> a;
    size_t n = 0;
    void resize_uninit(size_t cnt) {
        a.reset(cnt ? new T[cnt] : nullptr);
        n = cnt;
    }
    T &operator[](size_t i) { return a[i]; }
    const T &operator[](size_t i) const { return a[i]; }
    size_t size() const { return n; }
    const T *data() const { return a.get(); }
    T *data() { return a.get(); }
    bool empty() const { return n == 0; }
    void clear() { a.reset(); n = 0; }
};


// Host threads for the plan build (SLU_PLAN_THREADS; default the
// OMP_NUM_THREADS share when set, else the cores, at most 16).
inline int plan_threads() {
    static const int t = [] {
        if (const char *e = getenv("SLU_PLAN_THREADS")) return std::max(1, std::min(64, atoi(e)));
        int v = (int)std::thread::hardware_concurrency();
        if (const char *o = getenv("OMP_NUM_THREADS"); o && atoi(o) > 0) v = std::min(v, atoi(o));
        return std::max(1, std::min(16, v));
    }();
    return t;
}

// f(i) for i in [0, n): dynamic chunks over plan_threads() threads; the
// first exception is rethrown after every thread has stopped.
template <typename F> void parallel_for(int n, F &&f, int chunk = 64) {
    const int T = plan_threads();
    if (n <= chunk || T == 1) {
        for (int i = 0; i < n; ++i) f(i);
        return;
    }
    std::atomic<int> next(0);
    std::exception_ptr err;
    std::mutex mu;
    auto work = [&] {
        try {
            for (;;) {
                const int a = next.fetch_add(chunk);
                if (a >= n) break;
                const int b = std::min(n, a + chunk);
                for (int i = a; i < b; ++i) f(i);
            }
        } catch (...) {
            std::lock_guard<std::mutex> lk(mu);
            if (!err) err = std::current_exception();
            next = n;
        }
    };
    std::vector<std::thread> th;
    for (int t = 1; t < std::min(T, (n + chunk - 1) / chunk); ++t) th.emplace_back(work);
    work();
    for (auto &x : th) x.join();
    if (err) std::rethrow_exception(err);
}

} // namespace slu

#define SLU_REQUIRE(cond, ...)                                                 \
    do {                                                                       \
        if (!(cond)) throw ::slu::Error(::slu::fmt(__VA_ARGS__));              \
    } while (0)

#define HIPCHK(x)                                                              \
    do {                                                                       \
        hipError_t e_ = (x);                                                   \
        if (e_ != hipSuccess)                                                  \
            throw ::slu::Error(::slu::fmt("%s failed: %s (%s:%d)", #x,         \
                                          hipGetErrorString(e_), __FILE__,     \
                                          __LINE__));                          \
    } while (0)

#define NCCLCHK(x)                                                             \
    do {                                                                       \
        ncclResult_t r_ = (x);                                                 \
        if (r_ != ncclSuccess)                                                 \
            throw ::slu::Error(::slu::fmt("%s failed: %s (%s:%d)", #x,         \
                                          ncclGetErrorString(r_), __FILE__,    \
                                          __LINE__));                          \
    } while (0)

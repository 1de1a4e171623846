// Error plumbing shared by the host files.  No exception leaves the C ABI:
// every extern "C" entry point catches slu::Error and stores the message
// for slu_last_error().
#pragma once
#include <algorithm>
#include <atomic>
#include <condition_variable>
#include <cstdarg>
#include <cstdio>
#include <cstdlib>
#include <exception>
#include <functional>
#include <memory>
#include <mutex>
#include <stdexcept>
#include <string>
#include <thread>
#include <vector>

#include <sys/mman.h>
#include <unistd.h>
#include <type_traits>

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

// Host memory for large plan tables: 2 MB aligned and advised as
// transparent huge pages, so the first touch costs one fault per 2 MB
// instead of one per 4 KB (the faults were most of the plan build's
// system time); small ones from malloc.
inline void *big_alloc(size_t bytes) {
    constexpr size_t HP = size_t(2) << 20;
    if (bytes < 2 * HP) return malloc(bytes ? bytes : 1);
    const size_t r = (bytes + HP - 1) / HP * HP;
    void *p = aligned_alloc(HP, r);
    if (p) madvise(p, r, MADV_HUGEPAGE);
    return p;
}
struct BigFree {
    void operator()(void *p) const { free(p); }
};

// Host array without value-initialisation: large plan tables are filled by
// parallel passes, so the first touch (page faults) is spread over threads.
template <typename T> struct RawVec {
    static_assert(std::is_trivially_destructible<T>::value, "RawVec holds plain data");
    std::unique_ptr<T[], BigFree> a;
    size_t n = 0;
    void resize_uninit(size_t cnt) {
        a.reset(nullptr);
        if (cnt) {
            a.reset((T *)big_alloc(cnt * sizeof(T)));
            if (!a) throw std::bad_alloc();
        }
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

namespace detail {
// Persistent workers for parallel_for: the plan build calls it a few hundred
// times (twice per elimination level in build_schedule), and fresh threads
// per call cost their creation plus a fresh first touch of every
// thread_local scratch array (n-sized, 4 KB page faults that serialise in
// the kernel).  One job at a time; a second submitter (another host thread,
// or a parallel_for nested in a job) spawns its own threads as before.
inline thread_local bool t_in_pool = false;
struct Pool {
    std::mutex m;
    std::condition_variable cv, dcv;
    int nthreads = 0, want = 0, left = 0;
    uint64_t gen = 0;
    const std::function<void()> *job = nullptr;
    std::atomic<bool> busy{false};
    void ensure(int nw) { // (called by the submitter holding busy)
        for (; nthreads < nw; ++nthreads) {
            const int id = nthreads;
            std::thread([this, id] { run(id); }).detach();
        }
    }
    void run(int id) {
        t_in_pool = true;
        uint64_t seen = 0;
        for (;;) {
            const std::function<void()> *j;
            {
                std::unique_lock<std::mutex> lk(m);
                cv.wait(lk, [&] { return gen != seen; });
                seen = gen;
                if (id >= want) continue;
                j = job;
            }
            (*j)();
            std::lock_guard<std::mutex> lk(m);
            if (--left == 0) dcv.notify_all();
        }
    }
};
inline Pool &pool() {
    // never destroyed: its threads wait until exit.  A forked child has none
    // of its parent's workers: it starts a pool of its own.
    static std::atomic<Pool *> p{nullptr};
    static std::atomic<pid_t> owner{0};
    static std::mutex mk;
    if (owner.load() != getpid()) {
        std::lock_guard<std::mutex> lk(mk);
        if (owner.load() != getpid()) {
            p = new Pool;
            owner = getpid();
        }
    }
    return *p.load();
}
} // namespace detail

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
    const int nw = std::min(T, (n + chunk - 1) / chunk) - 1;
    detail::Pool &P = detail::pool();
    bool idle = false;
    if (!detail::t_in_pool && P.busy.compare_exchange_strong(idle, true)) {
        const std::function<void()> fn = work;
        {
            std::lock_guard<std::mutex> lk(P.m);
            P.ensure(T - 1);
            P.job = &fn;
            P.want = P.left = nw;
            ++P.gen;
        }
        P.cv.notify_all();
        work();
        {
            std::unique_lock<std::mutex> lk(P.m);
            P.dcv.wait(lk, [&] { return P.left == 0; });
            P.job = nullptr;
        }
        P.busy = false;
    } else {
        std::vector<std::thread> th;
        for (int t = 0; t < nw; ++t) th.emplace_back(work);
        work();
        for (auto &x : th) x.join();
    }
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

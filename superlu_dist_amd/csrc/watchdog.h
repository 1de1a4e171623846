// Exchange watchdog of a multi-rank communicator.
//
// Every exchange group the engine issues (Xport::flush: the plan-time
// all-gathers, and per level the diagonal-package and panel sections of
// factor()) is registered here with what it waits for: the phase, the level
// and this rank's pending sections (direction, peer, bytes).  RCCL groups are
// asynchronous: the record carries an event recorded on the transport's
// stream after ncclGroupEnd, and the watchdog thread polls it.  The host
// transports (MPI, gloo) block inside the callback: the record is closed when
// the callback returns.  A record's clock starts when it becomes the oldest
// open one (everything queued before it has completed), so device work
// queued between two exchanges counts against the bound, host queueing does
// not.
//
// When the oldest record stays open longer than SLU_WATCHDOG_S seconds
// (default 120; 0 disables), or RCCL reports an asynchronous error on one of
// the communicators (ncclCommGetAsyncError), the watchdog prints the rank,
// the phase, the level and the pending sections on stderr, aborts the RCCL
// communicators (ncclCommAbort: the peers' kernels see the abort instead of
// waiting forever) and ends the process with exit status 86.  An ordering
// mismatch between ranks -- the reference's look-ahead pipeline assumes the
// same MPI message order on every rank (SRC/pdgstrf.c:1113-1356) -- therefore
// ends a grid run with a diagnosis instead of a silent hang.
#pragma once
#include <hip/hip_runtime.h>
#include <unistd.h>

#include <chrono>
#include <condition_variable>
#include <cstdio>
#include <cstdlib>
#include <deque>
#include <functional>
#include <mutex>
#include <string>
#include <thread>

namespace slu {

struct Watchdog {
    static constexpr int EXIT_CODE = 86;
    using clk = std::chrono::steady_clock;
    struct Rec {
        uint64_t id;
        std::string what;
        hipEvent_t ev; // RCCL group: completes on the device; null: host-synchronous
        bool done;
    };
    double bound_s = 120;
    int device = -1;
    std::string who;                          // "rank r (row, column, layer)"
    std::function<void()> abort_comms;        // ncclCommAbort on every communicator
    std::function<std::string()> async_error; // non-empty: an RCCL communicator failed
    std::mutex mu;
    std::condition_variable cv;
    std::deque<Rec> q;
    clk::time_point head_since = clk::now();
    uint64_t next_id = 1, completed = 0;
    bool stop = false;
    std::thread th;

    // opt-in (default off): the watchdog ends the whole process (exit 86)
    // from a helper thread, so the library never arms it on its own;
    // bench.py and the grid tests set SLU_WATCHDOG_S for their ranks
    static double bound_from_env() {
        const char *e = getenv("SLU_WATCHDOG_S");
        return e ? atof(e) : 0.0;
    }
    bool enabled() const { return bound_s > 0; }

    ~Watchdog() {
        {
            std::lock_guard<std::mutex> lk(mu);
            stop = true;
        }
        cv.notify_all();
        if (th.joinable()) th.join();
        for (auto &r : q)
            if (r.ev) (void)hipEventDestroy(r.ev);
    }

    // a new exchange group: the event (or null for a host-synchronous one)
    uint64_t open(std::string what, hipEvent_t ev) {
        std::lock_guard<std::mutex> lk(mu);
        if (!th.joinable()) th = std::thread([this] { loop(); });
        if (q.empty()) head_since = clk::now();
        q.push_back({next_id, std::move(what), ev, false});
        return next_id++;
    }
    void close(uint64_t id) {
        std::lock_guard<std::mutex> lk(mu);
        for (auto &r : q)
            if (r.id == id) r.done = true;
        cv.notify_all();
    }

    [[noreturn]] void fire(const std::string &why, std::unique_lock<std::mutex> &) {
        fprintf(stderr, "[slu watchdog] %s: %s\n", who.c_str(), why.c_str());
        if (!q.empty()) {
            fprintf(stderr, "[slu watchdog] %s: oldest open exchange (#%llu, %llu completed before it): %s\n",
                    who.c_str(), (unsigned long long)q.front().id, (unsigned long long)completed,
                    q.front().what.c_str());
            if (q.size() > 1)
                fprintf(stderr, "[slu watchdog] %s: %zu more exchanges queued behind it\n", who.c_str(),
                        q.size() - 1);
        }
        fprintf(stderr, "[slu watchdog] %s: aborting the communicators and exiting with status %d\n",
                who.c_str(), EXIT_CODE);
        fflush(stderr);
        if (abort_comms) abort_comms();
        fflush(stderr);
        _exit(EXIT_CODE); // (no exec, no atexit handlers: a peer may be gone)
    }

    void loop() {
        if (device >= 0) (void)hipSetDevice(device);
        std::unique_lock<std::mutex> lk(mu);
        while (!stop) {
            cv.wait_for(lk, std::chrono::milliseconds(50));
            if (stop) break;
            while (!q.empty()) {
                Rec &h = q.front();
                if (h.ev) {
                    const hipError_t e = hipEventQuery(h.ev);
                    if (e == hipErrorNotReady) break;
                    if (e != hipSuccess)
                        fire(std::string("device error while an exchange was in flight: ") + hipGetErrorString(e),
                             lk);
                    (void)hipEventDestroy(h.ev);
                } else if (!h.done) {
                    break;
                }
                q.pop_front();
                ++completed;
                head_since = clk::now();
            }
            if (async_error) {
                const std::string e = async_error();
                if (!e.empty()) fire("RCCL asynchronous error: " + e, lk);
            }
            if (!q.empty()) {
                const double waited = std::chrono::duration<double>(clk::now() - head_since).count();
                if (waited > bound_s) {
                    char b[128];
                    snprintf(b, sizeof b, "an exchange has not completed after %.1f s (SLU_WATCHDOG_S = %g)",
                             waited, bound_s);
                    fire(b, lk);
                }
            }
        }
    }
};

} // namespace slu

// Host <-> HBM copies of the factor storage for the drop-in pdgstrf, whose
// caller times upload + factorization + download as one (utime[FACT],
// SRC/pdgssvx.c:1174-1180).  Measured on MI355X (tools/micro/pcie_micro.cpp,
// profiles/r02_pcie_micro.json): pageable hipMemcpy H2D 17.5 GB/s, pageable
// D2H 52.6 GB/s, hipHostRegister itself only 15.7 GB/s (so registering the
// caller's arrays costs as much as the slow copy), registered copies 56 GB/s.
//
// * H2D: staged through small pinned buffers by several host threads, each
//   with its own buffers and HIP stream: a thread memcpys chunk c into its
//   pinned buffer while the DMA engine moves its previous chunk.
// * D2H: finished blocks pushed by a kernel into pinned slots, scattered
//   into the caller's arrays by host threads (engine.hip, run_d2h).
#pragma once
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstring>
#include <mutex>
#include <thread>
#include <vector>

#include "common.h"

namespace slu {

struct Xfer {
    char *dev;
    char *host;
    size_t bytes;
};

// Coalesces transfers that are adjacent on both sides (sorted by device
// address first).
inline std::vector<Xfer> merge_xfers(std::vector<Xfer> v) {
    std::sort(v.begin(), v.end(), [](const Xfer &a, const Xfer &b) { return a.dev < b.dev; });
    std::vector<Xfer> out;
    for (const Xfer &x : v) {
        if (!x.bytes) continue;
        if (!out.empty() && out.back().dev + out.back().bytes == x.dev &&
            out.back().host + out.back().bytes == x.host)
            out.back().bytes += x.bytes;
        else
            out.push_back(x);
    }
    return out;
}

// Per-process pool of pinned staging buffers (allocated once: hipHostMalloc
// of the ring costs ~10 ms, not worth paying per call).
struct PinnedPool {
    std::mutex mu;
    std::mutex use; // held by one staged copy at a time
    std::vector<char *> bufs;
    size_t chunk = 0;
    std::vector<char *> get(int n, size_t bytes) {
        std::lock_guard<std::mutex> lk(mu);
        if (chunk != bytes) {
            for (char *b : bufs) (void)hipHostFree(b);
            bufs.clear();
            chunk = bytes;
        }
        while ((int)bufs.size() < n) {
            char *b = nullptr;
            HIPCHK(hipHostMalloc((void **)&b, bytes, hipHostMallocDefault));
            bufs.push_back(b);
        }
        return std::vector<char *>(bufs.begin(), bufs.begin() + n);
    }
};
// pool 0: H2D staging ring, pool 1: D2H slots
inline PinnedPool &pinned_pool(int which = 0) {
    static PinnedPool p[2];
    return p[which];
}

// One piece of a D2H "fill": bytes (<= 1 MB) at src (HBM) -> slot offset dst.
struct PushSeg {
    const char *src;
    int64_t dst;
    int bytes;
};

// GPU stores of finished factor blocks straight into a pinned host slot
// (zero-copy over PCIe; 32-128 workgroups saturate the link).  Workgroup w
// copies pieces w, w + G, ...; 8-byte words when the piece allows (d / z
// values always), else 4-byte (s).
__global__ void __launch_bounds__(256) k_push(const PushSeg *segs, int n, char *slot) {
    for (int i = blockIdx.x; i < n; i += gridDim.x) {
        const PushSeg g = segs[i];
        char *dst = slot + g.dst;
        if (((uintptr_t)g.src | (uintptr_t)dst | (uintptr_t)g.bytes) % 8 == 0) {
            const uint64_t *s8 = (const uint64_t *)g.src;
            uint64_t *d8 = (uint64_t *)dst;
            for (int e = threadIdx.x; e < g.bytes / 8; e += 256) __builtin_nontemporal_store(s8[e], d8 + e);
        } else {
            const uint32_t *s4 = (const uint32_t *)g.src;
            uint32_t *d4 = (uint32_t *)dst;
            for (int e = threadIdx.x; e < g.bytes / 4; e += 256) __builtin_nontemporal_store(s4[e], d4 + e);
        }
    }
}

// Host -> device through a pinned ring: nthr threads, 2 buffers each.
inline void staged_h2d(const std::vector<Xfer> &xs, int device, int nthr = 0,
                       size_t chunk = 32u << 20) {
    if (nthr <= 0) { // SLU_H2D_THREADS (default 4)
        const char *e = getenv("SLU_H2D_THREADS");
        nthr = e && atoi(e) > 0 ? std::min(32, atoi(e)) : 4;
    }
    struct Piece {
        const Xfer *x;
        size_t off, len;
    };
    std::vector<Piece> pieces;
    for (const Xfer &x : xs)
        for (size_t o = 0; o < x.bytes; o += chunk)
            pieces.push_back({&x, o, std::min(chunk, x.bytes - o)});
    if (pieces.empty()) return;
    nthr = std::max(1, std::min<int>(nthr, (int)pieces.size()));
    std::lock_guard<std::mutex> in_use(pinned_pool(0).use);
    std::vector<char *> pin = pinned_pool(0).get(2 * nthr, chunk);
    std::vector<std::string> errs(nthr);
    auto work = [&](int t) {
        hipStream_t s = nullptr;
        hipEvent_t ev[2] = {nullptr, nullptr};
        try {
            HIPCHK(hipSetDevice(device));
            HIPCHK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
            for (auto &e : ev) HIPCHK(hipEventCreateWithFlags(&e, hipEventDisableTiming));
            int k = 0;
            for (size_t i = t; i < pieces.size(); i += nthr, ++k) {
                const int b = k & 1;
                char *buf = pin[2 * t + b];
                if (k >= 2) HIPCHK(hipEventSynchronize(ev[b]));
                const Piece &p = pieces[i];
                memcpy(buf, p.x->host + p.off, p.len);
                HIPCHK(hipMemcpyAsync(p.x->dev + p.off, buf, p.len, hipMemcpyHostToDevice, s));
                HIPCHK(hipEventRecord(ev[b], s));
            }
            HIPCHK(hipStreamSynchronize(s));
        } catch (const std::exception &e) {
            errs[t] = e.what();
        }
        for (auto &e : ev)
            if (e) (void)hipEventDestroy(e);
        if (s) (void)hipStreamDestroy(s);
    };
    std::vector<std::thread> th;
    for (int t = 1; t < nthr; ++t) th.emplace_back(work, t);
    work(0);
    for (auto &x : th) x.join();
    for (auto &e : errs)
        if (!e.empty()) throw Error(e);
}

} // namespace slu

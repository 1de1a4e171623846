// MI355X numeric factorization engine: plan construction (host), level-
// synchronous execution of the batched kernels in kernels.h, RCCL panel
// exchange for 2D process grids, and the engine C API of include/slu_mi355x.h.
//
// Algorithm (what replaces the k-loop of SRC/pdgstrf.c:1108-1756):
//   The supernodal dependency DAG (k -> ib for every block L(ib,k), k -> jb
//   for every block U(k,jb)) is levelled once at plan time.  Supernodes of one
//   level are independent, so for each level every rank launches
//     1. k_diag_lu(_blk) on the diagonal blocks of the level it owns
//        (SRC/pdgstrf2.c:213-269),
//     2. (grids) one grouped broadcast of the factored diagonal blocks (+ their
//        inverted 32x32 diagonal sub-blocks) along process rows and columns
//        (SRC/pdgstrf2.c:280-289 sends U(k,k) down the column),
//     3. k_trsm_* on every local L / U panel block of the level
//        (SRC/pdgstrf2.c:302-355, 843-887),
//     4. (grids) one grouped broadcast of the level's L panels along process
//        rows and U panels along process columns (SRC/pdgstrf.c:1020-1729),
//     5. k_schur(_big) over every (L row tile x U column tile) of every
//        supernode of the level, scattering straight into the destination
//        blocks (SRC/dSchCompUdt-2Ddynamic.c, SRC/dscatter.c:110-277).
//   The set of updates and the per-element arithmetic are those of the
//   reference; only the order in which independent updates are applied
//   differs (the reference orders them by its static schedule,
//   SRC/dstatic_schedule.c:39).  Two supernodes of one level that update the
//   same destination block use atomic fp adds for those blocks.
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <algorithm>
#include <array>
#include <chrono>
#include <cstring>
#include <map>
#include <memory>
#include <numeric>
#include <string>
#include <type_traits>
#include <condition_variable>
#include <functional>
#include <thread>
#include <vector>

#include "common.h"
#include "kernels.h"
#include "diag_strips.h"
#include "diag_wave.h"
#include "fill.h"
#include "solve.h"
#include "hostio.h"
#include "amalg.h"
#include "amalg_dev.h"
#include "watchdog.h"
#include "slu_mi355x.h"

using std::vector;

namespace slu {

static thread_local std::string g_last_error;
void set_last_error(const std::string &s) { g_last_error = s; }

template <typename T> struct DevBuf {
    T *p = nullptr;
    size_t n = 0, guard = 0;
    DevBuf() = default;
    DevBuf(const DevBuf &) = delete;
    DevBuf &operator=(const DevBuf &) = delete;
    ~DevBuf() { release(); }
    void release() {
        if (p) (void)hipFree(p - guard);
        p = nullptr;
        n = guard = 0;
    }
    void alloc(size_t cnt) {
        release();
        n = cnt;
        if (cnt) HIPCHK(hipMalloc(&p, cnt * sizeof(T)));
    }
    // cnt elements with g more allocated on either side: a kernel may read
    // (and mask) up to g elements outside [p, p + cnt) without a clamp
    void alloc_guarded(size_t cnt, size_t g) {
        release();
        HIPCHK(hipMalloc(&p, (cnt + 2 * g) * sizeof(T)));
        HIPCHK(hipMemset(p, 0, g * sizeof(T)));
        HIPCHK(hipMemset(p + g + cnt, 0, g * sizeof(T)));
        p += g;
        n = cnt;
        guard = g;
    }
    void swap(DevBuf &o) {
        std::swap(p, o.p);
        std::swap(n, o.n);
        std::swap(guard, o.guard);
    }
    void upload(const vector<T> &v) { upload(v.data(), v.size()); }
    void upload(const RawVec<T> &v) { upload(v.data(), v.size()); }
    void upload(const T *h, size_t cnt) {
        alloc(cnt);
        if (cnt) HIPCHK(hipMemcpy(p, h, cnt * sizeof(T), hipMemcpyHostToDevice));
    }
    size_t bytes() const { return n * sizeof(T); }
};

} // namespace slu

// ------------------------------------------------------------------ comm
// One rank per GPU.  Production transport: RCCL communicators for the whole
// grid, its process rows and its process columns (the reference's
// grid->comm / rscp / cscp, SRC/superlu_grid.c:158-172).  Test transport
// (slu_comm_create_host): host-staged broadcasts through a caller callback,
// for several ranks sharing one GPU where RCCL refuses duplicate devices.
struct slu_comm {
    int nprow = 1, npcol = 1, iam = 0, myrow = 0, mycol = 0, device = 0;
    ncclComm_t world = nullptr, row = nullptr, col = nullptr;
    // 3D grids (SRC/superlu_grid3d.c: Pz layers of a Pr x Pc grid, the
    // reference's grid3d->zscp): world / row / col above are the layer's,
    // zcomm joins the ranks at my (row, column) position of every layer
    int npdep = 1, zlayer = 0;
    ncclComm_t all = nullptr, zcomm = nullptr;
    slu_host_bcast_fn host_fn = nullptr;
    slu_host_p2p_fn host_p2p = nullptr; // point-to-point test transport
    void *host_ctx = nullptr;
    // exchange watchdog (watchdog.h), created with the first exchange
    std::unique_ptr<slu::Watchdog> wd;
    bool wd_init = false;
    slu::Watchdog *watchdog() {
        if (wd_init) return wd.get();
        wd_init = true;
        const double b = slu::Watchdog::bound_from_env();
        if (b <= 0) return nullptr;
        wd.reset(new slu::Watchdog);
        wd->bound_s = b;
        wd->device = device;
        char w[160];
        snprintf(w, sizeof w, "rank %d of a %dx%d%s grid (row %d, column %d%s), %s transport", iam, nprow, npcol,
                 npdep > 1 ? ("x" + std::to_string(npdep)).c_str() : "", myrow, mycol,
                 npdep > 1 ? (", layer " + std::to_string(zlayer)).c_str() : "",
                 world || zcomm ? "RCCL" : host_p2p ? "host point-to-point" : "host broadcast");
        wd->who = w;
        if (world || zcomm) {
            ncclComm_t cs[5] = {row, col, world, zcomm, all};
            wd->abort_comms = [cs] {
                for (ncclComm_t cm : cs)
                    if (cm) ncclCommAbort(cm);
            };
            wd->async_error = [cs]() -> std::string {
                static const char *names[5] = {"row", "column", "layer", "z", "world"};
                for (int i = 0; i < 5; ++i) {
                    ncclResult_t r = ncclSuccess;
                    if (!cs[i] || ncclCommGetAsyncError(cs[i], &r) != ncclSuccess) continue;
                    if (r != ncclSuccess && r != ncclInProgress)
                        return std::string(names[i]) + " communicator: " + ncclGetErrorString(r);
                }
                return "";
            };
        }
        return wd.get();
    }
};

namespace slu {

using i64 = int64_t;

enum { G_WORLD = 0, G_ROW = 1, G_COL = 2, G_Z = 3 };

// Grouped broadcasts of device buffers within the world / a process row /
// a process column.  Ops are queued and issued together by flush() (one
// ncclGroupStart/End); every member of a communicator queues the same ops in
// the same order, which the plan guarantees by construction.
struct Xport {
    slu_comm *c = nullptr;
    hipStream_t s = nullptr;
    struct Op {
        int g, root;
        void *buf; // null on a member that does not need the section
        size_t bytes;
        uint32_t mask; // members (group ranks) that receive it
    };
    vector<Op> ops;
    vector<char> hbuf;
    double sent = 0, recvd = 0; // bytes this rank moved (RCCL sections)
    // what the next flush() is, for the watchdog's diagnostics
    const char *phase = "plan-time exchange";
    int level = -1;
    int gsize(int g) const {
        return g == G_WORLD ? c->nprow * c->npcol : g == G_ROW ? c->npcol : g == G_COL ? c->nprow : c->npdep;
    }
    int grank(int g) const {
        return g == G_WORLD ? c->iam : g == G_ROW ? c->mycol : g == G_COL ? c->myrow : c->zlayer;
    }
    ncclComm_t comm_of(int g) const {
        return g == G_WORLD ? c->world : g == G_ROW ? c->row : g == G_COL ? c->col : c->zcomm;
    }
    void bcast(int g, int root, void *buf, size_t bytes) {
        if (bytes && gsize(g) > 1) ops.push_back({g, root, buf, bytes, ~0u});
    }
    // A section of root's data for the members in mask (the reference sends
    // L(:,k) only to the process columns flagged in ToSendR,
    // SRC/pdgstrf.c:1039-1044, SRC/pddistribute.c:779).  Every member of the
    // group queues the op (buf = null when not in mask), so that the host
    // transport, which can only broadcast, stays in step.
    void section(int g, int root, uint32_t mask, void *buf, size_t bytes) {
        if (bytes && gsize(g) > 1 && (mask & ~(1u << root))) ops.push_back({g, root, buf, bytes, mask});
    }
    // This rank's point-to-point calls for the queued group, in issue order:
    // a section (and a broadcast, mask = all) becomes the root's sends to
    // every other member in the mask, in member order, and each member's
    // receive from the root.  The RCCL branch issues exactly this list as
    // ncclSend / ncclRecv inside one ncclGroupStart / End, and the
    // point-to-point test transport hands exactly this list to its callback
    // (staged through host memory, all posted before any completes), so the
    // send / receive pairing every grid test runs is the one the RCCL node
    // runs (tests/test_grid.py::test_rccl_call_sequence_is_the_tested_one_cpu
    // compares the two lists and checks the pairing across ranks).
    struct P2P {
        int g, peer, send; // group, group rank of the other side, 1 = send
        size_t bytes;
        int op; // index into ops
    };
    vector<P2P> expand() const {
        vector<P2P> q;
        for (size_t i = 0; i < ops.size(); ++i) {
            const Op &o = ops[i];
            const int me = grank(o.g), P = gsize(o.g);
            if (me == o.root) {
                for (int m = 0; m < P; ++m)
                    if (m != me && (o.mask >> m & 1)) q.push_back({o.g, m, 1, o.bytes, (int)i});
            } else if (o.mask >> me & 1) {
                q.push_back({o.g, o.root, 0, o.bytes, (int)i});
            }
        }
        return q;
    }
    int world_of(int g, int m) const {
        return g == G_WORLD ? m : g == G_ROW ? c->myrow * c->npcol + m : g == G_COL ? m * c->npcol + c->mycol : c->iam;
    }
    // SLU_XPORT_TRACE=<dir>: every flush appends this rank's call list to
    // <dir>/xport_<kind>.<world rank> (kind: the list the transport ran, and
    // on the host transports also "rccl", the calls the RCCL branch would
    // issue for the same group, recorded by a dry run of flush_rccl)
    const char *trace_dir = getenv("SLU_XPORT_TRACE");
    long trace_seq = 0;
    void trace(const char *kind, const vector<P2P> &q) const {
        if (!trace_dir) return;
        char fn[1024];
        snprintf(fn, sizeof fn, "%s/xport_%s.%d", trace_dir, kind, c->iam);
        FILE *f = fopen(fn, "a");
        if (!f) return;
        fprintf(f, "F %ld %s %d\n", trace_seq, phase, level);
        for (const P2P &p : q)
            fprintf(f, "%c %d %d %zu\n", p.send ? 'S' : 'R', p.g, world_of(p.g, p.peer), p.bytes);
        fclose(f);
    }
    vector<vector<char>> p2p_bufs;
    bool host_mem = false; // schedule-only plans: buffers are host memory
    void flush_p2p() {
        const vector<P2P> q0 = expand();
        trace("host", q0);
        if (trace_dir) flush_rccl(true);
        vector<slu_host_p2p_op> q;
        if (host_mem) {
            // no staging: the host buffers go to the transport as they are
            for (const P2P &p : q0) {
                const Op &o = ops[p.op];
                SLU_REQUIRE(o.buf, "section of group %d root %d has no buffer", o.g, o.root);
                q.push_back({p.g, p.peer, p.send, 0, o.buf, (int64_t)p.bytes});
                (p.send ? sent : recvd) += (double)p.bytes;
            }
            if (!q.empty())
                SLU_REQUIRE(c->host_p2p(c->host_ctx, (int)q.size(), q.data()) == 0,
                            "host point-to-point group of %zu ops failed", q.size());
            return;
        }
        HIPCHK(hipStreamSynchronize(s));
        // one host staging buffer per op: the root's D2H once, its sends read it
        p2p_bufs.resize(std::max(p2p_bufs.size(), ops.size()));
        vector<char> staged(ops.size(), 0);
        for (const P2P &p : q0) {
            const Op &o = ops[p.op];
            SLU_REQUIRE(o.buf, "section of group %d root %d has no buffer", o.g, o.root);
            vector<char> &hb = p2p_bufs[p.op];
            hb.resize(o.bytes);
            if (p.send && !staged[p.op]) {
                HIPCHK(hipMemcpyAsync(hb.data(), o.buf, o.bytes, hipMemcpyDeviceToHost, s));
                staged[p.op] = 1;
            }
            q.push_back({p.g, p.peer, p.send, 0, hb.data(), (int64_t)p.bytes});
            (p.send ? sent : recvd) += (double)p.bytes;
        }
        HIPCHK(hipStreamSynchronize(s));
        if (!q.empty())
            SLU_REQUIRE(c->host_p2p(c->host_ctx, (int)q.size(), q.data()) == 0,
                        "host point-to-point group of %zu ops failed", q.size());
        for (const P2P &p : q0)
            if (!p.send)
                HIPCHK(hipMemcpyAsync(ops[p.op].buf, p2p_bufs[p.op].data(), p.bytes, hipMemcpyHostToDevice, s));
        HIPCHK(hipStreamSynchronize(s));
    }
    // this rank's part of the queued group, for the watchdog
    std::string describe() const {
        static const char *gn[4] = {"layer", "row", "column", "z"};
        std::string s = phase;
        if (level >= 0) s += " of level " + std::to_string(level);
        int shown = 0, more = 0;
        double sb = 0, rb = 0;
        std::string lst;
        auto add = [&](bool send, int g, int m, size_t bytes) {
            (send ? sb : rb) += (double)bytes;
            if (shown == 12) {
                ++more;
                return;
            }
            char b[160];
            if (g == G_Z)
                snprintf(b, sizeof b, "%s layer %d: %zu bytes", send ? "send to" : "receive from", m, bytes);
            else
                snprintf(b, sizeof b, "%s %s peer %d (rank %d): %zu bytes", send ? "send to" : "receive from",
                         gn[g], m, world_of(g, m), bytes);
            lst += (shown++ ? "; " : "") + std::string(b);
        };
        for (const P2P &p : expand()) add(p.send != 0, p.g, p.peer, p.bytes);
        char b[160];
        snprintf(b, sizeof b, " (%zu ops; this rank sends %.0f and receives %.0f bytes): ", ops.size(), sb, rb);
        s += b + lst;
        if (more) s += "; ... " + std::to_string(more) + " more";
        return s;
    }
    void flush() {
        if (ops.empty()) return;
        ++trace_seq;
        Watchdog *wd = c->watchdog();
        if (c->host_p2p || c->host_fn) {
            // host transports block in the callback: the record is open for its duration
            const uint64_t id = wd ? wd->open(describe(), nullptr) : 0;
            if (c->host_p2p) flush_host_p2p();
            else {
                if (trace_dir) flush_rccl(true);
                flush_host_bcast();
            }
            if (wd) wd->close(id);
            ops.clear();
            return;
        }
        flush_rccl(false);
        if (wd) {
            hipEvent_t e;
            HIPCHK(hipEventCreateWithFlags(&e, hipEventDisableTiming));
            HIPCHK(hipEventRecord(e, s));
            wd->open(describe(), e);
        }
        ops.clear();
    }
    void flush_host_p2p() { flush_p2p(); }
    void flush_host_bcast() {
        {
            HIPCHK(hipStreamSynchronize(s));
            for (auto &o : ops) {
                hbuf.resize(o.bytes);
                const int me = grank(o.g);
                const bool root = me == o.root;
                // copies on the transport's stream and waited for: a pageable
                // hipMemcpy returns once the host buffer is staged, before the
                // DMA has landed, and kernels on a non-blocking stream could
                // read the destination first
                if (root) {
                    HIPCHK(hipMemcpyAsync(hbuf.data(), o.buf, o.bytes, hipMemcpyDeviceToHost, s));
                    HIPCHK(hipStreamSynchronize(s));
                }
                SLU_REQUIRE(c->host_fn(c->host_ctx, o.g, o.root, hbuf.data(), (int64_t)o.bytes) == 0,
                            "host broadcast (group %d, root %d, %zu bytes) failed", o.g, o.root,
                            o.bytes);
                if (!root && (o.mask >> me & 1)) {
                    SLU_REQUIRE(o.buf, "section of group %d root %d has no buffer", o.g, o.root);
                    HIPCHK(hipMemcpyAsync(o.buf, hbuf.data(), o.bytes, hipMemcpyHostToDevice, s));
                    HIPCHK(hipStreamSynchronize(s));
                }
            }
        }
    }
    // Every op as direct sends from the root to each member that needs it
    // (xGMI is point to point: a root's sends to its row / column peers use
    // distinct links; the plan-time all-gathers' broadcasts too, so there is
    // one call sequence, expand()'s, for RCCL and the tested transport).
    // dry: record the calls (SLU_XPORT_TRACE, kind "rccl") instead of
    // issuing them -- the host transports' check of this very code path.
    void flush_rccl(bool dry) {
        const vector<P2P> q = expand();
        if (dry) {
            trace("rccl", q);
            return;
        }
        trace("rccl", q);
        NCCLCHK(ncclGroupStart());
        for (const P2P &p : q) {
            const Op &o = ops[p.op];
            if (p.send) NCCLCHK(ncclSend(o.buf, o.bytes, ncclChar, p.peer, comm_of(o.g), s));
            else NCCLCHK(ncclRecv(o.buf, o.bytes, ncclChar, p.peer, comm_of(o.g), s));
            (p.send ? sent : recvd) += (double)p.bytes;
        }
        NCCLCHK(ncclGroupEnd());
    }
    // plan-time all-to-all of variable-length int64 blobs in the world
    // group: out[q] goes to rank q, the result's [p] came from rank p.  Sizes
    // first (an all-gather), then one section per ordered pair, queued in
    // the same order on every rank.
    vector<vector<i64>> alltoallv(const vector<vector<i64>> &out) {
        const int P = gsize(G_WORLD), me = grank(G_WORLD);
        SLU_REQUIRE((int)out.size() == P && P <= 32, "alltoallv over %d ranks", P);
        vector<vector<i64>> in(P);
        in[me] = out[me];
        if (P == 1) return in;
        vector<i64> mine(P);
        for (int q = 0; q < P; ++q) mine[q] = (i64)out[q].size();
        const vector<vector<i64>> sz = allgatherv(G_WORLD, mine); // sz[p][q]
        for (int p = 0; p < P; ++p)
            if (p != me) in[p].resize(sz[p][me]);
        if (host_mem) {
            for (int p = 0; p < P; ++p)
                for (int q = 0; q < P; ++q) {
                    if (p == q || !sz[p][q]) continue;
                    void *buf = me == p ? (void *)out[q].data() : me == q ? (void *)in[p].data() : nullptr;
                    section(G_WORLD, p, 1u << q, buf, (size_t)sz[p][q] * sizeof(i64));
                }
            flush();
            return in;
        }
        vector<i64> so(P + 1, 0), ro(P + 1, 0);
        for (int q = 0; q < P; ++q) {
            so[q + 1] = so[q] + (q == me ? 0 : sz[me][q]);
            ro[q + 1] = ro[q] + (q == me ? 0 : sz[q][me]);
        }
        DevBuf<i64> ds, dr;
        ds.alloc(std::max<i64>(so[P], 1));
        dr.alloc(std::max<i64>(ro[P], 1));
        for (int q = 0; q < P; ++q)
            if (q != me && sz[me][q])
                HIPCHK(hipMemcpy(ds.p + so[q], out[q].data(), sz[me][q] * sizeof(i64), hipMemcpyHostToDevice));
        for (int p = 0; p < P; ++p)
            for (int q = 0; q < P; ++q) {
                if (p == q || !sz[p][q]) continue;
                void *buf = me == p ? (void *)(ds.p + so[q]) : me == q ? (void *)(dr.p + ro[p]) : nullptr;
                section(G_WORLD, p, 1u << q, buf, (size_t)sz[p][q] * sizeof(i64));
            }
        flush();
        HIPCHK(hipStreamSynchronize(s));
        for (int p = 0; p < P; ++p)
            if (p != me && sz[p][me])
                HIPCHK(hipMemcpy(in[p].data(), dr.p + ro[p], sz[p][me] * sizeof(i64), hipMemcpyDeviceToHost));
        return in;
    }
    // plan-time all-gather of variable-length int64 blobs within group g
    vector<vector<i64>> allgatherv(int g, const vector<i64> &mine) {
        const int P = gsize(g), me = grank(g);
        vector<vector<i64>> out(P);
        if (P == 1) {
            out[0] = mine;
            return out;
        }
        if (host_mem) { // the same broadcasts over host buffers
            vector<i64> sz(P, 0);
            sz[me] = (i64)mine.size();
            for (int r = 0; r < P; ++r) bcast(g, r, &sz[r], sizeof(i64));
            flush();
            for (int r = 0; r < P; ++r) {
                out[r] = r == me ? mine : vector<i64>(sz[r]);
                bcast(g, r, out[r].data(), sz[r] * sizeof(i64));
            }
            flush();
            return out;
        }
        DevBuf<i64> dsz;
        dsz.alloc(P);
        vector<i64> sz(P, 0);
        sz[me] = (i64)mine.size();
        HIPCHK(hipMemcpy(dsz.p, sz.data(), P * sizeof(i64), hipMemcpyHostToDevice));
        for (int r = 0; r < P; ++r) bcast(g, r, dsz.p + r, sizeof(i64));
        flush();
        HIPCHK(hipStreamSynchronize(s));
        HIPCHK(hipMemcpy(sz.data(), dsz.p, P * sizeof(i64), hipMemcpyDeviceToHost));
        vector<i64> off(P + 1, 0);
        for (int r = 0; r < P; ++r) off[r + 1] = off[r] + sz[r];
        DevBuf<i64> d;
        d.alloc(std::max<i64>(off[P], 1));
        if (!mine.empty())
            HIPCHK(hipMemcpy(d.p + off[me], mine.data(), mine.size() * sizeof(i64),
                             hipMemcpyHostToDevice));
        for (int r = 0; r < P; ++r) bcast(g, r, d.p + off[r], sz[r] * sizeof(i64));
        flush();
        HIPCHK(hipStreamSynchronize(s));
        for (int r = 0; r < P; ++r) {
            out[r].resize(sz[r]);
            if (sz[r])
                HIPCHK(hipMemcpy(out[r].data(), d.p + off[r], sz[r] * sizeof(i64),
                                 hipMemcpyDeviceToHost));
        }
        return out;
    }
};

struct LevelRange {
    int diag_off = 0, diag_n = 0;
    int tl_off = 0, tl_n = 0;
    int tu_off = 0, tu_n = 0;
    int k_off = 0, k_n = 0;
    int tile_off = 0, tile_n = 0;
    int big_off = 0, big_n = 0; // 128x128 Schur tiles (first bigc_n: critical)
    int bigc_n = 0, tilec_n = 0; // critical tiles (destinations in the next level's panels)
    int df_off = 0, df_n = 0;   // fast diag items
    int df_maxw = 0;            // widest of them
    int tf_maxw = 0;            // widest supernode of the fast L / U panel TRSM items
    int lf_off = 0, lf_n = 0;   // fast L-panel TRSM items
    int uf_off = 0, uf_n = 0;   // fast U-panel TRSM items
    int dc_off = 0, dc_n = 0;   // diag-package copy items (2D grids)
    int pc_off = 0, pc_n = 0;   // panel-section copy items (2D grids)
    int ds_off = 0, ds_n = 0;   // diag-package broadcasts
    int ps_off = 0, ps_n = 0;   // panel broadcasts
    double schur_flops = 0, big_flops = 0;
    int atomic_tiles = 0; // tiles of supernodes whose destinations collide within the level
    bool big = false;
    // 2D grids: the level's panel exchange in nch chunks (Plan::pchunks).
    // Chunk c = row group c of every L panel and column group c of every U
    // panel; prefix offsets (relative to lf_off, uf_off, pc_off, ps_off and,
    // for the tiles, to the critical / rest parts of big_off / tile_off) of
    // each chunk's TRSM items, pack copies, sections and Schur tiles (a tile
    // waits for the chunks of its rows and of its columns: max of the two)
    static constexpr int NCHM = 4;
    int nch = 1;
    int lf_o[NCHM + 1] = {}, uf_o[NCHM + 1] = {}, pc_o[NCHM + 1] = {}, ps_o[NCHM + 1] = {};
    int bc_o[NCHM + 1] = {}, br_o[NCHM + 1] = {}, sc_o[NCHM + 1] = {}, sr_o[NCHM + 1] = {};
};

// one broadcast of a contiguous section of a device arena
struct Sec {
    int g, root, arena; // arena 0: diag packages, 1: panels
    i64 off, cnt;       // in elements; off < 0: not received here
    uint32_t mask;      // group ranks that receive the section
};

// 3D grids: one chunk (<= ZR_CHUNK values) of a contiguous range of this
// rank's L (arr 0) or U (arr 1) values -- a block column L(:,k) or block row
// U(k,:) of an ancestor supernode -- zeroed, packed into the exchange
// buffer, added from it (ancestor reduction, SRC/pd3dcomm.c:704-730: alpha =
// beta = 1) or copied from it (gather of the factored forests,
// SRC/pd3dcomm.c:733-760: alpha = 0).  HBM-bound copies, lanes over values.
struct ZRange {
    int64_t off, boff;
    int32_t len, arr;
};
enum { ZR_ZERO = 0, ZR_PACK = 1, ZR_ADD = 2, ZR_COPY = 3 };
constexpr int ZR_CHUNK = 1 << 16;

template <typename T>
__global__ void __launch_bounds__(256) k_zranges(const ZRange *r, T *L, T *U, T *buf, int op) {
    const ZRange z = r[blockIdx.x];
    T *v = (z.arr ? U : L) + z.off;
    T *b = buf + z.boff;
    using Sx = S<T>;
    for (int i = threadIdx.x; i < z.len; i += 256) {
        if (op == ZR_ZERO) v[i] = Sx::zero();
        else if (op == ZR_PACK) b[i] = v[i];
        else if (op == ZR_ADD) v[i] = Sx::sub(v[i], Sx::neg(b[i]));
        else v[i] = b[i];
    }
}

struct PlanBase {
    virtual ~PlanBase() = default;
    virtual void upload() = 0;
    virtual void factor(double anorm, int *info, int *tiny) = 0;
    virtual void download() = 0;
    virtual void snapshot() = 0;
    virtual void restore() = 0;
    virtual void sync() = 0;
    virtual void set_timing(int timing, int serial) = 0;
    virtual void solve(void *b, int64_t ldb, int nrhs) = 0;
    virtual void set_a_pattern(int64_t ncol, const int64_t *xa, const int64_t *asub) = 0;
    virtual void fill_a(const void *a, int on_device) = 0;
    virtual void refine(const void *b, void *x, int64_t ld, int nrhs, double *berr, int *steps) = 0;
    virtual void check_exchange(int64_t *nsec, int64_t *nbytes) = 0;
    virtual void gather_layers() { throw Error("gather_layers: not a 3D plan"); }
    virtual void adopt_factors() = 0; // upload host values that are already factors
    slu_plan_stats stats{};
};

// One rank's plan for value type T (double / float / zc) over the host
// LUstruct layout LocalLU / LUS.
//
// 2D grid (SRC/superlu_defs.h:260-270): block (I,J) lives on rank
// (I mod Pr, J mod Pc).  For supernode k, rank (r,c) needs
//   * L(:,k) restricted to process row r   -- held by (r, k mod Pc),
//   * U(k,:) restricted to process column c -- held by (k mod Pr, c),
//   * the factored diagonal block           -- held by (k mod Pr, k mod Pc)
//     when r == k mod Pr (U-panel TRSM) or c == k mod Pc (L-panel TRSM).
// The plan exchanges the index arrays once (row / column all-gathers), levels
// the global dependency DAG identically on every rank, and lays out per-level
// broadcast sections so that a level is: diag LU -> diag-package broadcast ->
// panel TRSMs -> L-panel (row) / U-panel (column) broadcasts -> Schur update.
template <typename T, typename HT, typename LocalLU, typename LUS>
struct Plan : PlanBase {
    using value_type = T;
    using host_type = HT;
    using local_type = LocalLU;
    using lus_type = LUS;
    // ---- problem
    int n = 0, nsupers = 0, Pr = 1, Pc = 1, iam = 0, myrow = 0, mycol = 0;
    slu_comm *comm = nullptr;
    slu_engine_opts opts{};
    LUS *LU = nullptr;
    vector<i64> xsup;
    int nlc = 0, nlr = 0;
    hipStream_t stream = nullptr;  // Schur updates that are off the critical path
    hipStream_t pstream = nullptr; // panels, exchanges, critical Schur tiles
    hipStream_t ustream = nullptr; // the U panels' TRSM beside the L panels' (launch_trsm_fast)
    // 2D grids: the exchanges on a stream of their own, between events from
    // the panel stream (packed sections) and to the panel and Schur streams
    // (received chunks): the next chunk's TRSM runs beside the current
    // chunk's transfer, a chunk's Schur tiles start when it is in
    hipStream_t cstream = nullptr;
    hipEvent_t ev_pk = nullptr, ev_dx = nullptr, ev_cx[LevelRange::NCHM] = {};
    vector<hipEvent_t> ev_pan, ev_rest; // per level
    hipEvent_t ev_start = nullptr, ev_pend = nullptr, ev_tu0 = nullptr, ev_tu1 = nullptr;
    bool xmode = false; // 2D grid with exchanges
    Xport X;

    // ---- local storage layout (destinations)
    vector<i64> lval_off, uval_off; // per local column / row, -1 if empty
    vector<int> lval_ld;            // nsupr per local column
    i64 lval_total = 0, uval_total = 0;
    bool l_contig = false, u_contig = false;
    vector<LBlk> lblk;
    vector<int> lblk_ib;
    vector<int> lcol_first, lcol_nblk; // per local column
    RawVec<int> lmap;
    vector<UBlk> ublk;
    vector<int> ublk_jb;
    vector<int> urow_first, urow_nblk;
    RawVec<i64> ucol_voff;
    RawVec<int> ucol_fst;

    // ---- panels of every supernode as seen from this rank
    vector<const int_t *> lidx; // L(:,k) on my process row (reference index format) or null
    vector<const int_t *> uidx; // U(k,:) on my process column or null
    vector<vector<i64>> xL, xU; // received index blobs (own the remote lidx/uidx)
    vector<i64> lpos, upos;     // remote panel value offsets in d_pan (-1: local / none)
    // Chunked panel exchange (2D grids, SLU_PANEL_CHUNKS, default 4; 1 =
    // one exchange per level): supernode k's L panel rows on my process row
    // in groups of lgsz[k] rows (a multiple of 128, so every Schur tile and
    // TRSM slab lies in one group), its U panel columns on my process column
    // in groups of ucsz[k] columns; lgpos / ugpos: each received group's
    // offset in d_pan (an L group column-major with ld = its rows); ugrun:
    // the U panel's value offset at each group's first column
    static constexpr int NCHM = LevelRange::NCHM;
    int pchunks = 1;
    vector<int> lgsz, ucsz, ucols;
    vector<std::array<i64, NCHM>> lgpos, ugpos, ugrun;
    int ngroups(int len, int gsz) const { return len > 0 ? (len + gsz - 1) / gsz : 0; }
    int group_size(int len) const {
        const int per = (len + pchunks - 1) / std::max(pchunks, 1);
        return std::max(128, (per + 127) / 128 * 128);
    }
    vector<i64> pkg;            // diag package offset in d_dpk (2D grids), -1 none
    vector<i64> dscr;           // 1x1: Dinv offset in the per-level scratch
    i64 dpk_total = 0, pan_total = 0, dscr_max = 0;

    // ---- schedule
    vector<int> level_of;
    vector<vector<int>> bylev;
    vector<LevelRange> levels;

    // ---- 3D grids (pdgstrf3d, SRC/pdgstrf3d.c:121-348).  Pz = 2^(maxlvl-1)
    // layers, each a Pr x Pc grid holding the whole LUstruct; the supernodal
    // etree is cut into 2^maxlvl - 1 forests (heap order: 0 = the top
    // ancestors, 2t+1 / 2t+2 the two halves below forest t).  Layer z factors
    // its leaf forest, then (phase p >= 1, layers with z % 2^p == 0) the
    // forest above, after adding the partner layer's partial updates of every
    // ancestor block (reduction at the end of phase p-1 between z and
    // z + 2^(p-1)); only the layer that factors an ancestor forest starts it
    // from A's values, the others from zero (SRC/pd3dcomm.c:754-771).
    bool zmode = false;
    int npdep = 1, zl = 0, maxlvl = 1, my_last = 0;
    vector<int> forest_of, phase_of; // per supernode; phase -1: not factored here
    vector<int> phase_lv;            // my phase p = levels [phase_lv[p], phase_lv[p+1])
    vector<int> zr_off;              // zero ranges [zr_off[0], zr_off[1]); reduction p: [zr_off[p+1], zr_off[p+2])
    vector<i64> zr_cnt;              // values exchanged by reduction p
    vector<ZRange> zr;
    DevBuf<ZRange> d_zr;
    DevBuf<T> d_zbuf;
    vector<i64> uval_len;
    double zbytes = 0; // reduction bytes sent + received per factorization
    // SLU_3D_SOLO=1 (measurement hook, tools/model3d.py): one layer alone on
    // a GPU -- the reductions pack / add but exchange nothing, so each
    // layer's phase times can be taken without the others running beside it
    bool zsolo = getenv("SLU_3D_SOLO") && atoi(getenv("SLU_3D_SOLO")) == 1;
    vector<DiagItem<T>> diag_items;
    vector<TrsmLItem<T>> tl_items;
    vector<TrsmUItem<T>> tu_items;
    vector<KInfo<T>> kinfos;
    vector<TileItem> tiles, tiles_big;

    vector<DiagItemF<T>> df_items;
    vector<TrsmItemF<T>> lf_items, uf_items;
    vector<CopyItem<T>> dcopy, pcopy;
    vector<Sec> dsecs, psecs;
    // per-k panel arrays (device copies referenced by KInfo / TrsmUItem)
    RawVec<int> h_rg, h_ra, h_cg, h_cb, h_pair, h_ct0;
    RawVec<i64> h_cvoff;

    // ---- device
    DevBuf<T> d_L, d_U, d_dpk, d_pan, d_dinv;
    DevBuf<LBlk> d_lblk;
    DevBuf<int> d_lmap;
    DevBuf<UBlk> d_ublk;
    DevBuf<i64> d_ucol_voff;
    DevBuf<int> d_ucol_fst;
    DevBuf<DiagItem<T>> d_diag;
    DevBuf<TrsmLItem<T>> d_tl;
    DevBuf<TrsmUItem<T>> d_tu;
    DevBuf<KInfo<T>> d_kinfo;
    DevBuf<TileItem> d_tiles, d_tiles_big;
    DevBuf<DiagItemF<T>> d_df;
    DevBuf<TrsmItemF<T>> d_lf, d_uf;
    DevBuf<CopyItem<T>> d_dcopy, d_pcopy;
    DevBuf<int> d_rg, d_ra, d_cg, d_cb, d_pair, d_ct0;
    DevBuf<DRec> d_prec;
    DevBuf<i64> d_cvoff;
    DevBuf<int> d_counters; // [0] tiny pivots, [1] k_diag_strips hand-off timeout
    DevBuf<unsigned> d_dsflags; // k_diag_strips: per fast diag item, DS_NFLAGS strip flags (A, B)
    unsigned ds_epoch = 0;      // ... set to the factorization's epoch when a strip is published
    DevBuf<int> d_zpiv;     // per supernode: max zero-pivot column + 1
    DevBuf<i64> d_info;     // 2D grids: all-gather of the per-rank info

    static constexpr bool cplx = sizeof(T) == 16;
    static constexpr int PW = PWOf<T>::v;

    int W(i64 k) const { return (int)(xsup[k + 1] - xsup[k]); }
    bool fast_w(int w) const { return w <= FAST_MAXW; }
    i64 dinv_len(int w) const { return fast_w(w) ? 2 * (i64)((w + PW - 1) / PW) * PW * PW : 0; }

    // pre (optional): the L / U value storage allocated ahead by the caller
    // (an amalgamated plan allocates it beside its analysis: fresh HBM costs
    // ~28 ms per GB), adopted when its sizes are this layout's
    Plan(LUS *lu, int n_, int nprow, int npcol, int iam_, slu_comm *c,
         const slu_engine_opts *o, DevBuf<T> *pre = nullptr) {
        LU = lu;
        n = n_;
        Pr = nprow;
        Pc = npcol;
        iam = iam_;
        myrow = iam / Pc;
        mycol = iam % Pc;
        comm = c;
        if (o) opts = *o;
        xmode = Pr * Pc > 1;
        if (xmode) {
            const char *e = getenv("SLU_PANEL_CHUNKS");
            pchunks = std::max(1, std::min(NCHM, e ? atoi(e) : 4));
        }
        SLU_REQUIRE(!xmode || (comm && (comm->world || comm->host_fn || comm->host_p2p)),
                    "a %dx%d grid needs a communicator (slu_comm_create)", Pr, Pc);
        zmode = comm && comm->npdep > 1;
        if (zmode) {
            npdep = comm->npdep;
            zl = comm->zlayer;
            while ((1 << (maxlvl - 1)) < npdep) ++maxlvl;
            SLU_REQUIRE(comm->zcomm || comm->host_p2p,
                        "a 3D grid needs RCCL (slu_comm_create3d) or the point-to-point host transport");
            SLU_REQUIRE(!(o && o->overlap_download), "3D grids: no overlapped download (factors are spread over the layers)");
        }
        if (xmode)
            SLU_REQUIRE(comm->nprow == Pr && comm->npcol == Pc && comm->iam == iam,
                        "communicator is for a %dx%d grid rank %d, plan for %dx%d rank %d",
                        comm->nprow, comm->npcol, comm->iam, Pr, Pc, iam);
        dry = opts.schedule_only != 0;
        if (dry)
            SLU_REQUIRE(!xmode || comm->host_p2p,
                        "a schedule-only plan of a grid needs the point-to-point host transport");
        X.c = comm;
        X.host_mem = dry;
        if (dry) {
            // host only (no HIP call): the layout, the index exchange, the
            // levels and the per-level exchange sections, for
            // slu_plan_check_exchange
            int_t *hx = LU->Glu_persist->xsup;
            nsupers = (int)(LU->Glu_persist->supno[n - 1] + 1);
            xsup.assign(hx, hx + nsupers + 1);
            nlc = (nsupers + Pc - 1) / Pc;
            nlr = (nsupers + Pr - 1) / Pr;
            value_layout();
            build_local();
            exchange_index();
            exchange_needs();
            compute_levels();
            layout_values();
            if (zmode) build_zranges(false);
            return;
        }
        if (comm) HIPCHK(hipSetDevice(comm->device));
        // the panel stream carries the critical path (critical Schur tiles,
        // next level's diag LU / TRSM / exchanges): higher priority, so its
        // workgroups are dispatched ahead of the bulk Schur update's
        // (created on a helper thread beside the host-side plan build --
        // the first streams of a process take ~35 ms -- and joined before
        // their first use)
        std::string stream_err;
        std::thread stream_thread([this, &stream_err] {
            try {
                if (comm) HIPCHK(hipSetDevice(comm->device));
                int prio_lo = 0, prio_hi = 0;
                const auto ts0 = std::chrono::steady_clock::now();
                HIPCHK(hipDeviceGetStreamPriorityRange(&prio_lo, &prio_hi));
                HIPCHK(hipStreamCreateWithPriority(&stream, hipStreamNonBlocking, prio_lo));
                HIPCHK(hipStreamCreateWithPriority(&pstream, hipStreamNonBlocking, prio_hi));
                HIPCHK(hipStreamCreateWithPriority(&ustream, hipStreamNonBlocking, prio_hi));
                if (xmode) HIPCHK(hipStreamCreateWithPriority(&cstream, hipStreamNonBlocking, prio_hi));
                if (getenv("SLU_PROFILE_PLAN"))
                    fprintf(stderr, "[slu plan %d] streams               %6.1f ms (helper thread)\n", iam,
                            ms_since(ts0));
            } catch (const std::exception &e) {
                stream_err = e.what();
            }
        });
        struct Joiner { // (an exception before the join must not leave it joinable)
            std::thread &t;
            ~Joiner() {
                if (t.joinable()) t.join();
            }
        } stream_joiner{stream_thread};
        auto join_streams = [&] {
            if (!stream_thread.joinable()) return;
            stream_thread.join();
            SLU_REQUIRE(stream_err.empty(), "%s", stream_err.c_str());
            X.s = pstream;
        };
        int_t *hx = LU->Glu_persist->xsup;
        nsupers = (int)(LU->Glu_persist->supno[n - 1] + 1);
        xsup.assign(hx, hx + nsupers + 1);
        nlc = (nsupers + Pc - 1) / Pc;
        nlr = (nsupers + Pr - 1) / Pr;
        for (int k = 0; k < nsupers; ++k)
            SLU_REQUIRE(W(k) <= 512, "supernode %d has %d columns (> MAX_SUPER_SIZE 512)", k, W(k));
        // k_schur_big reads up to a panel width before a U segment and 127
        // rows past an L column, unclamped, inside the buffers' guards
        static_assert(SB_UGUARD >= 512 + 128, "guards too small for the widest panel");
        const auto t0 = std::chrono::steady_clock::now();
        prof = getenv("SLU_PROFILE_PLAN") != nullptr;
        tprev = t0;
        value_layout();
        if (pre && pre[0].n == (size_t)std::max<i64>(lval_total, 1) && pre[0].guard == SB_UGUARD &&
            pre[1].n == (size_t)std::max<i64>(uval_total, 1) && pre[1].guard == SB_UGUARD) {
            d_L.swap(pre[0]);
            d_U.swap(pre[1]);
        } else {
            d_L.alloc_guarded(std::max<i64>(lval_total, 1), SB_UGUARD);
            d_U.alloc_guarded(std::max<i64>(uval_total, 1), SB_UGUARD);
        }
        tick("layout + alloc");
        if (opts.overlap_upload || xmode || zmode) join_streams();
        if (opts.overlap_upload) {
            // the H2D copy of the values runs beside the rest of the plan
            // build (index exchange, levels, schedule, device tables)
            up_thread = std::thread([this] {
                try {
                    HIPCHK(hipSetDevice(comm ? comm->device : 0));
                    upload_values();
                } catch (const std::exception &e) {
                    up_err = e.what();
                }
            });
        }
        if (opts.overlap_download) {
            // the pinned D2H slots (hipHostMalloc, ~0.1 s the first time in a
            // process) are allocated beside the plan build too
            if (const char *e = getenv("SLU_D2H_SLOT_KB")) {
                D2H_SLOT = std::max<i64>(16, atoll(e)) << 10;
                D2H_MIN = D2H_SLOT / 4;
            }
            pin_thread = std::thread([this] {
                try {
                    HIPCHK(hipSetDevice(comm ? comm->device : 0));
                    // get() frees slots of another size: never while a
                    // run_d2h (which holds `use`) still copies through them
                    std::lock_guard<std::mutex> in_use(pinned_pool(1).use);
                    pinned_pool(1).get(D2H_NS, D2H_SLOT);
                } catch (const std::exception &e) {
                    pin_err = e.what();
                }
            });
        }
        try {
            build_local();
            tick("build_local");
            exchange_index();
            exchange_needs();
            tick("exchange_index");
            compute_levels();
            tick("compute_levels");
            layout_values();
            tick("layout_values");
            if (zmode) build_zranges(true);
            build_schedule();
            if (prof)
                fprintf(stderr, "[slu plan %d]   (add_supernode %.1f ms, merge + atomics %.1f ms: "
                                "resize %.1f, copy %.1f, tiles %.1f)\n",
                        iam, t_addsn, t_merge, t_resize, t_put, t_tiles);
            tick("build_schedule");
            join_streams();
            build_device();
            tick("build_device");
            build_d2h();
            tick("build_d2h");
        } catch (...) {
            if (stream_thread.joinable()) stream_thread.join();
            if (up_thread.joinable()) up_thread.join();
            if (pin_thread.joinable()) pin_thread.join();
            throw;
        }
        stats.t_plan_ms = ms_since(t0);
    }

    bool dry = false;  // schedule-only plan (opts.schedule_only): no device state

    // Replays every level's exchange phases of factor() -- the diagonal
    // packages, then the panels, issue() for issue() -- through the
    // transport on host arenas.  Each section carries bytes derived from
    // (level, group, root, mask, position), written by its root and checked
    // by every receiver, so a section that goes to the wrong rank, in the
    // wrong order or with the wrong size fails (or, with a missing send,
    // hangs) here instead of on the RCCL node.
    void check_exchange(int64_t *nsec, int64_t *nbytes) override {
        SLU_REQUIRE(dry, "check_exchange needs a schedule-only plan");
        vector<unsigned char> hd((size_t)std::max<i64>(dpk_total, 1) * sizeof(T)),
            hp((size_t)std::max<i64>(pan_total, 1) * sizeof(T));
        // bytes of the k-th section of root rank gr in phase ph of level L
        // (an owner's diagonal package goes to its column and its row from
        // one buffer, so the group is not part of it)
        auto pat = [](size_t L, int ph, int gr, int k, size_t i) {
            uint64_t h = (uint64_t)(L * 2 + ph) * 0x9E3779B97F4A7C15ull ^
                         (uint64_t)(gr * 1031 + k) * 0xBF58476D1CE4E5B9ull ^
                         (uint64_t)i * 0xD6E8FEB86659FD93ull;
            return (unsigned char)(h ^ (h >> 29) ^ (h >> 43));
        };
        auto root_rank = [&](const Sec &sc) { // global rank of the section's root
            return sc.g == G_ROW ? myrow * Pc + sc.root : sc.root * Pc + mycol;
        };
        i64 ns = 0, nb = 0;
        const int nzp = zmode ? my_last + 1 : 1;
        for (int zp = 0; zp < nzp; ++zp) {
        const size_t L0 = zmode ? phase_lv[zp] : 0, L1 = zmode ? phase_lv[zp + 1] : levels.size();
        for (size_t L = L0; L < L1; ++L) {
            const LevelRange &R = levels[L];
            // phase 0: the diagonal packages; phase 1: the panels, one flush
            // per chunk as factor() issues them
            for (int ph = 0; ph < 2; ++ph) {
                const vector<Sec> &secs = ph ? psecs : dsecs;
                const int off = ph ? R.ps_off : R.ds_off, cnt = ph ? R.ps_n : R.ds_n;
                unsigned char *arena = ph ? hp.data() : hd.data();
                // k = position among the level phase's sections of (group, root)
                vector<int> kth(cnt);
                {
                    std::map<std::pair<int, int>, int> seen;
                    for (int i = 0; i < cnt; ++i) kth[i] = seen[{secs[off + i].g, secs[off + i].root}]++;
                }
                const int nparts = ph ? R.nch : 1;
                for (int part = 0; part < nparts; ++part) {
                const int a0 = ph ? off + R.ps_o[part] : off, a1 = ph ? off + R.ps_o[part + 1] : off + cnt;
                for (int i = a0; i < a1; ++i) {
                    const Sec &sc = secs[i];
                    const int me = sc.g == G_ROW ? mycol : myrow;
                    const size_t bytes = (size_t)sc.cnt * sizeof(T);
                    if (me == sc.root) {
                        SLU_REQUIRE(sc.off >= 0, "root of a section without a buffer");
                        for (size_t b = 0; b < bytes; ++b)
                            arena[(size_t)sc.off * sizeof(T) + b] = pat(L, ph, root_rank(sc), kth[i - off], b);
                    } else if (sc.off >= 0) {
                        memset(arena + (size_t)sc.off * sizeof(T), 0, bytes);
                    }
                }
                for (int i = a0; i < a1; ++i) {
                    const Sec &sc = secs[i];
                    X.section(sc.g, sc.root, sc.mask,
                              sc.off >= 0 ? arena + (size_t)sc.off * sizeof(T) : nullptr,
                              (size_t)sc.cnt * sizeof(T));
                }
                X.phase = ph ? "L/U panel exchange (replay)" : "diagonal-package exchange (replay)";
                X.level = (int)L;
                X.flush();
                X.phase = "plan-time exchange";
                X.level = -1;
                for (int i = a0; i < a1; ++i) {
                    const Sec &sc = secs[i];
                    const int me = sc.g == G_ROW ? mycol : myrow;
                    if (me == sc.root || !(sc.mask >> me & 1)) continue;
                    SLU_REQUIRE(sc.off >= 0, "level %zu: a section for this rank has no buffer", L);
                    const size_t bytes = (size_t)sc.cnt * sizeof(T);
                    for (size_t b = 0; b < bytes; ++b)
                        SLU_REQUIRE(arena[(size_t)sc.off * sizeof(T) + b] ==
                                        pat(L, ph, root_rank(sc), kth[i - off], b),
                                    "level %zu: section (group %d root %d) byte %zu differs", L, sc.g,
                                    sc.root, b);
                    ++ns;
                    nb += (i64)bytes;
                }
                }
            }
        }
        if (zmode && zp < maxlvl - 1) { // the ancestor reduction after my phase zp
            const bool recv = zl % (2 << zp) == 0;
            const int peer = recv ? zl + (1 << zp) : zl - (1 << zp), root = recv ? peer : zl;
            const size_t bytes = (size_t)zr_cnt[zp] * sizeof(T);
            vector<unsigned char> zb(std::max<size_t>(bytes, 1), 0);
            if (!recv)
                for (size_t b = 0; b < bytes; ++b) zb[b] = pat(1000000 + zp, 0, root, iam, b);
            X.section(G_Z, root, 1u << (recv ? zl : peer), zb.data(), bytes);
            X.phase = "3D ancestor reduction (replay)";
            X.level = zp;
            X.flush();
            X.phase = "plan-time exchange";
            X.level = -1;
            if (recv && bytes) {
                for (size_t b = 0; b < bytes; ++b)
                    SLU_REQUIRE(zb[b] == pat(1000000 + zp, 0, root, iam, b),
                                "3D reduction %d: byte %zu from layer %d differs", zp, b, root);
                ++ns;
                nb += (i64)bytes;
            }
        }
        }
        // the final info reduction of factor()
        vector<i64> mine(1, iam);
        auto all = X.allgatherv(G_WORLD, mine);
        for (int r = 0; r < Pr * Pc; ++r) SLU_REQUIRE(all[r].size() == 1 && all[r][0] == r, "info all-gather");
        if (zmode) {
            mine[0] = zl;
            auto az = X.allgatherv(G_Z, mine);
            for (int z = 0; z < npdep; ++z) SLU_REQUIRE(az[z].size() == 1 && az[z][0] == z, "3D info all-gather");
        }
        *nsec = ns;
        *nbytes = nb;
    }

    bool prof = false; // SLU_PROFILE_PLAN: phase times of the plan build on stderr
    std::chrono::steady_clock::time_point tprev;
    void tick(const char *what) {
        if (!prof) return;
        const auto now = std::chrono::steady_clock::now();
        fprintf(stderr, "[slu plan %d] %-18s %8.1f ms\n", iam, what,
                std::chrono::duration<double, std::milli>(now - tprev).count());
        tprev = now;
    }

    static double ms_since(std::chrono::steady_clock::time_point t0) {
        return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0)
            .count();
    }

    ~Plan() override {
        if (up_thread.joinable()) up_thread.join();
        if (pin_thread.joinable()) pin_thread.join();
        for (auto e : ev_pan) (void)hipEventDestroy(e);
        for (auto e : ev_rest) (void)hipEventDestroy(e);
        if (ev_start) (void)hipEventDestroy(ev_start);
        if (ev_pend) (void)hipEventDestroy(ev_pend);
        if (ev_tu0) (void)hipEventDestroy(ev_tu0);
        if (ev_tu1) (void)hipEventDestroy(ev_tu1);
        if (ev_pk) (void)hipEventDestroy(ev_pk);
        if (ev_dx) (void)hipEventDestroy(ev_dx);
        for (hipEvent_t e : ev_cx)
            if (e) (void)hipEventDestroy(e);
        if (cstream) (void)hipStreamDestroy(cstream);
        if (stream) (void)hipStreamDestroy(stream);
        if (pstream) (void)hipStreamDestroy(pstream);
        if (ustream) (void)hipStreamDestroy(ustream);
    }

    // ------------------------------------------------------- local layout
    // Value offsets of the rank's L block columns / U block rows in d_L /
    // d_U (the order of Lnzval_bc_dat / Unzval_br_dat, so that the upload can
    // start before the rest of the plan exists).
    void value_layout() {
        LocalLU *Llu = LU->Llu;
        lval_off.assign(nlc, -1);
        lval_ld.assign(nlc, 0);
        i64 off = 0;
        l_contig = Llu->Lnzval_bc_dat != nullptr;
        for (int ljb = 0; ljb < nlc; ++ljb) {
            const int_t *index = Llu->Lrowind_bc_ptr[ljb];
            if (!index) continue;
            lval_off[ljb] = off;
            lval_ld[ljb] = (int)index[1];
            if (Llu->Lnzval_bc_dat && (HT *)Llu->Lnzval_bc_ptr[ljb] != (HT *)Llu->Lnzval_bc_dat + off)
                l_contig = false;
            off += (i64)index[1] * W(ljb * Pc + mycol);
        }
        lval_total = off;
        uval_off.assign(nlr, -1);
        uval_len.assign(nlr, 0);
        off = 0;
        u_contig = Llu->Unzval_br_dat != nullptr;
        for (int lb = 0; lb < nlr; ++lb) {
            const int_t *index = Llu->Ufstnz_br_ptr[lb];
            if (!index) continue;
            uval_off[lb] = off;
            uval_len[lb] = index[1];
            if (Llu->Unzval_br_dat && (HT *)Llu->Unzval_br_ptr[lb] != (HT *)Llu->Unzval_br_dat + off)
                u_contig = false;
            off += index[1];
        }
        uval_total = off;
    }

    // Destination tables (LBlk + lmap per L block, UBlk + per-column segment
    // offsets per U block) in two parallel passes: sizes per block column /
    // row, prefix sums, then every column / row fills its own slice.
    void build_local() {
        LocalLU *Llu = LU->Llu;
        // ---- L block columns
        lcol_first.assign(nlc + 1, 0);
        lcol_nblk.assign(nlc, 0);
        vector<i64> mapbase(nlc + 1, 0);
        parallel_for(nlc, [&](int ljb) {
            const int_t *index = Llu->Lrowind_bc_ptr[ljb];
            if (!index) return;
            i64 p = SLU_BC_HEADER, ml = 0;
            for (int b = 0; b < index[0]; ++b) {
                ml += W(index[p]);
                p += SLU_LB_DESCRIPTOR + index[p + 1];
            }
            lcol_nblk[ljb] = (int)index[0];
            mapbase[ljb + 1] = ml;
        });
        for (int j = 0; j < nlc; ++j) {
            lcol_first[j + 1] = lcol_first[j] + lcol_nblk[j];
            mapbase[j + 1] += mapbase[j];
        }
        lblk.assign(lcol_first[nlc], LBlk{});
        lblk_ib.assign(lcol_first[nlc], 0);
        lmap.resize_uninit(mapbase[nlc]);
        parallel_for(nlc, [&](int ljb) {
            const int jb = ljb * Pc + mycol;
            const int_t *index = Llu->Lrowind_bc_ptr[ljb];
            if (!index) return;
            const int nb = (int)index[0], nsupr = (int)index[1];
            i64 p = SLU_BC_HEADER, mo = mapbase[ljb];
            std::fill(&lmap[mapbase[ljb]], &lmap[0] + mapbase[ljb + 1], -1);
            int rs = 0;
            for (int b = 0; b < nb; ++b) {
                const int gb = (int)index[p], nr = (int)index[p + 1];
                SLU_REQUIRE(gb % Pr == myrow, "L block (%d,%d) is not on process row %d", gb, jb, myrow);
                LBlk &L = lblk[lcol_first[ljb] + b];
                L.colvoff = lval_off[ljb];
                L.mapoff = mo;
                L.ld = nsupr;
                L.fcol = (int)xsup[jb];
                L.frow = (int)xsup[gb];
                for (int i = 0; i < nr; ++i) lmap[mo + index[p + 2 + i] - xsup[gb]] = rs + i;
                lblk_ib[lcol_first[ljb] + b] = gb;
                mo += W(gb);
                rs += nr;
                p += SLU_LB_DESCRIPTOR + nr;
            }
            SLU_REQUIRE(rs == nsupr, "L column %d: block rows %d != nsupr %d", jb, rs, nsupr);
        });
        lcol_first.resize(nlc);

        // ---- U block rows
        urow_first.assign(nlr + 1, 0);
        urow_nblk.assign(nlr, 0);
        vector<i64> colbase(nlr + 1, 0);
        parallel_for(nlr, [&](int lb) {
            const int_t *index = Llu->Ufstnz_br_ptr[lb];
            if (!index) return;
            i64 p = SLU_BR_HEADER, nc = 0;
            for (int b = 0; b < index[0]; ++b) {
                nc += W(index[p]);
                p += SLU_UB_DESCRIPTOR + W(index[p]);
            }
            urow_nblk[lb] = (int)index[0];
            colbase[lb + 1] = nc;
        });
        for (int j = 0; j < nlr; ++j) {
            urow_first[j + 1] = urow_first[j] + urow_nblk[j];
            colbase[j + 1] += colbase[j];
        }
        ublk.assign(urow_first[nlr], UBlk{});
        ublk_jb.assign(urow_first[nlr], 0);
        ucol_voff.resize_uninit(colbase[nlr]);
        ucol_fst.resize_uninit(colbase[nlr]);
        parallel_for(nlr, [&](int lb) {
            const int gb = lb * Pr + myrow;
            const int_t *index = Llu->Ufstnz_br_ptr[lb];
            if (!index) return;
            const int nb = (int)index[0];
            const i64 len = index[1], klst = xsup[gb + 1], off = uval_off[lb];
            i64 p = SLU_BR_HEADER, run = 0, co = colbase[lb];
            for (int b = 0; b < nb; ++b) {
                const int jb = (int)index[p];
                SLU_REQUIRE(jb % Pc == mycol, "U block (%d,%d) is not on process column %d", gb, jb, mycol);
                UBlk &U = ublk[urow_first[lb] + b];
                U.coloff = co;
                U.fcol = (int)xsup[jb];
                for (int c = 0; c < W(jb); ++c, ++co) {
                    const i64 fst = index[p + SLU_UB_DESCRIPTOR + c];
                    ucol_voff[co] = off + run;
                    ucol_fst[co] = (int)fst;
                    run += klst - fst;
                }
                ublk_jb[urow_first[lb] + b] = jb;
                p += SLU_UB_DESCRIPTOR + W(jb);
            }
            SLU_REQUIRE(run == len, "U row %d: segment lengths %lld != %lld", gb, (long long)run, (long long)len);
        });
        urow_first.resize(nlr);
    }

    int find_lblk(int ib, int jb) const { // local column jb, block ib
        int ljb = jb / Pc, f = lcol_first[ljb], nb = lcol_nblk[ljb];
        auto b = lblk_ib.begin() + f, e = b + nb;
        auto it = std::lower_bound(b, e, ib);
        SLU_REQUIRE(it != e && *it == ib, "missing L block (%d,%d)", ib, jb);
        return (int)(it - lblk_ib.begin());
    }
    int find_ublk(int ib, int jb) const { // local row ib, block jb
        int lb = ib / Pr, f = urow_first[lb], nb = urow_nblk[lb];
        auto b = ublk_jb.begin() + f, e = b + nb;
        auto it = std::lower_bound(b, e, jb);
        SLU_REQUIRE(it != e && *it == jb, "missing U block (%d,%d)", ib, jb);
        return (int)(it - ublk_jb.begin());
    }

    // length of an index array in the reference formats
    i64 lidx_len(const int_t *ix) const {
        i64 p = SLU_BC_HEADER;
        for (i64 b = 0; b < ix[0]; ++b) p += SLU_LB_DESCRIPTOR + ix[p + 1];
        return p;
    }
    i64 uidx_len(const int_t *ix) const {
        i64 p = SLU_BR_HEADER;
        for (i64 b = 0; b < ix[0]; ++b) p += SLU_UB_DESCRIPTOR + W(ix[p]);
        return p;
    }
    // rows of L(:,k) on my process row below the diagonal block, and the
    // number of rows of the diagonal block stored on top (0 or W(k))
    void lrows(int k, int &m, int &r0) const {
        m = r0 = 0;
        const int_t *ix = lidx[k];
        if (!ix) return;
        i64 p = SLU_BC_HEADER;
        for (i64 b = 0; b < ix[0]; ++b) {
            int nr = (int)ix[p + 1];
            if (ix[p] == k) r0 += nr;
            else m += nr;
            p += SLU_LB_DESCRIPTOR + nr;
        }
    }

    // ------------------------------------------------------- index exchange
    // The reference ships lsub/usub with every panel message
    // (SRC/pdgstrf.c:1039-1044,1330-1335); the structure never changes during
    // the factorization, so it is exchanged once here.
    void exchange_index() {
        LocalLU *Llu = LU->Llu;
        lidx.assign(nsupers, nullptr);
        uidx.assign(nsupers, nullptr);
        for (int ljb = 0; ljb < nlc; ++ljb)
            if (ljb * Pc + mycol < nsupers) lidx[ljb * Pc + mycol] = Llu->Lrowind_bc_ptr[ljb];
        for (int lb = 0; lb < nlr; ++lb)
            if (lb * Pr + myrow < nsupers) uidx[lb * Pr + myrow] = Llu->Ufstnz_br_ptr[lb];
        if (!xmode) return;
        if (Pc > 1) {
            vector<i64> blob;
            for (int ljb = 0; ljb < nlc; ++ljb) {
                const int_t *ix = Llu->Lrowind_bc_ptr[ljb];
                if (!ix) continue;
                i64 len = lidx_len(ix);
                blob.push_back(ljb);
                blob.push_back(len);
                blob.insert(blob.end(), ix, ix + len);
            }
            xL = X.allgatherv(G_ROW, blob);
            for (int c = 0; c < Pc; ++c) {
                if (c == mycol) continue;
                const vector<i64> &v = xL[c];
                for (size_t p = 0; p < v.size();) {
                    i64 ljb = v[p], len = v[p + 1];
                    lidx[ljb * Pc + c] = (const int_t *)&v[p + 2];
                    p += 2 + len;
                }
            }
        }
        if (Pr > 1) {
            vector<i64> blob;
            for (int lb = 0; lb < nlr; ++lb) {
                const int_t *ix = Llu->Ufstnz_br_ptr[lb];
                if (!ix) continue;
                i64 len = uidx_len(ix);
                blob.push_back(lb);
                blob.push_back(len);
                blob.insert(blob.end(), ix, ix + len);
            }
            xU = X.allgatherv(G_COL, blob);
            for (int r = 0; r < Pr; ++r) {
                if (r == myrow) continue;
                const vector<i64> &v = xU[r];
                for (size_t p = 0; p < v.size();) {
                    i64 lb = v[p], len = v[p + 1];
                    uidx[lb * Pr + r] = (const int_t *)&v[p + 2];
                    p += 2 + len;
                }
            }
        }
    }

    // Who needs what (2D grids), as the reference's ToSendR / ToSendD
    // (SRC/pddistribute.c:752-801) but derived from the exchanged structure:
    //   rneed[k*Pc + pc]: U(k,:) has blocks on process column pc -- those
    //     ranks need L(:,k) and the factored diagonal block (U-TRSM on the
    //     owner's process row);
    //   cneed[k*Pr + pr]: L(:,k) has rows below the diagonal block on process
    //     row pr -- those ranks need U(k,:) and the diagonal block (L-TRSM).
    // Each rank knows its own column's / row's entries; one row and one
    // column all-gather make them global on every rank.
    vector<char> rneed, cneed;
    void exchange_needs() {
        if (!xmode) return;
        rneed.assign((size_t)nsupers * Pc, 0);
        cneed.assign((size_t)nsupers * Pr, 0);
        vector<i64> mine_r(nsupers), mine_c(nsupers);
        for (int k = 0; k < nsupers; ++k) {
            mine_r[k] = uidx[k] != nullptr;
            mine_c[k] = lsend(k);
        }
        vector<vector<i64>> ar, ac;
        if (Pc > 1) ar = X.allgatherv(G_ROW, mine_r);
        else ar.push_back(mine_r);
        if (Pr > 1) ac = X.allgatherv(G_COL, mine_c);
        else ac.push_back(mine_c);
        for (int k = 0; k < nsupers; ++k) {
            for (int c = 0; c < Pc; ++c) rneed[(size_t)k * Pc + c] = (char)ar[c][k];
            for (int r = 0; r < Pr; ++r) cneed[(size_t)k * Pr + r] = (char)ac[r][k];
        }
    }
    uint32_t rmask(int k) const {
        uint32_t m = 0;
        for (int c = 0; c < Pc; ++c) m |= (uint32_t)rneed[(size_t)k * Pc + c] << c;
        return m;
    }
    uint32_t cmask(int k) const {
        uint32_t m = 0;
        for (int r = 0; r < Pr; ++r) m |= (uint32_t)cneed[(size_t)k * Pr + r] << r;
        return m;
    }

    // ------------------------------------------------------- levels
    // Dependency DAG k -> ib (L(ib,k) != 0) and k -> jb (U(k,jb) != 0); all
    // edges point to larger supernode numbers, so one ascending sweep gives
    // the longest-path level.  On a grid every rank contributes its local
    // blocks and all ranks compute the same levels.
    void compute_levels() {
        vector<i64> edges;
        for (int ljb = 0; ljb < nlc; ++ljb) {
            int k = ljb * Pc + mycol;
            if (k >= nsupers || !lidx[k]) continue;
            const int_t *ix = lidx[k];
            i64 p = SLU_BC_HEADER;
            for (i64 b = 0; b < ix[0]; ++b) {
                if (ix[p] != k) {
                    edges.push_back(k);
                    edges.push_back(ix[p]);
                }
                p += SLU_LB_DESCRIPTOR + ix[p + 1];
            }
        }
        for (int lb = 0; lb < nlr; ++lb) {
            int k = lb * Pr + myrow;
            if (k >= nsupers || !uidx[k]) continue;
            const int_t *ix = uidx[k];
            i64 p = SLU_BR_HEADER;
            for (i64 b = 0; b < ix[0]; ++b) {
                edges.push_back(k);
                edges.push_back(ix[p]);
                p += SLU_UB_DESCRIPTOR + W(ix[p]);
            }
        }
        vector<vector<i64>> all;
        if (xmode) all = X.allgatherv(G_WORLD, edges);
        else all.push_back(std::move(edges));
        // CSR of the edges by source
        vector<i64> cnt(nsupers + 1, 0);
        for (auto &v : all)
            for (size_t e = 0; e < v.size(); e += 2) cnt[v[e] + 1]++;
        for (int k = 0; k < nsupers; ++k) cnt[k + 1] += cnt[k];
        vector<int> tgt(cnt[nsupers]);
        vector<i64> fill(cnt.begin(), cnt.end() - 1);
        for (auto &v : all)
            for (size_t e = 0; e < v.size(); e += 2) {
                SLU_REQUIRE(v[e + 1] > v[e] && v[e + 1] < nsupers, "bad dependency %lld -> %lld",
                            (long long)v[e], (long long)v[e + 1]);
                tgt[fill[v[e]]++] = (int)v[e + 1];
            }
        if (zmode) return compute_levels_3d(cnt, tgt);
        level_of.assign(nsupers, 0);
        int maxlev = 0;
        for (int k = 0; k < nsupers; ++k) {
            maxlev = std::max(maxlev, level_of[k]);
            for (i64 e = cnt[k]; e < cnt[k + 1]; ++e)
                level_of[tgt[e]] = std::max(level_of[tgt[e]], level_of[k] + 1);
        }
        bylev.assign(maxlev + 1, {});
        for (int k = 0; k < nsupers; ++k) bylev[level_of[k]].push_back(k);
        levels.assign(maxlev + 1, LevelRange{});
        stats.nsupers = nsupers;
        stats.nsupers_in = nsupers;
        stats.nlevels = maxlev + 1;
    }

    // ------------------------------------------------------- 3D forests
    // The forest partition of SRC/supernodalForest.c (getGreedyLoadBalForests
    // :794, iterativeFrPartitioning :618, getLoadImbalance :463): starting
    // from the etree's roots, while the two-way greedy split of the current
    // tree set is more than 20 % imbalanced (and fewer than 1024 trees), the
    // heaviest tree's single-child chain from its root down to the first
    // branching goes to the ancestor forest and the branch's children replace
    // it; the set is then split greedily (heaviest first, into the lighter
    // half) and each half is partitioned the same way one level down; the
    // halves at the bottom are the layers' leaf forests.  The tree is the
    // elimination tree of the block dependency DAG (Liu's algorithm with path
    // compression over the DAG's edges), so every supernode a block column
    // or row of k updates is an ancestor of k -- the property the phases rely
    // on.  Weights estimate each supernode's Schur work, w * m^2 with m the
    // summed widths of its successors (the reference's scuWeight, from the
    // same block structure).
    void compute_forests(const vector<i64> &cnt, const vector<int> &tgt) {
        const int ns = nsupers;
        vector<int> parent(ns, -1), anc(ns, -1);
        {   // edges by target
            vector<i64> rc(ns + 1, 0);
            for (int k = 0; k < ns; ++k)
                for (i64 e = cnt[k]; e < cnt[k + 1]; ++e) rc[tgt[e] + 1]++;
            for (int k = 0; k < ns; ++k) rc[k + 1] += rc[k];
            vector<int> src(rc[ns]);
            vector<i64> f(rc.begin(), rc.end() - 1);
            for (int k = 0; k < ns; ++k)
                for (i64 e = cnt[k]; e < cnt[k + 1]; ++e) src[f[tgt[e]]++] = k;
            for (int t = 0; t < ns; ++t)
                for (i64 e = rc[t]; e < rc[t + 1]; ++e) {
                    int r = src[e];
                    while (anc[r] != -1 && anc[r] != t) { // root of r's current subtree
                        const int nx = anc[r];
                        anc[r] = t;                       // path compression
                        r = nx;
                    }
                    if (anc[r] == -1 && r != t) {
                        parent[r] = t;
                        anc[r] = t;
                    }
                }
        }
        vector<double> wt(ns, 0), sub(ns, 0);
        for (int k = 0; k < ns; ++k) {
            double m = 0;
            for (i64 e = cnt[k]; e < cnt[k + 1]; ++e) m += W(tgt[e]);
            wt[k] = (double)W(k) * (m * m + (double)W(k) * W(k) / 3.0) + 1.0;
        }
        vector<vector<int>> kids(ns);
        vector<int> roots;
        for (int k = 0; k < ns; ++k) {
            sub[k] += wt[k];
            if (parent[k] >= 0) {
                sub[parent[k]] += sub[k];
                kids[parent[k]].push_back(k);
            } else {
                roots.push_back(k);
            }
        }
        const int nf = (1 << maxlvl) - 1;
        forest_of.assign(ns, -1);
        if (opts.forest_map) { // the caller's partition (pdgstrf3d: supernode2treeMap)
            for (int k = 0; k < ns; ++k) {
                SLU_REQUIRE(opts.forest_map[k] >= 0 && opts.forest_map[k] < nf,
                            "forest map: supernode %d in forest %lld of %d", k,
                            (long long)opts.forest_map[k], nf);
                forest_of[k] = (int)opts.forest_map[k];
            }
            return;
        }
        vector<vector<int>> heads((size_t)nf);
        heads[0] = roots;
        auto split2 = [&](vector<int> set, vector<int> *out) {
            std::stable_sort(set.begin(), set.end(), [&](int a, int b) { return sub[a] > sub[b]; });
            double w[2] = {0, 0};
            for (int t : set) {
                const int h = w[0] > w[1] ? 1 : 0;
                w[h] += sub[t];
                if (out) out[h].push_back(t);
            }
            return w[0] + w[1] > 0 ? std::fabs(w[0] - w[1]) / (w[0] + w[1]) : 0.0;
        };
        auto mark_subtrees = [&](const vector<int> &hs, int f) {
            vector<int> st(hs.begin(), hs.end());
            while (!st.empty()) {
                const int v = st.back();
                st.pop_back();
                forest_of[v] = f;
                for (int c : kids[v]) st.push_back(c);
            }
        };
        if (maxlvl == 1) mark_subtrees(heads[0], 0);
        for (int lvl = 0; lvl < maxlvl - 1; ++lvl)
            for (int tr = (1 << lvl) - 1; tr < (1 << (lvl + 1)) - 1; ++tr) {
                vector<int> set = heads[tr];
                while (split2(set, nullptr) > 0.2 && set.size() < 1024) {
                    size_t idx = 0;
                    for (size_t i = 1; i < set.size(); ++i)
                        if (sub[set[i]] > sub[set[idx]]) idx = i;
                    int v = set[idx];
                    while (kids[v].size() == 1) v = kids[v][0];
                    if (kids[v].empty()) break;
                    for (int u = set[idx];; u = kids[u][0]) { // the chain joins the ancestors
                        forest_of[u] = tr;
                        if (u == v) break;
                    }
                    set.erase(set.begin() + idx);
                    set.insert(set.end(), kids[v].begin(), kids[v].end());
                }
                vector<int> half[2];
                split2(set, half);
                if (lvl == maxlvl - 2) {
                    mark_subtrees(half[0], 2 * tr + 1);
                    mark_subtrees(half[1], 2 * tr + 2);
                } else {
                    heads[2 * tr + 1] = half[0];
                    heads[2 * tr + 2] = half[1];
                }
            }
        for (int k = 0; k < ns; ++k) SLU_REQUIRE(forest_of[k] >= 0, "supernode %d in no forest", k);
    }

    // heap index of layer z's forest at level ilvl (0 = leaves), as
    // SRC/supernodal_etree.c:802-812 (getGridTrees)
    int tree_of(int z, int ilvl) const {
        int t = npdep - 1 + z;
        for (int i = 0; i < ilvl; ++i) t = (t - 1) / 2;
        return t;
    }
    int ilvl_of_forest(int f) const { // 0 = leaves
        int d = 0;
        while ((2 << d) - 1 <= f) ++d;
        return maxlvl - 1 - d;
    }

    void compute_levels_3d(const vector<i64> &cnt, const vector<int> &tgt) {
        compute_forests(cnt, tgt);
        my_last = 0;
        while (my_last < maxlvl - 1 && zl % (2 << my_last) == 0) ++my_last;
        phase_of.assign(nsupers, -1);
        for (int k = 0; k < nsupers; ++k) {
            const int il = ilvl_of_forest(forest_of[k]);
            if (forest_of[k] == tree_of(zl, il) && il <= my_last) phase_of[k] = il;
        }
        // every block a factored supernode updates lies on this layer's path
        // of forests at its phase or above (the partition's invariant)
        for (int k = 0; k < nsupers; ++k) {
            if (phase_of[k] < 0) continue;
            for (i64 e = cnt[k]; e < cnt[k + 1]; ++e) {
                const int t = tgt[e], il = ilvl_of_forest(forest_of[t]);
                SLU_REQUIRE(il >= phase_of[k] && forest_of[t] == tree_of(zl, il),
                            "3D forests: supernode %d (phase %d) updates %d outside its path", k,
                            phase_of[k], t);
            }
        }
        vector<int> lin(nsupers, 0);
        vector<int> depth(maxlvl, 0);
        for (int k = 0; k < nsupers; ++k) {
            if (phase_of[k] < 0) continue;
            depth[phase_of[k]] = std::max(depth[phase_of[k]], lin[k] + 1);
            for (i64 e = cnt[k]; e < cnt[k + 1]; ++e)
                if (phase_of[tgt[e]] == phase_of[k]) lin[tgt[e]] = std::max(lin[tgt[e]], lin[k] + 1);
        }
        phase_lv.assign(my_last + 2, 0);
        for (int p = 0; p <= my_last; ++p) phase_lv[p + 1] = phase_lv[p] + depth[p];
        const int nl = phase_lv[my_last + 1];
        level_of.assign(nsupers, -1);
        bylev.assign(nl, {});
        for (int k = 0; k < nsupers; ++k)
            if (phase_of[k] >= 0) {
                level_of[k] = phase_lv[phase_of[k]] + lin[k];
                bylev[level_of[k]].push_back(k);
            }
        levels.assign(nl, LevelRange{});
        int nf = 0;
        for (int k = 0; k < nsupers; ++k) nf += phase_of[k] >= 0;
        stats.npdep = npdep;
        stats.zlayer = zl;
        stats.phase_last = my_last;
        stats.nsupers = nf;
        stats.nsupers_in = nsupers;
        stats.nlevels = nl;
    }

    // local value ranges of supernode k's L block column / U block row,
    // appended to zr in chunks (buffer positions from *bo on)
    void add_zranges(int k, i64 *bo) {
        auto add = [&](i64 off, i64 len, int arr) {
            for (i64 c = 0; c < len; c += ZR_CHUNK) {
                const int l = (int)std::min<i64>(ZR_CHUNK, len - c);
                zr.push_back(ZRange{off + c, *bo, l, arr});
                *bo += l;
            }
        };
        if (k % Pc == mycol && lval_off[k / Pc] >= 0)
            add(lval_off[k / Pc], (i64)lval_ld[k / Pc] * W(k), 0);
        if (k % Pr == myrow && uval_off[k / Pr] >= 0) add(uval_off[k / Pr], uval_len[k / Pr], 1);
    }

    void build_zranges(bool device) {
        zr.clear();
        zr_off.assign(1, 0);
        zr_cnt.clear();
        i64 bo = 0;
        // ancestor forests this layer does not factor start from zero
        for (int k = 0; k < nsupers; ++k) {
            const int il = ilvl_of_forest(forest_of[k]);
            if (il >= 1 && forest_of[k] == tree_of(zl, il) && il > my_last) add_zranges(k, &bo);
        }
        zr_off.push_back((int)zr.size());
        // reduction after phase p: every ancestor forest above it on my path
        i64 mx = 0;
        for (int p = 0; p < maxlvl - 1; ++p) {
            bo = 0;
            if (p <= my_last)
                for (int k = 0; k < nsupers; ++k) {
                    const int il = ilvl_of_forest(forest_of[k]);
                    if (il > p && forest_of[k] == tree_of(zl, il)) add_zranges(k, &bo);
                }
            zr_off.push_back((int)zr.size());
            zr_cnt.push_back(bo);
            if (p < 8) stats.zred_bytes[p] = (double)bo * sizeof(T);
            mx = std::max(mx, bo);
        }
        if (!device) return;
        d_zr.upload(zr);
        d_zbuf.alloc(std::max<i64>(mx, 1));
    }

    void launch_zranges(int a, int b, int op, hipStream_t st) {
        if (b > a)
            hipLaunchKernelGGL(k_zranges<T>, dim3(b - a), dim3(256), 0, st, d_zr.p + a, d_L.p, d_U.p,
                               d_zbuf.p, op);
    }

    // ancestor reduction at the end of phase p (SRC/pd3dcomm.c:786-813):
    // layer z + 2^p sends its partial sums, layer z adds them
    void zreduce(int p, hipStream_t st) {
        const bool recv = zl % (2 << p) == 0;
        const int peer = recv ? zl + (1 << p) : zl - (1 << p);
        const int a = zr_off[p + 1], b = zr_off[p + 2];
        const i64 cnt = zr_cnt[p];
        if (!recv) launch_zranges(a, b, ZR_PACK, st);
        X.s = st;
        if (!zsolo) {
            X.section(G_Z, recv ? peer : zl, 1u << (recv ? zl : peer), d_zbuf.p, (size_t)cnt * sizeof(T));
            X.phase = "3D ancestor reduction";
            X.level = p;
            X.flush();
            X.phase = "plan-time exchange";
            X.level = -1;
        }
        zbytes += (double)cnt * sizeof(T);
        if (recv) launch_zranges(a, b, ZR_ADD, st);
    }

    // After factor(): the factored forests travel to layer 0 (every layer's
    // part of it), as pdgssvx3d's dgatherAllFactoredLU (SRC/pd3dcomm.c:816-858).
    void gather_layers() override {
        SLU_REQUIRE(zmode, "gather_layers: not a 3D plan");
        SLU_REQUIRE(vstate == 2, "gather_layers: factor first");
        sync();
        hipStream_t st = stream;
        for (int il = 0; il < maxlvl - 1; ++il) {
            if (zl % (1 << il)) break;
            const bool recv = zl % (2 << il) == 0;
            const int sender = recv ? zl + (1 << il) : zl, peer = recv ? sender : zl - (1 << il);
            // forests the sender's half of the layers factored: at level a
            // <= il, trees (2^(maxlvl-1-a) - 1) + (sender >> a) + [0, 2^(il-a))
            vector<char> want((size_t)(1 << maxlvl), 0);
            for (int a = 0; a <= il; ++a) {
                const int t0 = (1 << (maxlvl - 1 - a)) - 1 + (sender >> a);
                for (int t = t0; t < t0 + (1 << (il - a)); ++t) want[t] = 1;
            }
            vector<ZRange> keep;
            keep.swap(zr);
            i64 bo = 0;
            for (int k = 0; k < nsupers; ++k)
                if (want[forest_of[k]]) add_zranges(k, &bo);
            DevBuf<ZRange> dr;
            dr.upload(zr);
            DevBuf<T> buf;
            buf.alloc(std::max<i64>(bo, 1));
            const int nr = (int)zr.size();
            zr.swap(keep);
            if (!recv && nr)
                hipLaunchKernelGGL(k_zranges<T>, dim3(nr), dim3(256), 0, st, dr.p, d_L.p, d_U.p, buf.p,
                                   (int)ZR_PACK);
            X.s = st;
            X.section(G_Z, sender, 1u << (recv ? zl : peer), buf.p, (size_t)bo * sizeof(T));
            X.phase = "3D gather to layer 0";
            X.level = il;
            X.flush();
            X.phase = "plan-time exchange";
            X.level = -1;
            if (recv && nr)
                hipLaunchKernelGGL(k_zranges<T>, dim3(nr), dim3(256), 0, st, dr.p, d_L.p, d_U.p, buf.p,
                                   (int)ZR_COPY);
            HIPCHK(hipStreamSynchronize(st));
            if (!recv) break;
        }
        host_current = false;
    }

    // ------------------------------------------------------- value layout
    // Diagonal packages [w*w factored block, ld w | Dinv] and remote panels
    // are laid out per level in broadcast order: sections of the owners in my
    // process column (root = their process row), then of my process row.
    // Receive buffers are a ring, as the reference's num_lookaheads + 1
    // rotating Lsub_buf_2 / Lval_buf_2 (SRC/pdgstrf.c:454-512): with the
    // one-level look-ahead of factor() only levels L and L+1 are live at a
    // time -- panel(L+2) is issued on the panel stream after it waited for
    // the rest of level L's Schur update (ev_rest[L]) -- so the panels use
    // two slots of the largest level, and the diagonal packages (read only
    // by the TRSMs of their own level, on the same stream) one.
    vector<i64> pan_level; // panel bytes (elements) per level
    bool lsend(int k) const { // L(:,k) on my process row has rows below the diagonal block
        int m, r0;
        lrows(k, m, r0);
        return m > 0;
    }
    // U(k,:) on my process column: its nonempty columns (the Schur update's
    // columns, in order) and the panel's value offset where each group of
    // csz of them starts (the U panel is the concatenation of the columns'
    // segments, SRC/superlu_defs.h:152-198)
    int ucols_runs(int k, int csz, std::array<i64, NCHM> *run) const {
        if (run) run->fill(0);
        if (!uidx[k]) return 0;
        const int_t *ix = uidx[k];
        const i64 klst = xsup[k + 1];
        i64 p = SLU_BR_HEADER, r = 0;
        int nc = 0;
        for (i64 b = 0; b < ix[0]; ++b) {
            const int jb = (int)ix[p];
            for (int c = 0; c < W(jb); ++c) {
                const i64 fst = ix[p + SLU_UB_DESCRIPTOR + c];
                if (fst >= klst) continue;
                if (run && csz > 0 && nc % csz == 0 && nc / csz < NCHM) (*run)[nc / csz] = r;
                ++nc;
                r += klst - fst;
            }
            p += SLU_UB_DESCRIPTOR + W(jb);
        }
        return nc;
    }
    void layout_values() {
        pkg.assign(nsupers, -1);
        dscr.assign(nsupers, -1);
        lpos.assign(nsupers, -1);
        upos.assign(nsupers, -1);
        if (xmode) {
            std::array<i64, NCHM> none;
            none.fill(-1);
            lgsz.assign(nsupers, 0);
            ucsz.assign(nsupers, 0);
            ucols.assign(nsupers, 0);
            lgpos.assign(nsupers, none);
            ugpos.assign(nsupers, none);
            ugrun.assign(nsupers, none);
            for (int k = 0; k < nsupers; ++k) {
                int m, r0;
                lrows(k, m, r0);
                lgsz[k] = group_size(m);
                ucols[k] = ucols_runs(k, 0, nullptr);
                ucsz[k] = group_size(ucols[k]);
                ucols_runs(k, ucsz[k], &ugrun[k]);
            }
        }
        for (size_t L = 0; L < levels.size(); ++L) {
            LevelRange &R = levels[L];
            const vector<int> &ks = bylev[L];
            if (!xmode) { // 1x1: Dinv in a per-level scratch
                i64 off = 0;
                for (int k : ks) {
                    dscr[k] = off;
                    off += dinv_len(W(k));
                }
                dscr_max = std::max(dscr_max, off);
                continue;
            }
            // ---- diag packages: owner (r, mycol) for all r, then (myrow, c),
            // c != mycol.  One section per owner and group; its mask is the
            // union over the owner's supernodes of the ranks that need a
            // package (packages are small: w*w + Dinv per supernode).
            dpk_total = 0;  // per-level cursor (one slot, reused by every level)
            pan_total = 0;  // per-level cursor (the slot base is added below)
            // layout first (owners (r, mycol) for all r, then (myrow, c)), then
            // the sections in the canonical order every member of a group
            // shares: column groups by root row, row groups by root column
            struct Own {
                uint32_t cm = 0, rm = 0;
                i64 start = -1, cnt = 0;
            };
            vector<Own> own(Pr * Pc);
            auto lay_owner = [&](int orow, int ocol) {
                const bool me = orow == myrow && ocol == mycol;
                Own &o = own[orow * Pc + ocol];
                for (int k : ks)
                    if (k % Pr == orow && k % Pc == ocol) {
                        o.cm |= cmask(k);
                        o.rm |= rmask(k);
                        o.cnt += (i64)W(k) * W(k) + dinv_len(W(k));
                    }
                if (!o.cnt) return;
                o.cm &= ~(1u << orow);
                o.rm &= ~(1u << ocol);
                const bool here = me || (ocol == mycol && (o.cm >> myrow & 1)) ||
                                  (orow == myrow && (o.rm >> mycol & 1));
                if (!here) return;
                o.start = dpk_total;
                for (int k : ks)
                    if (k % Pr == orow && k % Pc == ocol) {
                        pkg[k] = dpk_total;
                        dpk_total += (i64)W(k) * W(k) + dinv_len(W(k));
                    }
            };
            for (int r = 0; r < Pr; ++r) lay_owner(r, mycol);
            for (int c = 0; c < Pc; ++c)
                if (c != mycol) lay_owner(myrow, c);
            R.ds_off = (int)dsecs.size();
            auto sec = [&](int g, int root, const Own &o, uint32_t mask) {
                if (!mask || !o.cnt) return;
                const int me = g == G_ROW ? mycol : myrow;
                const bool rcv = me != root && (mask >> me & 1);
                dsecs.push_back({g, root, 0, (me == root || rcv) ? o.start : -1, o.cnt, mask});
                if (me == root) comm_volume += o.cnt * __builtin_popcount(mask);
                else if (rcv) comm_volume += o.cnt;
            };
            if (Pr > 1)
                for (int r = 0; r < Pr; ++r) sec(G_COL, r, own[r * Pc + mycol], own[r * Pc + mycol].cm);
            if (Pc > 1)
                for (int c = 0; c < Pc; ++c) sec(G_ROW, c, own[myrow * Pc + c], own[myrow * Pc + c].rm);
            R.ds_n = (int)dsecs.size() - R.ds_off;
            // ---- panels: L(:,k) along my process row (root = owning column),
            //      U(k,:) along my process column (root = owning row).  The
            //      supernodes of a root are grouped by the set of ranks that
            //      need them (same order on every member), one section per
            //      group and chunk, sent only to those ranks.  Chunk c of a
            //      group holds row group c of its L panels (resp. column group
            //      c of its U panels): the level's sections go out chunk by
            //      chunk, the sender's TRSM of the next chunk beside the
            //      current chunk's transfer, the receivers' Schur tiles of a
            //      chunk as soon as it is in.
            R.ps_off = (int)psecs.size();
            R.pc_off = (int)pcopy.size();
            const int nch = pchunks;
            vector<vector<Sec>> csec(nch);
            vector<vector<CopyItem<T>>> ccp(nch);
            vector<vector<char>> ccp_src(nch);
            auto lay_panels = [&](int g, int root, vector<std::pair<uint32_t, int>> &km) {
                std::sort(km.begin(), km.end());
                const int me = g == G_ROW ? mycol : myrow;
                for (size_t i = 0; i < km.size();) {
                    size_t j = i;
                    while (j < km.size() && km[j].first == km[i].first) ++j;
                    const uint32_t mask = km[i].first;
                    const bool rcv = me != root && (mask >> me & 1);
                    for (int ch = 0; mask && ch < nch; ++ch) {
                        const i64 start = (me == root || rcv) ? pan_total : -1;
                        i64 cnt = 0;
                        for (size_t q = i; q < j; ++q) {
                            const int k = km[q].second;
                            i64 len;
                            if (g == G_ROW) {
                                int m, r0;
                                lrows(k, m, r0);
                                const int gs = lgsz[k], a = ch * gs;
                                if (a >= m) continue;
                                const int rows = std::min(gs, m - a);
                                len = (i64)rows * W(k);
                                if (me == root) {
                                    const int ljb = k / Pc;
                                    add_copy(ccp[ch], ccp_src[ch], /*src*/ 0, lval_off[ljb] + r0 + a,
                                             lval_ld[ljb], 1, pan_total, rows, rows, W(k));
                                } else if (rcv) {
                                    lgpos[k][ch] = pan_total;
                                    if (ch == 0) lpos[k] = pan_total;
                                }
                            } else {
                                const int nc = ucols[k], cs = ucsz[k];
                                if (ch * cs >= nc) continue;
                                const i64 r1 = (ch + 1) * cs < nc ? ugrun[k][ch + 1] : (i64)uidx[k][1];
                                len = r1 - ugrun[k][ch];
                                if (!len) continue;
                                if (me == root) {
                                    add_copy(ccp[ch], ccp_src[ch], /*src*/ 1, uval_off[k / Pr] + ugrun[k][ch], len, 1,
                                             pan_total, len, len, 1);
                                } else if (rcv) {
                                    ugpos[k][ch] = pan_total;
                                    if (ch == 0) upos[k] = pan_total;
                                }
                            }
                            if (me == root || rcv) pan_total += len;
                            cnt += len;
                        }
                        if (!cnt) continue;
                        csec[ch].push_back({g, root, 1, start, cnt, mask});
                        if (me == root) comm_volume += cnt * __builtin_popcount(mask);
                        else if (rcv) comm_volume += cnt;
                    }
                    i = j;
                }
            };
            if (Pc > 1)
                for (int c = 0; c < Pc; ++c) {
                    vector<std::pair<uint32_t, int>> km;
                    for (int k : ks)
                        if (k % Pc == c && lsend(k)) km.push_back({rmask(k) & ~(1u << c), k});
                    lay_panels(G_ROW, c, km);
                }
            if (Pr > 1)
                for (int r = 0; r < Pr; ++r) {
                    vector<std::pair<uint32_t, int>> km;
                    for (int k : ks)
                        if (k % Pr == r && uidx[k]) km.push_back({cmask(k) & ~(1u << r), k});
                    lay_panels(G_COL, r, km);
                }
            R.nch = nch;
            R.ps_o[0] = R.pc_o[0] = 0;
            for (int ch = 0; ch < nch; ++ch) {
                psecs.insert(psecs.end(), csec[ch].begin(), csec[ch].end());
                pcopy.insert(pcopy.end(), ccp[ch].begin(), ccp[ch].end());
                pcopy_src.insert(pcopy_src.end(), ccp_src[ch].begin(), ccp_src[ch].end());
                R.ps_o[ch + 1] = (int)psecs.size() - R.ps_off;
                R.pc_o[ch + 1] = (int)pcopy.size() - R.pc_off;
            }
            R.ps_n = (int)psecs.size() - R.ps_off;
            R.pc_n = (int)pcopy.size() - R.pc_off;
            pan_level.push_back(pan_total);
            dpk_slot = std::max(dpk_slot, dpk_total);
        }
        if (!xmode) return;
        // odd levels use the second panel slot
        // (a 3D layer may factor nothing: no levels)
        const i64 slot = pan_level.empty() ? 0 : *std::max_element(pan_level.begin(), pan_level.end());
        for (size_t L = 1; L < levels.size(); L += 2) {
            const LevelRange &R = levels[L];
            for (int k : bylev[L]) {
                if (lpos[k] >= 0) lpos[k] += slot;
                if (upos[k] >= 0) upos[k] += slot;
                for (int ch = 0; ch < NCHM; ++ch) {
                    if (lgpos[k][ch] >= 0) lgpos[k][ch] += slot;
                    if (ugpos[k][ch] >= 0) ugpos[k][ch] += slot;
                }
            }
            for (int i = R.ps_off; i < R.ps_off + R.ps_n; ++i)
                if (psecs[i].off >= 0) psecs[i].off += slot;
            for (int i = R.pc_off; i < R.pc_off + R.pc_n; ++i)
                pcopy[i].dst = (T *)((intptr_t)pcopy[i].dst + slot);
        }
        pan_total = levels.size() > 1 ? 2 * slot : slot;
        dpk_total = dpk_slot;
    }
    i64 dpk_slot = 0, comm_volume = 0;

    // Copy items are recorded with symbolic bases (src space 0 = L values,
    // 1 = U values; dst = d_dpk (dst_space 0) or d_pan (1)) and relocated in
    // build_device.  Chunked to <= COPY_CHUNK elements.
    vector<char> pcopy_src, dcopy_src;
    static void add_copy(vector<CopyItem<T>> &v, vector<char> &tag, int src_space, i64 src_off,
                         i64 lds, int dst_space, i64 dst_off, i64 ldd, i64 rows, i64 cols) {
        if (cols == 1) {
            for (i64 e = 0; e < rows; e += COPY_CHUNK) {
                CopyItem<T> c{};
                c.src = (const T *)(intptr_t)(src_off + e);
                c.dst = (T *)(intptr_t)(dst_off + e);
                c.lds = c.ldd = 0;
                c.rows = (int)std::min<i64>(COPY_CHUNK, rows - e);
                c.cols = 1;
                v.push_back(c);
                tag.push_back((char)(src_space | (dst_space << 1)));
            }
            return;
        }
        if (lds == rows && ldd == rows) { // contiguous: copy as 1D
            add_copy(v, tag, src_space, src_off, 0, dst_space, dst_off, 0, rows * cols, 1);
            return;
        }
        const i64 cpc = std::max<i64>(1, COPY_CHUNK / std::max<i64>(rows, 1));
        for (i64 c0 = 0; c0 < cols; c0 += cpc) {
            CopyItem<T> c{};
            c.src = (const T *)(intptr_t)(src_off + c0 * lds);
            c.dst = (T *)(intptr_t)(dst_off + c0 * ldd);
            c.lds = lds;
            c.ldd = ldd;
            c.rows = (int)rows;
            c.cols = (int)std::min<i64>(cpc, cols - c0);
            v.push_back(c);
            tag.push_back((char)(src_space | (dst_space << 1)));
        }
    }

    // ------------------------------------------------------- schedule
    // One supernode's (or a chunk of one level's supernodes') share of the
    // schedule; offsets into its own h_* arrays are relocated when merged.
    struct KInfoHost {
        vector<int> dests;
    };
    struct SchedOut {
        vector<DiagItem<T>> diag_items;
        vector<DiagItemF<T>> df_items;
        vector<TrsmLItem<T>> tl_items;
        vector<TrsmUItem<T>> tu_items;
        vector<TrsmItemF<T>> lf_c[NCHM], uf_c[NCHM]; // per exchange chunk
        vector<KInfo<T>> kinfos;
        vector<KInfoHost> khost;
        vector<TileItem> big[2][NCHM], small[2][NCHM]; // [0] critical, [1] rest; per chunk
        vector<CopyItem<T>> dcopy;
        vector<char> dcopy_src;
        vector<int> h_rg, h_ra, h_cg, h_cb, h_pair, h_ct0;
        vector<i64> h_cvoff;
        double panel_flops = 0, schur_flops = 0, schur_flops_padded = 0, scatter_bytes = 0;
        double R_schur_flops = 0, R_big_flops = 0;
        i64 n_diag = 0, n_trsm_items = 0, n_schur_tiles = 0;
        bool R_big = false;
    };
    vector<KInfoHost> khost;

    template <typename V> static void append(V &dst, const V &src) {
        dst.insert(dst.end(), src.begin(), src.end());
    }
    template <typename P> static P *shift(P *p, i64 d) { return (P *)((intptr_t)p + d); }

    double t_addsn = 0, t_merge = 0, t_resize = 0, t_put = 0, t_tiles = 0;
    // Supernodes are scheduled in chunks (a level's supernodes in order, the
    // levels in order) into SchedOut's, all chunks of all levels at once
    // (add_supernode reads only the plan's structure); the tables are then
    // sized once and every chunk copies (and relocates) its slices in
    // parallel, which reproduces the sequential layout exactly.  Sizing per
    // level instead regrew and value-initialised every table once per level,
    // serially (66 of the 131 ms at 100^3).
    void build_schedule() {
        // value buffers first: work items point straight into them
        d_dpk.alloc(std::max<i64>(dpk_total, 1));
        d_pan.alloc_guarded(std::max<i64>(pan_total, 1), SB_UGUARD);
        d_dinv.alloc(std::max<i64>(dscr_max, 1));
        const int NL = (int)levels.size();
        vector<int> first(NL + 1, 0); // chunks of level L: [first[L], first[L+1])
        for (int L = 0; L < NL; ++L) {
            const int nk = (int)bylev[L].size();
            first[L + 1] = first[L] + (nk >= 128 ? std::min(4 * plan_threads(), nk / 32) : 1);
        }
        const int NC = first[NL];
        vector<SchedOut> outs(NC);
        const auto ta = std::chrono::steady_clock::now();
        parallel_for(NC, [&](int t) {
            const int L = (int)(std::upper_bound(first.begin(), first.end(), t) - first.begin()) - 1;
            const vector<int> &ks = bylev[L];
            const i64 nk = (i64)ks.size(), nch = first[L + 1] - first[L], c = t - first[L];
            for (i64 i = nk * c / nch; i < nk * (c + 1) / nch; ++i) add_supernode(ks[i], outs[t]);
        }, 1);
        t_addsn += ms_since(ta);
        const auto tm0 = std::chrono::steady_clock::now();
        enum { V_DIAG, V_DF, V_TL, V_TU, V_LF, V_UF, V_K, V_DC, V_RG, V_CG, V_PAIR, V_N };
        vector<std::array<i64, V_N>> base(NC + 1);
        {
            SLU_REQUIRE(kinfos.empty() && h_rg.empty() && h_cg.empty() && h_pair.empty(),
                        "build_schedule runs once per plan");
            std::array<i64, V_N> b = {(i64)diag_items.size(), (i64)df_items.size(), (i64)tl_items.size(),
                                      (i64)tu_items.size(), (i64)lf_items.size(), (i64)uf_items.size(),
                                      0, (i64)dcopy.size(), 0, 0, 0};
            for (int t = 0; t < NC; ++t) {
                const SchedOut &O = outs[t];
                base[t] = b;
                b[V_DIAG] += O.diag_items.size();
                b[V_DF] += O.df_items.size();
                b[V_TL] += O.tl_items.size();
                b[V_TU] += O.tu_items.size();
                for (int ch = 0; ch < NCHM; ++ch) {
                    b[V_LF] += O.lf_c[ch].size();
                    b[V_UF] += O.uf_c[ch].size();
                }
                b[V_K] += O.kinfos.size();
                b[V_DC] += O.dcopy.size();
                b[V_RG] += O.h_rg.size();
                b[V_CG] += O.h_cg.size();
                b[V_PAIR] += O.h_pair.size();
            }
            base[NC] = b;
            diag_items.resize(b[V_DIAG]);
            df_items.resize(b[V_DF]);
            tl_items.resize(b[V_TL]);
            tu_items.resize(b[V_TU]);
            lf_items.resize(b[V_LF]);
            uf_items.resize(b[V_UF]);
            kinfos.resize(b[V_K]);
            khost.resize(b[V_K]);
            dcopy.resize(b[V_DC]);
            dcopy_src.resize(b[V_DC]);
            h_rg.resize_uninit(b[V_RG]);
            h_ra.resize_uninit(b[V_RG]);
            h_cg.resize_uninit(b[V_CG]);
            h_cb.resize_uninit(b[V_CG]);
            h_ct0.resize_uninit(b[V_CG]);
            h_cvoff.resize_uninit(b[V_CG]);
            h_pair.resize_uninit(b[V_PAIR]);
        }
        t_resize += ms_since(tm0);
        // the TRSM items of a level chunk by chunk (each chunk's items of all
        // the level's supernode groups together), so that one launch covers
        // a chunk
        vector<std::array<i64, NCHM>> lfpos(NC), ufpos(NC);
        for (int L = 0; L < NL; ++L) {
            LevelRange &R = levels[L];
            i64 pl = base[first[L]][V_LF], pu = base[first[L]][V_UF];
            const i64 l0 = pl, u0 = pu;
            R.lf_o[0] = R.uf_o[0] = 0;
            for (int ch = 0; ch < NCHM; ++ch) {
                for (int t = first[L]; t < first[L + 1]; ++t) {
                    lfpos[t][ch] = pl;
                    ufpos[t][ch] = pu;
                    pl += outs[t].lf_c[ch].size();
                    pu += outs[t].uf_c[ch].size();
                }
                if (ch < R.nch) {
                    R.lf_o[ch + 1] = (int)(pl - l0);
                    R.uf_o[ch + 1] = (int)(pu - u0);
                } else {
                    SLU_REQUIRE(pl - l0 == R.lf_o[R.nch] && pu - u0 == R.uf_o[R.nch],
                                "level %d: TRSM items past the level's %d chunks", L, R.nch);
                }
            }
        }
        const auto tp0 = std::chrono::steady_clock::now();
        parallel_for(NC, [&](int c) {
            SchedOut &O = outs[c];
            const std::array<i64, V_N> &B = base[c];
            const i64 bc = B[V_CG], br = B[V_RG], bp = B[V_PAIR];
            for (auto &k : O.kinfos) {
                k.cvoff = shift(k.cvoff, bc);
                k.ct0 = shift(k.ct0, bc);
                k.cg = shift(k.cg, bc);
                k.cb = shift(k.cb, bc);
                k.rg = shift(k.rg, br);
                k.ra = shift(k.ra, br);
                k.pair = shift(k.pair, bp);
            }
            for (auto &v : O.uf_c)
                for (auto &t : v) {
                    t.voff = shift(t.voff, bc);
                    t.t0 = shift(t.t0, bc);
                }
            for (auto &t : O.tu_items) {
                t.voff = shift(t.voff, bc);
                t.t0 = shift(t.t0, bc);
            }
            auto put = [](auto &dst, const auto &src, i64 at) {
                std::copy(src.begin(), src.end(), dst.data() + at);
            };
            put(diag_items, O.diag_items, B[V_DIAG]);
            put(df_items, O.df_items, B[V_DF]);
            put(tl_items, O.tl_items, B[V_TL]);
            put(tu_items, O.tu_items, B[V_TU]);
            for (int ch = 0; ch < NCHM; ++ch) {
                put(lf_items, O.lf_c[ch], lfpos[c][ch]);
                put(uf_items, O.uf_c[ch], ufpos[c][ch]);
            }
            put(kinfos, O.kinfos, B[V_K]);
            for (size_t i = 0; i < O.khost.size(); ++i) khost[B[V_K] + i] = std::move(O.khost[i]);
            put(dcopy, O.dcopy, B[V_DC]);
            put(dcopy_src, O.dcopy_src, B[V_DC]);
            put(h_rg, O.h_rg, br);
            put(h_ra, O.h_ra, br);
            put(h_cg, O.h_cg, bc);
            put(h_cb, O.h_cb, bc);
            put(h_ct0, O.h_ct0, bc);
            put(h_cvoff, O.h_cvoff, bc);
            put(h_pair, O.h_pair, bp);
        }, 1);
        t_put += ms_since(tp0);
        vector<int> owner(lblk.size() + ublk.size(), -1), touched;
        for (int L = 0; L < NL; ++L) {
            const auto tt0 = std::chrono::steady_clock::now();
            LevelRange &R = levels[L];
            const std::array<i64, V_N> &B0 = base[first[L]], &B1 = base[first[L + 1]];
            R.diag_off = (int)B0[V_DIAG];
            R.tl_off = (int)B0[V_TL];
            R.tu_off = (int)B0[V_TU];
            R.k_off = (int)B0[V_K];
            R.tile_off = (int)tiles.size();
            R.big_off = (int)tiles_big.size();
            R.df_off = (int)B0[V_DF];
            R.lf_off = (int)B0[V_LF];
            R.uf_off = (int)B0[V_UF];
            R.dc_off = (int)B0[V_DC];
            for (int t = first[L]; t < first[L + 1]; ++t) {
                const SchedOut &O = outs[t];
                stats.panel_flops += O.panel_flops;
                stats.schur_flops += O.schur_flops;
                stats.schur_flops_padded += O.schur_flops_padded;
                stats.scatter_bytes += O.scatter_bytes;
                stats.n_diag += O.n_diag;
                stats.n_trsm_items += O.n_trsm_items;
                stats.n_schur_tiles += O.n_schur_tiles;
                R.schur_flops += O.R_schur_flops;
                R.big_flops += O.R_big_flops;
                R.big = R.big || O.R_big;
            }
            // critical tiles first: they are launched ahead of the rest so the
            // next level's panels can be factored while the rest runs
            // (chunk by chunk within each class: prefix offsets bc_o / br_o,
            // sc_o / sr_o relative to the class's first tile)
            for (int cls = 0; cls < 2; ++cls) {
                const int b0 = (int)tiles_big.size(), s0 = (int)tiles.size();
                int *bo = cls ? R.br_o : R.bc_o, *so = cls ? R.sr_o : R.sc_o;
                bo[0] = so[0] = 0;
                for (int ch = 0; ch < NCHM; ++ch) {
                    for (int t = first[L]; t < first[L + 1]; ++t) {
                        const int kb = (int)(base[t][V_K] - R.k_off);
                        for (TileItem x : outs[t].big[cls][ch]) {
                            x.kslot += kb;
                            tiles_big.push_back(x);
                        }
                        for (TileItem x : outs[t].small[cls][ch]) {
                            x.kslot += kb;
                            tiles.push_back(x);
                        }
                    }
                    if (ch < R.nch) {
                        bo[ch + 1] = (int)tiles_big.size() - b0;
                        so[ch + 1] = (int)tiles.size() - s0;
                    } else {
                        SLU_REQUIRE((int)tiles_big.size() - b0 == bo[R.nch] && (int)tiles.size() - s0 == so[R.nch],
                                    "level %d: Schur tiles past the level's %d chunks", L, R.nch);
                    }
                }
                if (cls == 0) {
                    R.bigc_n = bo[R.nch];
                    R.tilec_n = so[R.nch];
                }
            }
            R.big_n = (int)tiles_big.size() - R.big_off;
            R.df_n = (int)(B1[V_DF] - B0[V_DF]);
            for (int i = R.df_off; i < R.df_off + R.df_n; ++i) R.df_maxw = std::max(R.df_maxw, df_items[i].w);
            R.lf_n = (int)(B1[V_LF] - B0[V_LF]);
            R.uf_n = (int)(B1[V_UF] - B0[V_UF]);
            for (int i = R.lf_off; i < R.lf_off + R.lf_n; ++i) R.tf_maxw = std::max(R.tf_maxw, lf_items[i].w);
            for (int i = R.uf_off; i < R.uf_off + R.uf_n; ++i) R.tf_maxw = std::max(R.tf_maxw, uf_items[i].w);
            R.diag_n = (int)(B1[V_DIAG] - B0[V_DIAG]);
            R.tl_n = (int)(B1[V_TL] - B0[V_TL]);
            R.tu_n = (int)(B1[V_TU] - B0[V_TU]);
            R.k_n = (int)(B1[V_K] - B0[V_K]);
            R.tile_n = (int)tiles.size() - R.tile_off;
            R.dc_n = (int)(B1[V_DC] - B0[V_DC]);
            t_tiles += ms_since(tt0);
            // conflicting destinations inside the level -> atomics
            touched.clear();
            for (int s = R.k_off; s < R.k_off + R.k_n; ++s) {
                KInfoHost &kh = khost[s];
                for (int h : kh.dests) {
                    int key = h >= 0 ? h : (int)lblk.size() + ~h;
                    if (owner[key] == -1) {
                        owner[key] = s;
                        touched.push_back(key);
                    } else if (owner[key] != s) {
                        kinfos[owner[key]].atomic = 1;
                        kinfos[s].atomic = 1;
                    }
                }
            }
            for (int key : touched) owner[key] = -1;
            for (int i = R.big_off; i < R.big_off + R.big_n; ++i)
                R.atomic_tiles += kinfos[R.k_off + tiles_big[i].kslot].atomic;
            for (int i = R.tile_off; i < R.tile_off + R.tile_n; ++i)
                R.atomic_tiles += kinfos[R.k_off + tiles[i].kslot].atomic;
        }
        t_merge += ms_since(tm0);
        khost.clear();
    }

    void add_supernode(int k, SchedOut &O) const {
        const int w = W(k);
        const int ljb = k / Pc, lb = k / Pr;
        const bool lcol_here = (k % Pc) == mycol && lidx[k];
        const bool urow_here = (k % Pr) == myrow && uidx[k];
        const bool diag_here = lcol_here && (k % Pr) == myrow;
        const bool fast = fast_w(w);
        const int nbk = (w + PW - 1) / PW;
        constexpr int RB = cplx ? RBOf<T>::v : 16 * TR_WAVES;
        // ---- diagonal block: factored in place by its owner; other ranks of
        // its process row / column read the broadcast package
        T *dT = nullptr, *dinv = nullptr;
        int dld = 0;
        if (diag_here) {
            SLU_REQUIRE(lblk_ib[lcol_first[ljb]] == k, "diagonal block of %d is not first", k);
            dT = d_L.p + lval_off[ljb];
            dld = lval_ld[ljb];
            dinv = xmode ? d_dpk.p + pkg[k] + (i64)w * w : d_dinv.p + dscr[k];
        } else if (pkg[k] >= 0) {
            dT = d_dpk.p + pkg[k];
            dld = w;
            dinv = dT + (i64)w * w;
        }
        if (diag_here) {
            if (fast) {
                DiagItemF<T> d{};
                d.a = dT;
                d.dinv = dinv;
                d.ld = dld;
                d.w = w;
                d.k = k;
                d.fcol = (int)xsup[k];
                O.df_items.push_back(d);
            } else {
                DiagItem<T> d{};
                d.a = dT;
                d.ld = dld;
                d.w = w;
                d.k = k;
                d.fcol = (int)xsup[k];
                O.diag_items.push_back(d);
            }
            if (xmode) add_copy(O.dcopy, O.dcopy_src, 0, lval_off[ljb], dld, 0, pkg[k], w, w, w);
            O.n_diag++;
            // SRC/pdgstrf2.c:252,262 (complex weights SRC/pzgstrf2.c:253,263)
            double wd = w, s1 = wd * (wd - 1) / 2, s2 = (wd - 1) * wd * (2 * wd - 1) / 6;
            O.panel_flops += cplx ? 6 * s1 + 10 * wd + 8 * s2 : s1 + 2 * s2;
        }
        // ---- L panel TRSM (rows of column k below the diagonal block)
        int m = 0, r0 = 0;
        lrows(k, m, r0);
        if (lcol_here && m > 0) {
            SLU_REQUIRE(dT, "no diagonal block for the L panel of %d", k);
            if (fast) {
                for (int c0 = 0; c0 < m; c0 += RB) {
                    TrsmItemF<T> t{};
                    t.x = d_L.p + lval_off[ljb] + r0 + c0;
                    t.t = dT;
                    t.dinv = dinv;
                    t.ldx = lval_ld[ljb];
                    t.ldt = dld;
                    t.w = w;
                    t.nrows = std::min(RB, m - c0);
                    O.lf_c[xmode ? c0 / lgsz[k] : 0].push_back(t); // (RB divides the group size)
                    O.n_trsm_items++;
                }
            } else {
                for (int c0 = 0; c0 < m; c0 += TRSM_THREADS) {
                    TrsmLItem<T> t{};
                    t.x = d_L.p + lval_off[ljb] + r0 + c0;
                    t.u = dT;
                    t.ldx = lval_ld[ljb];
                    t.ldu = dld;
                    t.w = w;
                    t.nrows = std::min(TRSM_THREADS, m - c0);
                    O.tl_items.push_back(t);
                    O.n_trsm_items++;
                }
            }
            O.panel_flops += (cplx ? 4.0 : 1.0) * (double)w * (w + 1) * m;
        }
        // ---- U panel: nonempty columns of block row k on my process column
        vector<int> ujb; // U blocks with a nonempty column
        int ncols = 0, kmin = w;
        const int cols_off = (int)O.h_cg.size();
        if (uidx[k]) {
            const int_t *ix = uidx[k];
            const i64 klst = xsup[k + 1];
            const i64 base = urow_here ? uval_off[lb] : upos[k];
            i64 p = SLU_BR_HEADER, run = 0;
            for (i64 b = 0; b < ix[0]; ++b) {
                const int jb = (int)ix[p];
                const int bidx = (int)ujb.size();
                bool any = false;
                for (int c = 0; c < W(jb); ++c) {
                    const i64 fst = ix[p + SLU_UB_DESCRIPTOR + c];
                    if (fst >= klst) continue;
                    any = true;
                    O.h_cg.push_back((int)xsup[jb] + c);
                    O.h_cb.push_back(bidx);
                    if (xmode && !urow_here) { // received in column groups (layout_values)
                        const int g = ncols / ucsz[k];
                        O.h_cvoff.push_back(ugpos[k][g] + run - ugrun[k][g]);
                    } else {
                        O.h_cvoff.push_back(base + run);
                    }
                    const int t0 = (int)(fst - xsup[k]);
                    O.h_ct0.push_back(t0);
                    kmin = std::min(kmin, t0);
                    ++ncols;
                    run += klst - fst;
                    if (urow_here) {
                        double seg = (double)(klst - fst);
                        O.panel_flops += seg * (seg + 1);
                    }
                }
                if (any) ujb.push_back(jb);
                p += SLU_UB_DESCRIPTOR + W(jb);
            }
            SLU_REQUIRE(run == ix[1], "U row %d: segment lengths %lld != %lld", k, (long long)run,
                        (long long)ix[1]);
        }
        if (urow_here && ncols > 0) {
            SLU_REQUIRE(dT, "no diagonal block for the U panel of %d", k);
            for (int c0 = 0; fast && c0 < ncols; c0 += RB) {
                TrsmItemF<T> t{};
                t.x = d_U.p;
                t.voff = (const i64 *)(intptr_t)(cols_off + c0); // relocated
                t.t0 = (const int *)(intptr_t)(cols_off + c0);
                t.t = dT;
                t.dinv = dinv + (i64)nbk * PW * PW;
                t.ldt = dld;
                t.w = w;
                t.nrows = std::min(RB, ncols - c0);
                O.uf_c[xmode ? c0 / ucsz[k] : 0].push_back(t);
                O.n_trsm_items++;
            }
            for (int c0 = 0; !fast && c0 < ncols; c0 += TRSM_THREADS) {
                TrsmUItem<T> t{};
                t.l = dT;
                t.ubase = d_U.p;
                t.ldl = dld;
                t.w = w;
                t.ncols = std::min(TRSM_THREADS, ncols - c0);
                t.voff = (const i64 *)(intptr_t)(cols_off + c0); // relocated
                t.t0 = (const int *)(intptr_t)(cols_off + c0);
                int km = w;
                for (int c = 0; c < t.ncols; ++c) km = std::min(km, O.h_ct0[cols_off + c0 + c]);
                t.kmin = km;
                O.tu_items.push_back(t);
                O.n_trsm_items++;
            }
        }
        if (m == 0 || ncols == 0) return; // nothing to update from k here
        // ---- Schur update of k on this rank's destinations
        KInfo<T> ki{};
        if (!lcol_here) SLU_REQUIRE(lpos[k] >= 0, "L panel %d not received", k);
        SLU_REQUIRE(urow_here || upos[k] >= 0, "U panel %d not received", k);
        ki.ubase = urow_here ? d_U.p : d_pan.p;
        ki.n = ncols;
        ki.kmin = kmin;
        ki.kw = w - kmin;
        ki.nub = (int)ujb.size();
        ki.cvoff = (const i64 *)(intptr_t)cols_off;
        ki.ct0 = (const int *)(intptr_t)cols_off;
        ki.cg = (const int *)(intptr_t)cols_off;
        ki.cb = (const int *)(intptr_t)cols_off;
        const int rows_off = (int)O.h_rg.size();
        vector<int> lib_; // L blocks (ib) of the panel below the diagonal
        {
            const int_t *ix = lidx[k];
            i64 p = SLU_BC_HEADER;
            for (i64 b = 0; b < ix[0]; ++b) {
                const int gb = (int)ix[p], nr = (int)ix[p + 1];
                if (gb != k) {
                    const int a = (int)lib_.size();
                    lib_.push_back(gb);
                    for (int i = 0; i < nr; ++i) {
                        O.h_rg.push_back((int)ix[p + 2 + i]);
                        O.h_ra.push_back(a);
                    }
                }
                p += SLU_LB_DESCRIPTOR + nr;
            }
        }
        const int pair_off = (int)O.h_pair.size();
        KInfoHost kh;
        for (int ib : lib_)
            for (int jb : ujb) {
                int h = ib >= jb ? find_lblk(ib, jb) : ~find_ublk(ib, jb);
                O.h_pair.push_back(h);
                kh.dests.push_back(h);
            }
        ki.pair = (const int *)(intptr_t)pair_off;
        ki.atomic = 0;
        constexpr int BBN = BigCfg<T>::BN; // 128 (d, s) or 64 (z) columns per big tile
        const bool big = m >= SB_BM && ncols >= BBN;
        const int BM = big ? SB_BM : SC_BM, BN = big ? BBN : SC_BN;
        const int tm = (m + BM - 1) / BM, tn = (ncols + BN - 1) / BN;
        // K split near the root: a level of one or two supernodes whose
        // update is a few 128 x 128 tiles leaves most CUs idle for a whole
        // tile's latency (K up to 256: ~90 us).  Its K range is cut into
        // chunks of >= 64, one KInfo per chunk (same tables, kmin / kw
        // moved); the chunks' tiles add into the same destinations, which
        // the level's conflict analysis below turns into atomic scatters.
        int nsplit = 1;
        if (ksplit_tiles > 0 && big && bylev[level_of[k]].size() <= 2 && tm * tn < ksplit_tiles)
            nsplit = std::max(1, std::min({4, (w - kmin) / 64, ksplit_tiles / (tm * tn)}));
        const int kch = ((w - kmin + nsplit - 1) / nsplit + 15) / 16 * 16;
        // A destination (ib,jb) belongs to the panel of supernode min(ib,jb);
        // it is critical when that panel is factored at the next level.  All
        // destinations in a row of L block ib (resp. a column of U block jb)
        // with level(ib) == level(k)+1 are critical, and no others.
        const int nl = level_of[k] + 1;
        vector<char> ccol(tn, 0);
        for (int c = 0; c < ncols; ++c)
            if (level_of[ujb[O.h_cb[cols_off + c]]] == nl) ccol[c / BN] = 1;
        // 2D grids: one KInfo per row group of the L panel (its own rows,
        // base and leading dimension: a received group is column-major with
        // ld = its rows), the tiles of a group in the exchange chunk of their
        // rows and columns
        const int gs = xmode ? lgsz[k] : m, ng = xmode ? ngroups(m, gs) : 1;
        for (int g = 0; g < ng; ++g) {
            const int ga = g * gs, rows = std::min(gs, m - ga);
            KInfo<T> kg = ki;
            if (lcol_here) {
                kg.a = d_L.p + lval_off[ljb] + r0 + ga;
                kg.lda = lval_ld[ljb];
            } else if (xmode) {
                SLU_REQUIRE(lgpos[k][g] >= 0, "L panel %d row group %d not received", k, g);
                kg.a = d_pan.p + lgpos[k][g];
                kg.lda = rows;
            } else {
                kg.a = d_pan.p + lpos[k];
                kg.lda = m;
            }
            kg.m = rows;
            kg.rg = (const int *)(intptr_t)(rows_off + ga);
            kg.ra = (const int *)(intptr_t)(rows_off + ga);
            const int tmg = (rows + BM - 1) / BM;
            vector<char> crow(tmg, 0);
            for (int r = 0; r < rows; ++r)
                if (level_of[lib_[O.h_ra[rows_off + ga + r]]] == nl) crow[r / BM] = 1;
            const int slot0 = (int)O.kinfos.size(); // relocated by the merge
            int ns = nsplit;
            for (int c = 0; c < ns; ++c) {
                KInfo<T> kc = kg;
                kc.kmin = kmin + c * kch;
                kc.kw = std::min(kch, w - kc.kmin);
                if (kc.kw <= 0) {
                    ns = c;
                    break;
                }
                O.kinfos.push_back(kc);
                O.khost.push_back(kh);
            }
            for (int c = 0; c < ns; ++c)
                for (int i = 0; i < tmg; ++i)
                    for (int j = 0; j < tn; ++j) {
                        const int cls = (crow[i] || ccol[j]) ? 0 : 1;
                        const int ch = xmode ? std::max(g, j * BN / ucsz[k]) : 0;
                        (big ? O.big[cls][ch] : O.small[cls][ch]).push_back(TileItem{slot0 + c, i, j});
                    }
        }
        // algorithmic work: exact unpadded flops and padded flops
        double fl = 0;
        for (int c = 0; c < ncols; ++c) fl += 2.0 * m * (w - O.h_ct0[cols_off + c]);
        const double mult = cplx ? 4.0 : 1.0; // complex: 8 real flops per multiply-add
        O.schur_flops += fl * mult;
        O.schur_flops_padded += 2.0 * m * ncols * (double)(w - kmin) * mult;
        O.scatter_bytes += 3.0 * sizeof(T) * (double)m * ncols;
        O.n_schur_tiles += (i64)tm * tn;
        O.R_schur_flops += fl * mult;
        if (big) O.R_big_flops += fl * mult;
        if (w >= 64 && m >= 256 && ncols >= 256) O.R_big = true;
    }

    // ------------------------------------------------------- device
    void build_device() {
        const auto tb0 = std::chrono::steady_clock::now();
        auto sub = [&](const char *what, double mb) {
            if (prof) fprintf(stderr, "[slu plan %d]   build_device %-10s %6.1f ms %8.1f MB\n", iam, what, ms_since(tb0), mb);
        };
        d_rg.upload(h_rg);
        d_ra.upload(h_ra);
        d_cg.upload(h_cg);
        d_cb.upload(h_cb);
        d_pair.upload(h_pair);
        {
            // destinations resolved once (DRec, kernels.h): the Schur
            // epilogue reads one record per (L block, U block) of a tile
            RawVec<DRec> prec;
            prec.resize_uninit(h_pair.size());
            parallel_for((int)((h_pair.size() + 4095) / 4096), [&](int ch) {
                const size_t e = std::min(h_pair.size(), (size_t)(ch + 1) * 4096);
                for (size_t i = (size_t)ch * 4096; i < e; ++i) {
                    const int h = h_pair[i];
                    DRec d{0, 0, -1, 0};
                    if (h >= 0) {
                        const LBlk &L = lblk[h];
                        d.base = L.colvoff - (i64)L.fcol * L.ld;
                        d.mb = L.mapoff - L.frow;
                        d.ld = L.ld;
                    } else {
                        const UBlk &U = ublk[~h];
                        d.base = U.coloff - U.fcol;
                    }
                    prec[i] = d;
                }
            });
            d_prec.upload(prec);
        }
        d_ct0.upload(h_ct0);
        d_cvoff.upload(h_cvoff);
        sub("panels", (d_rg.bytes() + d_ra.bytes() + d_cg.bytes() + d_cb.bytes() + d_pair.bytes() + d_prec.bytes() +
                       d_ct0.bytes() + d_cvoff.bytes()) / 1e6);
        for (auto &t : tu_items) {
            intptr_t co = (intptr_t)t.voff;
            t.voff = d_cvoff.p + co;
            t.t0 = d_ct0.p + co;
        }
        for (auto &k : kinfos) {
            intptr_t co = (intptr_t)k.cvoff, ro = (intptr_t)k.rg, po = (intptr_t)k.pair;
            k.cvoff = d_cvoff.p + co;
            k.ct0 = d_ct0.p + co;
            k.cg = d_cg.p + co;
            k.cb = d_cb.p + co;
            k.rg = d_rg.p + ro;
            k.ra = d_ra.p + ro;
            k.pair = d_pair.p + po;
            k.prec = d_prec.p + po;
        }
        for (auto &t : uf_items) {
            intptr_t co = (intptr_t)t.voff;
            t.voff = d_cvoff.p + co;
            t.t0 = d_ct0.p + co;
        }
        auto reloc = [&](vector<CopyItem<T>> &v, const vector<char> &tag) {
            for (size_t i = 0; i < v.size(); ++i) {
                const int ss = tag[i] & 1, ds = tag[i] >> 1;
                v[i].src = (ss ? d_U.p : d_L.p) + (intptr_t)v[i].src;
                v[i].dst = (ds ? d_pan.p : d_dpk.p) + (intptr_t)v[i].dst;
            }
        };
        reloc(dcopy, dcopy_src);
        reloc(pcopy, pcopy_src);
        d_df.upload(df_items);
        d_lf.upload(lf_items);
        d_uf.upload(uf_items);
        d_diag.upload(diag_items);
        d_tl.upload(tl_items);
        d_tu.upload(tu_items);
        d_kinfo.upload(kinfos);
        d_tiles.upload(tiles);
        d_tiles_big.upload(tiles_big);
        d_dcopy.upload(dcopy);
        d_pcopy.upload(pcopy);
        sub("items", (d_df.bytes() + d_lf.bytes() + d_uf.bytes() + d_kinfo.bytes() + d_tiles.bytes() +
                      d_tiles_big.bytes()) / 1e6);
        d_lblk.upload(lblk);
        d_lmap.upload(lmap);
        d_ublk.upload(ublk);
        d_ucol_voff.upload(ucol_voff);
        d_ucol_fst.upload(ucol_fst);
        sub("blocks", (d_lblk.bytes() + d_lmap.bytes() + d_ublk.bytes() + d_ucol_voff.bytes() + d_ucol_fst.bytes()) / 1e6);
        d_counters.alloc(4);
        d_zpiv.alloc(nsupers);
        d_dsflags.alloc(std::max<size_t>(df_items.size(), 1) * DS_NFLAGS);
        HIPCHK(hipMemset(d_dsflags.p, 0, d_dsflags.bytes()));
        ev_pan.resize(levels.size());
        ev_rest.resize(levels.size());
        for (size_t L = 0; L < levels.size(); ++L) {
            HIPCHK(hipEventCreateWithFlags(&ev_pan[L], hipEventDisableTiming));
            HIPCHK(hipEventCreateWithFlags(&ev_rest[L], hipEventDisableTiming));
        }
        HIPCHK(hipEventCreateWithFlags(&ev_start, hipEventDisableTiming));
        HIPCHK(hipEventCreateWithFlags(&ev_pend, hipEventDisableTiming));
        HIPCHK(hipEventCreateWithFlags(&ev_tu0, hipEventDisableTiming));
        HIPCHK(hipEventCreateWithFlags(&ev_tu1, hipEventDisableTiming));
        if (xmode) {
            HIPCHK(hipEventCreateWithFlags(&ev_pk, hipEventDisableTiming));
            HIPCHK(hipEventCreateWithFlags(&ev_dx, hipEventDisableTiming));
            for (hipEvent_t &e : ev_cx) HIPCHK(hipEventCreateWithFlags(&e, hipEventDisableTiming));
        }
        d_info.alloc(Pr * Pc);
        stats.lu_bytes = (double)(lval_total + uval_total) * sizeof(T);
        stats.index_bytes = (double)(d_lblk.bytes() + d_lmap.bytes() + d_ublk.bytes() +
                                     d_ucol_voff.bytes() + d_ucol_fst.bytes() + d_diag.bytes() +
                                     d_tl.bytes() + d_tu.bytes() + d_kinfo.bytes() + d_tiles_big.bytes() +
                                     d_df.bytes() + d_lf.bytes() + d_uf.bytes() + d_dinv.bytes() +
                                     d_tiles.bytes() + d_rg.bytes() + d_ra.bytes() +
                                     d_cg.bytes() + d_cb.bytes() + d_pair.bytes() + d_prec.bytes() +
                                     d_ct0.bytes() + d_cvoff.bytes() + d_dcopy.bytes() +
                                     d_pcopy.bytes());
        double zvol = 0; // 3D: the ancestor reductions this layer takes part in
        if (zmode)
            for (int p = 0; p <= std::min(my_last, maxlvl - 2); ++p) zvol += (double)zr_cnt[p] * sizeof(T);
        stats.comm_bytes = (double)comm_volume * sizeof(T) + zvol;
        stats.comm_buf_bytes = (double)(dpk_total + pan_total) * sizeof(T) + (double)d_zbuf.bytes();
        // the tables went up by pageable hipMemcpy on the null stream; the
        // plan's streams are non-blocking, so make sure every copy has landed
        HIPCHK(hipDeviceSynchronize());
    }

    // ------------------------------------------------------- values
    // What the device factor storage holds: 0 nothing, 1 values
    // of A not yet factored (upload / restore / fill_a), 2 factors of them.
    // d_acur = the values of A behind the storage (fill_a only; an upload
    // does not tell which A it came from), a_fact = d_acur of the factors.
    int vstate = 0;
    const T *a_fact = nullptr, *snap_acur = nullptr;
    int snap_state = 0;

    // ---- host <-> HBM copies of the values (hostio.h)
    std::thread up_thread, pin_thread;
    std::string up_err, pin_err; // one per helper thread (no shared writes)
    double up_ms = 0;
    bool host_current = false; // the host LUstruct holds what the device holds

    vector<Xfer> value_xfers() {
        LocalLU *Llu = LU->Llu;
        vector<Xfer> xs;
        if (l_contig && lval_total)
            xs.push_back({(char *)d_L.p, (char *)Llu->Lnzval_bc_dat, lval_total * sizeof(T)});
        else
            for (int ljb = 0; ljb < nlc; ++ljb)
                if (lval_off[ljb] >= 0)
                    xs.push_back({(char *)(d_L.p + lval_off[ljb]), (char *)Llu->Lnzval_bc_ptr[ljb],
                                  (size_t)lval_ld[ljb] * W(ljb * Pc + mycol) * sizeof(T)});
        if (u_contig && uval_total)
            xs.push_back({(char *)d_U.p, (char *)Llu->Unzval_br_dat, uval_total * sizeof(T)});
        else
            for (int lb = 0; lb < nlr; ++lb)
                if (uval_off[lb] >= 0)
                    xs.push_back({(char *)(d_U.p + uval_off[lb]), (char *)Llu->Unzval_br_ptr[lb],
                                  (size_t)Llu->Ufstnz_br_ptr[lb][1] * sizeof(T)});
        return merge_xfers(std::move(xs));
    }

    void upload_values() {
        const auto t0 = std::chrono::steady_clock::now();
        vector<Xfer> xs = value_xfers();
        staged_h2d(xs, comm ? comm->device : 0);
        double b = 0;
        for (auto &x : xs) b += (double)x.bytes;
        stats.h2d_bytes = b;
        up_ms = ms_since(t0);
    }

    void upload() override {
        const auto t0 = std::chrono::steady_clock::now();
        if (pin_thread.joinable()) pin_thread.join();
        if (!pin_err.empty()) {
            if (up_thread.joinable()) up_thread.join();
            std::string e;
            e.swap(pin_err);
            throw Error(e);
        }
        if (up_thread.joinable()) {
            up_thread.join();
            if (!up_err.empty()) {
                std::string e;
                e.swap(up_err);
                throw Error(e);
            }
            stats.t_upload_wait_ms = ms_since(t0);
        } else {
            upload_values();
            stats.t_upload_wait_ms = ms_since(t0);
        }
        stats.t_upload_ms = up_ms;
        vstate = 1;
        d_acur = nullptr;
        host_current = true;
    }

    // D2H of the factors while the factorization runs (opts.overlap_download).
    // After the panels of level L are done, the L columns and U rows of its
    // supernodes are final (right-looking LU; later levels only read them).
    // Measured on the box (profiles/r02_pcie_micro.json): pageable D2H needs
    // copies of >= 4 MB to reach 49 GB/s (512 KB: 12 GB/s), while GPU stores
    // into pinned host memory reach 51-56 GB/s with 32-128 workgroups and
    // pinned -> pageable memcpy 60 / 121 GB/s on 4 / 8 host threads.  So the
    // finished blocks are pushed by a small kernel (k_push) into a pinned
    // slot of <= SLOT bytes ("fill"), and host threads scatter the slot into
    // the caller's arrays while the next fill is pushed.
    // slot / minimum fill (SLU_D2H_SLOT_KB overrides the slot: tests use tiny
    // slots so that blocks split across fills)
    i64 D2H_SLOT = 128ll << 20, D2H_MIN = 32ll << 20;
    static constexpr i64 D2H_PIECE = 1ll << 20;
    static constexpr int D2H_NS = 4; // pinned slots in flight
    struct D2HFill {
        int level;        // all blocks final after ev_pan[level]
        int seg_off, seg_n; // PushSeg range
        int hs_off, hs_n; // HostSeg range
        i64 bytes;
    };
    struct HostSeg {
        char *host;
        i64 off, bytes; // in the slot
    };
    vector<D2HFill> d2h_fills;
    // called on the D2H stream before fill F's push, after its level's
    // panels are done (AmalgPlan: compress the level into the caller's layout)
    std::function<void(int, hipStream_t)> d2h_pre;
    vector<PushSeg> h_push;
    vector<HostSeg> h_unpack;
    DevBuf<PushSeg> d_push;
    DevBuf<char> d_stage; // HBM staging slots of the D2H (SDMA mode)

    void build_d2h() {
        if (!opts.overlap_download) return;
        LocalLU *Llu = LU->Llu;
        i64 fb = 0; // bytes in the open fill
        int seg0 = 0, hs0 = 0;
        auto close = [&](int L) {
            if (fb == 0) return;
            d2h_fills.push_back({L, seg0, (int)h_push.size() - seg0, hs0, (int)h_unpack.size() - hs0, fb});
            seg0 = (int)h_push.size();
            hs0 = (int)h_unpack.size();
            fb = 0;
        };
        auto add = [&](const char *dev, char *host, i64 bytes, int L) {
            i64 done = 0;
            while (done < bytes) {
                const i64 take = std::min(bytes - done, D2H_SLOT - fb);
                for (i64 o = 0; o < take; o += D2H_PIECE)
                    h_push.push_back({dev + done + o, fb + o, (int)std::min(D2H_PIECE, take - o)});
                // host pieces of <= 4 MB so the unpack threads balance
                for (i64 o = 0; o < take; o += 4 * D2H_PIECE)
                    h_unpack.push_back({host + done + o, fb + o, std::min(4 * D2H_PIECE, take - o)});
                fb += (take + 15) & ~(i64)15; // 16-byte aligned slot offsets
                done += take;
                if (fb >= D2H_SLOT) close(L);
            }
        };
        for (size_t L = 0; L < levels.size(); ++L) {
            for (int k : bylev[L]) {
                if (k % Pc == mycol && lval_off[k / Pc] >= 0) {
                    const int ljb = k / Pc;
                    add((const char *)(d_L.p + lval_off[ljb]), (char *)Llu->Lnzval_bc_ptr[ljb],
                        (i64)lval_ld[ljb] * W(k) * (i64)sizeof(T), (int)L);
                }
                if (k % Pr == myrow && uval_off[k / Pr] >= 0) {
                    const int lb = k / Pr;
                    add((const char *)(d_U.p + uval_off[lb]), (char *)Llu->Unzval_br_ptr[lb],
                        (i64)Llu->Ufstnz_br_ptr[lb][1] * (i64)sizeof(T), (int)L);
                }
            }
            if (fb >= D2H_MIN || L + 1 == levels.size()) close((int)L);
        }
        d_push.upload(h_push.empty() ? vector<PushSeg>(1) : h_push);
    }

    // The D2H pipeline (runs on a helper thread during factor()): this
    // thread queues k_push of fill j into slot j % NS as soon as the slot's
    // previous fill has been scattered; an unpack thread scatters fill j once
    // its push event has fired (parallel host memcpy).
    void run_d2h(double &bytes, int64_t &ncopies) {
        double t_wait_push = 0, t_unpack = 0, t_wait_slot = 0;
        HIPCHK(hipSetDevice(comm ? comm->device : 0));
        constexpr int NS = D2H_NS;
        std::lock_guard<std::mutex> in_use(pinned_pool(1).use);
        std::vector<char *> slot = pinned_pool(1).get(NS, D2H_SLOT);
        hipStream_t cs = nullptr;
        hipEvent_t evf[NS] = {};
        std::mutex mu;
        std::condition_variable cv;
        int pushed = 0, unpacked = 0;
        bool fail = false;
        std::string err;
        auto set_err = [&](const char *what) {
            std::lock_guard<std::mutex> lk(mu);
            if (err.empty()) err = what;
            fail = true;
            cv.notify_all();
        };
        const int nf = (int)d2h_fills.size();
        std::thread unpacker;
        try {
            int prio_lo = 0, prio_hi = 0;
            HIPCHK(hipDeviceGetStreamPriorityRange(&prio_lo, &prio_hi));
            const char *pe = getenv("SLU_D2H_PRIO"); // diagnostics: lo | hi
            HIPCHK(hipStreamCreateWithPriority(&cs, hipStreamNonBlocking,
                                               pe && !strcmp(pe, "hi") ? prio_hi : prio_lo));
            const char *ge = getenv("SLU_D2H_WG");
            const int nwg = ge ? std::max(1, atoi(ge)) : 128; // (32: +25 ms of tail at 100^3, tools/d2h_variants.py)
            const char *me = getenv("SLU_D2H_MODE"); // diagnostics: push (zero-copy) | sdma
            const bool use_sdma = !(me && !strcmp(me, "push"));
            if (use_sdma && d_stage.n < (size_t)NS * D2H_SLOT) d_stage.alloc((size_t)NS * D2H_SLOT);
            for (auto &e : evf) HIPCHK(hipEventCreateWithFlags(&e, hipEventDisableTiming));
            unpacker = std::thread([&] {
                try {
                    HIPCHK(hipSetDevice(comm ? comm->device : 0));
                    for (int j = 0; j < nf; ++j) {
                        {
                            std::unique_lock<std::mutex> lk(mu);
                            cv.wait(lk, [&] { return pushed > j || fail; });
                            if (fail) return;
                        }
                        const auto tw = std::chrono::steady_clock::now();
                        HIPCHK(hipEventSynchronize(evf[j % NS]));
                        const auto tu = std::chrono::steady_clock::now();
                        t_wait_push += std::chrono::duration<double, std::milli>(tu - tw).count();
                        const D2HFill &F = d2h_fills[j];
                        const char *src = slot[j % NS];
                        parallel_for(F.hs_n, [&](int i) {
                            const HostSeg &h = h_unpack[F.hs_off + i];
                            memcpy(h.host, src + h.off, (size_t)h.bytes);
                        }, 1);
                        t_unpack += ms_since(tu);
                        for (int i = 0; i < F.hs_n; ++i) bytes += (double)h_unpack[F.hs_off + i].bytes;
                        ncopies += F.hs_n;
                        std::lock_guard<std::mutex> lk(mu);
                        unpacked = j + 1;
                        cv.notify_all();
                    }
                } catch (const std::exception &e) {
                    set_err(e.what());
                }
            });
            for (int j = 0; j < nf; ++j) {
                {
                    const auto tw = std::chrono::steady_clock::now();
                    std::unique_lock<std::mutex> lk(mu);
                    cv.wait(lk, [&] { return unpacked >= j - NS + 1 || fail; });
                    t_wait_slot += ms_since(tw);
                    if (fail) break;
                }
                const D2HFill &F = d2h_fills[j];
                HIPCHK(hipStreamWaitEvent(cs, ev_pan[F.level], 0));
                if (d2h_pre) d2h_pre(F.level, cs); // (amalgamated plan: relayout of the levels)
                if (use_sdma) {
                    // gather into an HBM slot (HBM-bound, microseconds), then
                    // one DMA-engine copy to the pinned slot: the PCIe-bound
                    // part occupies no CU while the factorization runs
                    char *ds = d_stage.p + (size_t)(j % NS) * D2H_SLOT;
                    hipLaunchKernelGGL(k_push, dim3(std::min(F.seg_n, 4 * nwg)), dim3(256), 0, cs,
                                       (const PushSeg *)(d_push.p + F.seg_off), F.seg_n, ds);
                    HIPCHK(hipGetLastError());
                    HIPCHK(hipMemcpyAsync(slot[j % NS], ds, (size_t)F.bytes, hipMemcpyDeviceToHost, cs));
                } else {
                    hipLaunchKernelGGL(k_push, dim3(std::min(F.seg_n, nwg)), dim3(256), 0, cs,
                                       (const PushSeg *)(d_push.p + F.seg_off), F.seg_n, slot[j % NS]);
                    HIPCHK(hipGetLastError());
                }
                HIPCHK(hipEventRecord(evf[j % NS], cs));
                std::lock_guard<std::mutex> lk(mu);
                pushed = j + 1;
                cv.notify_all();
            }
        } catch (const std::exception &e) {
            set_err(e.what());
        }
        if (unpacker.joinable()) unpacker.join();
        if (prof)
            fprintf(stderr, "[slu d2h %d] fills %d, unpack waits for push %.1f ms, unpack %.1f ms, "
                    "push waits for a slot %.1f ms\n", iam, nf, t_wait_push, t_unpack, t_wait_slot);
        if (cs) (void)hipStreamSynchronize(cs);
        for (auto &e : evf)
            if (e) (void)hipEventDestroy(e);
        if (cs) (void)hipStreamDestroy(cs);
        if (!err.empty()) throw Error(err);
    }

    DevBuf<T> d_L0, d_U0; // pristine copies (snapshot)
    void snapshot() override {
        d_L0.alloc(d_L.n);
        d_U0.alloc(d_U.n);
        HIPCHK(hipMemcpyAsync(d_L0.p, d_L.p, d_L.bytes(), hipMemcpyDeviceToDevice, stream));
        HIPCHK(hipMemcpyAsync(d_U0.p, d_U.p, d_U.bytes(), hipMemcpyDeviceToDevice, stream));
        HIPCHK(hipStreamSynchronize(stream));
        snap_state = vstate;
        snap_acur = d_acur;
    }
    void restore() override {
        SLU_REQUIRE(d_L0.p && d_U0.p, "restore without snapshot");
        vstate = snap_state;
        d_acur = snap_acur;
        host_current = false;
        HIPCHK(hipMemcpyAsync(d_L.p, d_L0.p, d_L.bytes(), hipMemcpyDeviceToDevice, stream));
        HIPCHK(hipMemcpyAsync(d_U.p, d_U0.p, d_U.bytes(), hipMemcpyDeviceToDevice, stream));
    }
    void set_timing(int timing, int serial) override {
        opts.timing = timing;
        opts.serial = serial;
    }
    void adopt_factors() override {
        upload();
        sync();
        vstate = 2;
    }
    void sync() override {
        HIPCHK(hipStreamSynchronize(pstream));
        HIPCHK(hipStreamSynchronize(stream));
    }

    void download() override {
        LocalLU *Llu = LU->Llu;
        sync();
        if (host_current) return; // overlap_download already wrote them back
        if (l_contig && lval_total) {
            HIPCHK(hipMemcpy(Llu->Lnzval_bc_dat, d_L.p, lval_total * sizeof(T), hipMemcpyDeviceToHost));
        } else {
            for (int ljb = 0; ljb < nlc; ++ljb)
                if (lval_off[ljb] >= 0)
                    HIPCHK(hipMemcpy(Llu->Lnzval_bc_ptr[ljb], d_L.p + lval_off[ljb],
                                     (size_t)lval_ld[ljb] * W(ljb * Pc + mycol) * sizeof(T),
                                     hipMemcpyDeviceToHost));
        }
        if (u_contig && uval_total) {
            HIPCHK(hipMemcpy(Llu->Unzval_br_dat, d_U.p, uval_total * sizeof(T), hipMemcpyDeviceToHost));
        } else {
            for (int lb = 0; lb < nlr; ++lb)
                if (uval_off[lb] >= 0)
                    HIPCHK(hipMemcpy(Llu->Unzval_br_ptr[lb], d_U.p + uval_off[lb],
                                     (size_t)Llu->Ufstnz_br_ptr[lb][1] * sizeof(T),
                                     hipMemcpyDeviceToHost));
        }
    }

    // SLU_KSPLIT_TILES: levels of <= 2 supernodes with fewer big tiles than
    // this split their K range (default 0, off: the chunks of a destination
    // add atomically in no fixed order, so the root levels' factors would not
    // be bit-reproducible from run to run, for ~0.3 ms at 100^3)
    int ksplit_tiles = getenv("SLU_KSPLIT_TILES") ? atoi(getenv("SLU_KSPLIT_TILES")) : 0;
    // SLU_TRSM_NARROW: 0 the 256-wide k_trsm_reg everywhere, 1 the 64-wide
    // instantiation for levels whose TRSM supernodes are <= 64 wide, 2 (default)
    // also the 128-wide one for <= 128
    int trsm_narrow = getenv("SLU_TRSM_NARROW") ? atoi(getenv("SLU_TRSM_NARROW")) : 2;
    // SLU_TRSM_2STREAM=1 (default): the U panel's TRSM on a stream of its
    // own beside the L panel's (both only wait for the diagonal block; near
    // the root each is a few slabs, latency-bound)
    int trsm_2stream = getenv("SLU_TRSM_2STREAM") ? atoi(getenv("SLU_TRSM_2STREAM")) : 1;
    // SLU_TRSM_PF=1 (default): k_trsm_reg's latency form (next block's T and
    // Dinv loaded during the current block, columns stored when final)
    int trsm_pf = getenv("SLU_TRSM_PF") ? atoi(getenv("SLU_TRSM_PF")) : 1;
    // the level's fast-path TRSM items, or (ch >= 0) those of exchange chunk ch
    void launch_trsm_fast(const LevelRange &R, hipStream_t st, int ch = -1) {
        const int lo = R.lf_off + (ch >= 0 ? R.lf_o[ch] : 0), ln = ch >= 0 ? R.lf_o[ch + 1] - R.lf_o[ch] : R.lf_n;
        const int uo = R.uf_off + (ch >= 0 ? R.uf_o[ch] : 0), un = ch >= 0 ? R.uf_o[ch + 1] - R.uf_o[ch] : R.uf_n;
        // the U launch on ustream when both panels have slabs
        const bool two = trsm_2stream && ustream && st == pstream && ln && un;
        hipStream_t su = two ? ustream : st;
        if (two) {
            HIPCHK(hipEventRecord(ev_tu0, st));
            HIPCHK(hipStreamWaitEvent(ustream, ev_tu0, 0));
        }
        auto go = [&](auto maxw, auto pf) {
            constexpr int MW = decltype(maxw)::value;
            constexpr bool P = decltype(pf)::value;
            if (ln) hipLaunchKernelGGL((k_trsm_reg<T, 0, MW, P>), dim3(ln), dim3(64 * TR_WAVES), 0, st, d_lf.p + lo);
            if (un) hipLaunchKernelGGL((k_trsm_reg<T, 1, MW, P>), dim3(un), dim3(64 * TR_WAVES), 0, su, d_uf.p + uo);
        };
        auto go_pf = [&](auto maxw) {
            if (trsm_pf) go(maxw, std::true_type{});
            else go(maxw, std::false_type{});
        };
        if constexpr (cplx) {
            if (ln) hipLaunchKernelGGL((k_trsm_blk<T, 0>), dim3(ln), dim3(256), 0, st, d_lf.p + lo);
            if (un) hipLaunchKernelGGL((k_trsm_blk<T, 1>), dim3(un), dim3(256), 0, su, d_uf.p + uo);
        } else if (R.tf_maxw <= 64 && trsm_narrow) {
            // narrow levels: the 64-wide instantiation (several workgroups per CU)
            go_pf(std::integral_constant<int, 64>{});
        } else if (R.tf_maxw <= 128 && trsm_narrow >= 2) {
            go_pf(std::integral_constant<int, 128>{});
        } else {
            go_pf(std::integral_constant<int, FAST_MAXW>{});
        }
        if (two) {
            HIPCHK(hipEventRecord(ev_tu1, ustream));
            HIPCHK(hipStreamWaitEvent(st, ev_tu1, 0));
        }
    }

    // The rest of a level's Schur tiles go out as two launches, the first
    // with rest_split %% of them (SLU_REST_SPLIT: A/B).  The
    // next level's diag LU and TRSM workgroups (150 / 85 KB of LDS, up to 256
    // VGPRs) fit only on a CU that no Schur workgroup holds; inside one
    // launch every freed slot is refilled with the next Schur tile, so they
    // would wait for the whole level.  Where the first launch drains they get
    // CUs and run beside the second (100^3: 363 -> 345 ms; more split points
    // gain nothing further, tools/ab_env.sh).
    int rest_split = getenv("SLU_REST_SPLIT") ? atoi(getenv("SLU_REST_SPLIT")) : 30;
    // k_diag_strips (diag_strips.h) for the levels near the root: a few wide
    // real blocks, each factored by one workgroup per 32-column strip
    // (SLU_DIAG_STRIPS=0: k_diag_lu_f everywhere; SLU_DIAG_STRIPS_MAX: the
    // most blocks a level may hold for it, default 32)
    // (SLU_DIAG_STRIPS=2, test hook: every fast level, narrow blocks too)
    int strips_mode = getenv("SLU_DIAG_STRIPS") ? atoi(getenv("SLU_DIAG_STRIPS")) : 1;
    int strips_max = getenv("SLU_DIAG_STRIPS_MAX") ? atoi(getenv("SLU_DIAG_STRIPS_MAX")) : 32;
    bool strips_ok(const LevelRange &R) const {
        if (cplx || strips_mode == 0) return false;
        return strips_mode == 2 || (R.df_maxw > DF_SMALLW && R.df_n <= strips_max);
    }
    // k_diag_lu_w (diag_wave.h): one wave per narrow diagonal block, real
    // types (SLU_DIAG_WAVE=0: k_diag_lu_f's 256-thread path instead)
    int diag_wave = getenv("SLU_DIAG_WAVE") ? atoi(getenv("SLU_DIAG_WAVE")) : 1;
    bool diag_wave_ok() const { return !cplx && diag_wave != 0; }
    void launch_diag_wave(const LevelRange &R, double thresh, hipStream_t st) {
        if constexpr (!cplx) {
            const dim3 g((unsigned)((R.df_n + DW_WAVES - 1) / DW_WAVES)), b(64 * DW_WAVES);
            if (R.df_maxw <= 32)
                hipLaunchKernelGGL((k_diag_lu_w<T, 32>), g, b, 0, st, d_df.p + R.df_off, R.df_n, thresh,
                                   opts.replace_tiny_pivot, d_counters.p, d_zpiv.p);
            else
                hipLaunchKernelGGL((k_diag_lu_w<T, 64>), g, b, 0, st, d_df.p + R.df_off, R.df_n, thresh,
                                   opts.replace_tiny_pivot, d_counters.p, d_zpiv.p);
        }
    }
    void launch_strips(const LevelRange &R, double thresh, hipStream_t st) {
        if constexpr (!cplx)
            hipLaunchKernelGGL(k_diag_strips<T>, dim3(ds_grid(R.df_n)), dim3(DS_THREADS), 0, st, d_df.p + R.df_off,
                               R.df_n, d_dsflags.p + (size_t)R.df_off * DS_NFLAGS, ds_epoch, d_counters.p + 1, thresh,
                               opts.replace_tiny_pivot, d_counters.p, d_zpiv.p);
    }
    void launch_big(const LevelRange &R, int off, int cnt, hipStream_t st) {
        hipLaunchKernelGGL(k_schur_big<T>, dim3(cnt), dim3(BigCfg<T>::THREADS), 0, st,
                           d_tiles_big.p + off, d_kinfo.p + R.k_off, d_L.p, d_U.p,
                           d_lblk.p, d_lmap.p, d_ublk.p, d_ucol_voff.p, d_ucol_fst.p);
    }
    void launch_small(const LevelRange &R, int off, int cnt, hipStream_t st) {
        hipLaunchKernelGGL(k_schur<T>, dim3(cnt), dim3(SC_THREADS), 0, st, d_tiles.p + off,
                           d_kinfo.p + R.k_off, d_L.p, d_U.p, d_lblk.p, d_lmap.p, d_ublk.p,
                           d_ucol_voff.p, d_ucol_fst.p);
    }

    void issue(const vector<Sec> &secs, int off, int n_, const char *phase, int level) {
        for (int i = off; i < off + n_; ++i) {
            const Sec &s = secs[i];
            T *base = s.arena ? d_pan.p : d_dpk.p;
            X.section(s.g, s.root, s.mask, s.off >= 0 ? base + s.off : nullptr,
                      (size_t)s.cnt * sizeof(T));
        }
        X.phase = phase;
        X.level = level;
        X.flush();
        X.phase = "plan-time exchange";
        X.level = -1;
    }

    // ------------------------------------------------------- factor
    void factor(double anorm, int *info, int *tiny) override {
        SLU_REQUIRE(vstate == 1, "factor: no unfactored values on the device (%s)",
                    vstate == 2 ? "already factored; upload / restore / fill_a first"
                                : "upload or fill_a first");
        vstate = 2;
        a_fact = d_acur;
        // thresh = smach_dist("Epsilon") * anorm (SRC/pdgstrf.c:412-413); in
        // psgstrf thresh is a float product.
        const float s_eps = 5.9604644775390625e-08f; // FLT_EPSILON * 0.5
        double thresh = sizeof(T) == 4 ? (double)(float)(s_eps * (float)anorm) : (double)s_eps * anorm;
        HIPCHK(hipMemsetAsync(d_counters.p, 0, d_counters.bytes(), stream));
        if (++ds_epoch >= 0x7fffffffu) { // (strip flags: a new epoch per factorization)
            HIPCHK(hipMemsetAsync(d_dsflags.p, 0, d_dsflags.bytes(), stream));
            ds_epoch = 1;
        }
        HIPCHK(hipMemsetAsync(d_zpiv.p, 0, d_zpiv.bytes(), stream));
#ifdef SLU_SB_STAMP
        {
            const unsigned z = 0;
            HIPCHK(hipMemcpyToSymbol(HIP_SYMBOL(slu_stamp_n), &z, sizeof z));
        }
#endif
        const bool timing = opts.timing != 0;
        vector<hipEvent_t> ev;
        auto mark = [&]() -> int {
            hipEvent_t e;
            HIPCHK(hipEventCreate(&e));
            HIPCHK(hipEventRecord(e, stream));
            ev.push_back(e);
            return (int)ev.size() - 1;
        };
        // kind: 0 diag, 1 trsm, 2 schur (128x128 tiles), 3 schur (64x64), 4 comm
        struct Span { int a, b, kind, level; };
        vector<Span> spans;
        int cur_level = 0;
        auto mark_on = [&](hipStream_t st) -> int {
            hipEvent_t e;
            HIPCHK(hipEventCreate(&e));
            HIPCHK(hipEventRecord(e, st));
            ev.push_back(e);
            return (int)ev.size() - 1;
        };
        auto span = [&](int kind, hipStream_t st, auto &&fn) {
            int a = timing ? mark_on(st) : -1;
            fn();
            if (timing) spans.push_back({a, mark_on(st), kind, cur_level});
        };
        if (zmode) { // ancestor forests another layer factors start from zero
            launch_zranges(zr_off[0], zr_off[1], ZR_ZERO, stream);
            zbytes = 0;
        }
        int e_start = timing ? mark() : -1;
        vector<int> lvl_end;
        HIPCHK(hipEventRecord(ev_start, stream));
        HIPCHK(hipStreamWaitEvent(pstream, ev_start, 0));
        X.s = opts.serial ? stream : pstream;
        stats.n_schur_launches = 0;
        stats.n_schur_big_launches = 0;
        // Look-ahead of one level on two streams:
        //   pstream: panel(L) -> [wait rest(L-1)] -> critical tiles(L) -> panel(L+1) ...
        //   stream : [wait panel(L)] -> rest tiles(L) -> [rest(L) done] ...
        // Critical tiles update exactly the destinations in the panels of
        // level L+1, so panel(L+1) (diag LU, TRSM, exchanges) runs beside the
        // bulk of level L's Schur update (SRC/pdgstrf.c:1115-1356 look-ahead).
        // 3D grids: my phases one after the other, each followed by its
        // ancestor reduction (SRC/pdgstrf3d.c:300-345)
        const int nph = zmode ? my_last + 1 : 1;
        int last_L = -1;
        vector<std::array<int, 3>> zmarks; // (phase start, phase end, reduction end) events
        int zstart = e_start;
        for (int ph = 0; ph < nph; ++ph) {
        const size_t L0 = zmode ? phase_lv[ph] : 0, L1 = zmode ? phase_lv[ph + 1] : levels.size();
        for (size_t L = L0; L < L1; ++L) {
            const LevelRange &R = levels[L];
            cur_level = (int)L;
            last_L = (int)L;
            hipStream_t P = opts.serial ? stream : pstream;
            if (R.diag_n)
                span(0, P, [&] {
                    hipLaunchKernelGGL(k_diag_lu<T>, dim3(R.diag_n), dim3(DIAG_THREADS), 0, P,
                                       d_diag.p + R.diag_off, thresh, opts.replace_tiny_pivot,
                                       d_counters.p, d_zpiv.p);
                });
            if (R.df_n)
                span(0, P, [&] {
                    if (strips_ok(R))
                        launch_strips(R, thresh, P);
                    else if (R.df_maxw <= DF_SMALLW && diag_wave_ok())
                        launch_diag_wave(R, thresh, P);
                    else if (R.df_maxw <= DF_SMALLW)
                        hipLaunchKernelGGL((k_diag_lu_f<T, DF_SMALLW, DF_SMALL_THREADS>), dim3(R.df_n),
                                           dim3(DF_SMALL_THREADS), 0, P, d_df.p + R.df_off, thresh,
                                           opts.replace_tiny_pivot, d_counters.p, d_zpiv.p);
                    else
                        hipLaunchKernelGGL(k_diag_lu_f<T>, dim3(R.df_n), dim3(DF_THREADS), 0, P,
                                           d_df.p + R.df_off, thresh, opts.replace_tiny_pivot,
                                           d_counters.p, d_zpiv.p);
                });
            if (xmode && !opts.serial) {
                // 2D grid: the exchanges on the comm stream C, the panels in
                // R.nch chunks.  P: TRSM(c) -> pack(c) -> [C: send / receive
                // chunk c] for every c, so chunk c + 1's TRSM runs beside
                // chunk c's transfer; the critical tiles of chunk c (P) and
                // its rest tiles (Schur stream) start when chunk c is in.
                hipStream_t C = cstream;
                auto exchange = [&](const vector<Sec> &secs, int off, int cnt, const char *what, hipEvent_t done) {
                    HIPCHK(hipEventRecord(ev_pk, P));
                    HIPCHK(hipStreamWaitEvent(C, ev_pk, 0));
                    X.s = C;
                    if (cnt) span(4, C, [&] { issue(secs, off, cnt, what, (int)L); });
                    HIPCHK(hipEventRecord(done, C));
                };
                if (R.dc_n || R.ds_n) {
                    if (R.dc_n)
                        span(4, P, [&] {
                            hipLaunchKernelGGL(k_copy<T>, dim3(R.dc_n), dim3(256), 0, P, d_dcopy.p + R.dc_off);
                        });
                    exchange(dsecs, R.ds_off, R.ds_n, "diagonal-package exchange", ev_dx);
                    HIPCHK(hipStreamWaitEvent(P, ev_dx, 0));
                }
                for (int ch = 0; ch < R.nch; ++ch) {
                    if (R.lf_o[ch + 1] > R.lf_o[ch] || R.uf_o[ch + 1] > R.uf_o[ch])
                        span(1, P, [&] { launch_trsm_fast(R, P, ch); });
                    if (ch == 0 && (R.tl_n || R.tu_n)) // (wide supernodes' generic items: all in chunk 0)
                        span(1, P, [&] {
                            if (R.tl_n)
                                hipLaunchKernelGGL(k_trsm_l<T>, dim3(R.tl_n), dim3(TRSM_THREADS), 0, P,
                                                   d_tl.p + R.tl_off);
                            if (R.tu_n)
                                hipLaunchKernelGGL(k_trsm_u<T>, dim3(R.tu_n), dim3(TRSM_THREADS), 0, P,
                                                   d_tu.p + R.tu_off);
                        });
                    const int pcn = R.pc_o[ch + 1] - R.pc_o[ch];
                    if (pcn)
                        span(4, P, [&] {
                            hipLaunchKernelGGL(k_copy<T>, dim3(pcn), dim3(256), 0, P, d_pcopy.p + R.pc_off + R.pc_o[ch]);
                        });
                    exchange(psecs, R.ps_off + R.ps_o[ch], R.ps_o[ch + 1] - R.ps_o[ch], "L/U panel exchange",
                             ev_cx[ch]);
                }
                // critical tiles of L on the panel stream, after the rest of L-1
                if (L > 0) HIPCHK(hipStreamWaitEvent(P, ev_rest[L - 1], 0));
                for (int ch = 0; ch < R.nch; ++ch) {
                    HIPCHK(hipStreamWaitEvent(P, ev_cx[ch], 0));
                    const int nb = R.bc_o[ch + 1] - R.bc_o[ch], nsm = R.sc_o[ch + 1] - R.sc_o[ch];
                    if (nb) {
                        span(2, P, [&] { launch_big(R, R.big_off + R.bc_o[ch], nb, P); });
                        stats.n_schur_launches++;
                        stats.n_schur_big_launches++;
                    }
                    if (nsm) {
                        span(3, P, [&] { launch_small(R, R.tile_off + R.sc_o[ch], nsm, P); });
                        stats.n_schur_launches++;
                    }
                }
                HIPCHK(hipEventRecord(ev_pan[L], P));
                // the rest of L on the Schur stream, chunk by chunk as they arrive
                for (int ch = 0; ch < R.nch; ++ch) {
                    HIPCHK(hipStreamWaitEvent(stream, ev_cx[ch], 0));
                    const int nb = R.br_o[ch + 1] - R.br_o[ch], nsm = R.sr_o[ch + 1] - R.sr_o[ch];
                    if (nb) {
                        span(2, stream, [&] { launch_big(R, R.big_off + R.bigc_n + R.br_o[ch], nb, stream); });
                        stats.n_schur_launches++;
                        stats.n_schur_big_launches++;
                    }
                    if (nsm) {
                        span(3, stream, [&] { launch_small(R, R.tile_off + R.tilec_n + R.sr_o[ch], nsm, stream); });
                        stats.n_schur_launches++;
                    }
                }
            } else {
                if (R.dc_n || R.ds_n)
                    span(4, P, [&] {
                        if (R.dc_n)
                            hipLaunchKernelGGL(k_copy<T>, dim3(R.dc_n), dim3(256), 0, P,
                                               d_dcopy.p + R.dc_off);
                        issue(dsecs, R.ds_off, R.ds_n, "diagonal-package exchange", (int)L);
                    });
                if (R.lf_n || R.uf_n) span(1, P, [&] { launch_trsm_fast(R, P); });
                if (R.tl_n || R.tu_n)
                    span(1, P, [&] {
                        if (R.tl_n)
                            hipLaunchKernelGGL(k_trsm_l<T>, dim3(R.tl_n), dim3(TRSM_THREADS), 0, P,
                                               d_tl.p + R.tl_off);
                        if (R.tu_n)
                            hipLaunchKernelGGL(k_trsm_u<T>, dim3(R.tu_n), dim3(TRSM_THREADS), 0, P,
                                               d_tu.p + R.tu_off);
                    });
                if (R.pc_n || R.ps_n)
                    span(4, P, [&] {
                        if (R.pc_n)
                            hipLaunchKernelGGL(k_copy<T>, dim3(R.pc_n), dim3(256), 0, P,
                                               d_pcopy.p + R.pc_off);
                        issue(psecs, R.ps_off, R.ps_n, "L/U panel exchange", (int)L);
                    });
                HIPCHK(hipEventRecord(ev_pan[L], P));
                // critical tiles of L on the panel stream, after the rest of L-1
                if (L > 0) HIPCHK(hipStreamWaitEvent(P, ev_rest[L - 1], 0));
                if (R.bigc_n) {
                    span(2, P, [&] { launch_big(R, R.big_off, R.bigc_n, P); });
                    stats.n_schur_launches++;
                    stats.n_schur_big_launches++;
                }
                if (R.tilec_n) {
                    span(3, P, [&] { launch_small(R, R.tile_off, R.tilec_n, P); });
                    stats.n_schur_launches++;
                }
                // the rest of L on the Schur stream, once the panels of L exist
                HIPCHK(hipStreamWaitEvent(stream, ev_pan[L], 0));
                if (R.big_n > R.bigc_n) {
                    // the first rest_split %% of the rest tiles as a launch of their own
                    const int nrest = R.big_n - R.bigc_n;
                    const int n1 = rest_split > 0 && !opts.serial ? (int)((i64)nrest * rest_split / 100) : 0;
                    span(2, stream, [&] {
                        if (n1 > 0) launch_big(R, R.big_off + R.bigc_n, n1, stream);
                        if (nrest > n1) launch_big(R, R.big_off + R.bigc_n + n1, nrest - n1, stream);
                    });
                    stats.n_schur_launches++;
                    stats.n_schur_big_launches++;
                }
                if (R.tile_n > R.tilec_n) {
                    span(3, stream, [&] {
                        launch_small(R, R.tile_off + R.tilec_n, R.tile_n - R.tilec_n, stream);
                    });
                    stats.n_schur_launches++;
                }
            }
            HIPCHK(hipEventRecord(ev_rest[L], stream));
            if (opts.timing >= 2) lvl_end.push_back(mark_on(stream)); // level wall time
        }
        if (zmode) {
            hipStream_t P = opts.serial ? stream : pstream;
            if (last_L >= 0) HIPCHK(hipStreamWaitEvent(P, ev_rest[last_L], 0));
            const int e_ph = timing ? mark_on(P) : -1;
            if (ph < maxlvl - 1) {
                span(4, P, [&] { zreduce(ph, P); });
                HIPCHK(hipEventRecord(ev_pend, P));
                HIPCHK(hipStreamWaitEvent(stream, ev_pend, 0));
            }
            if (timing) {
                const int e_red = mark_on(P);
                zmarks.push_back({zstart, e_ph, e_red});
                zstart = e_red;
            }
        }
        }
        if (xmode && !opts.serial) { // the comm stream's last group before the end of the factorization
            HIPCHK(hipEventRecord(ev_pend, cstream));
            HIPCHK(hipStreamWaitEvent(stream, ev_pend, 0));
        }
        X.s = opts.serial ? stream : pstream;
        HIPCHK(hipEventRecord(ev_pend, pstream));
        HIPCHK(hipStreamWaitEvent(stream, ev_pend, 0));
        HIPCHK(hipGetLastError());
        int e_end = timing ? mark() : -1;
        std::thread d2h;
        std::string d2h_err;
        double d2h_ms = 0;
        int64_t ncopies = 0;
        double dbytes = 0;
        const bool overlap_dl = opts.overlap_download != 0;
        // diagnostics: SLU_D2H_AFTER=1 starts the D2H only after the device
        // finished the factorization (no overlap, same copy path)
        const bool d2h_after = overlap_dl && getenv("SLU_D2H_AFTER");
        if (d2h_after) sync();
        if (overlap_dl) {
            d2h = std::thread([&] {
                const auto t0 = std::chrono::steady_clock::now();
                try {
                    run_d2h(dbytes, ncopies);
                } catch (const std::exception &e) {
                    d2h_err = e.what();
                }
                d2h_ms = ms_since(t0);
            });
        }
        try {
            sync();
        } catch (...) {
            if (d2h.joinable()) d2h.join();
            throw;
        }
        if (overlap_dl) {
            const auto t1 = std::chrono::steady_clock::now();
            d2h.join();
            SLU_REQUIRE(d2h_err.empty(), "factor download: %s", d2h_err.c_str());
            stats.t_d2h_tail_ms = ms_since(t1);
            stats.t_d2h_ms = d2h_ms;
            stats.d2h_bytes = dbytes;
            stats.n_d2h_copies = ncopies;
        }
        host_current = overlap_dl;
        int hc[4];
        HIPCHK(hipMemcpy(hc, d_counters.p, sizeof hc, hipMemcpyDeviceToHost));
        SLU_REQUIRE(hc[1] == 0, "factor: a diagonal-block strip waited more than a second for its left "
                                "neighbour (k_diag_strips hand-off timeout)");
        vector<int> zp(nsupers);
        HIPCHK(hipMemcpy(zp.data(), d_zpiv.p, nsupers * sizeof(int), hipMemcpyDeviceToHost));
        // per-rank info: the zero pivot of the last supernode (in elimination
        // order) that had one (SRC/pdgstrf2.c:246-247 overwrites *info); the
        // grid value is the MIN over ranks (SRC/pdgstrf.c:1927-1931)
        int my_info = 0;
        for (int k = 0; k < nsupers; ++k)
            if (zp[k]) my_info = zp[k];
        if (xmode || zmode) { // MIN over the grid (3D: all layers, SRC/pdgstrf3d.c:351-355)
            vector<i64> mine(1, my_info ? my_info : n + 1);
            i64 g = n + 1;
            if (xmode)
                for (auto &v : X.allgatherv(G_WORLD, mine)) g = std::min(g, v[0]);
            if (zmode && !zsolo) {
                mine[0] = g;
                X.s = stream;
                for (auto &v : X.allgatherv(G_Z, mine)) g = std::min(g, v[0]);
            }
            my_info = g == n + 1 ? 0 : (int)g;
        }
        *info = my_info;
        *tiny = hc[0];
        if (timing) {
            float ms;
            HIPCHK(hipEventElapsedTime(&ms, ev[e_start], ev[e_end]));
            stats.t_total_ms = ms;
            stats.t_diag_ms = stats.t_trsm_ms = stats.t_schur_ms = stats.t_schur_big_ms = 0;
            stats.t_comm_ms = 0;
            stats.schur_big_flops = 0;
            for (auto &s : spans) {
                HIPCHK(hipEventElapsedTime(&ms, ev[s.a], ev[s.b]));
                if (s.kind == 0) stats.t_diag_ms += ms;
                else if (s.kind == 1) stats.t_trsm_ms += ms;
                else if (s.kind == 4) stats.t_comm_ms += ms;
                else {
                    stats.t_schur_ms += ms;
                    if (s.kind == 2) stats.t_schur_big_ms += ms;
                }
            }
            for (auto &R : levels) stats.schur_big_flops += R.big_flops;
            for (int i = 0; i < 8; ++i) stats.t_phase_ms[i] = 0;
            stats.t_zreduce_ms = 0;
            for (size_t i = 0; i < zmarks.size() && i < 8; ++i) {
                HIPCHK(hipEventElapsedTime(&ms, ev[zmarks[i][0]], ev[zmarks[i][1]]));
                stats.t_phase_ms[i] = ms;
                HIPCHK(hipEventElapsedTime(&ms, ev[zmarks[i][1]], ev[zmarks[i][2]]));
                stats.t_zreduce_ms += ms;
            }
            if (opts.timing >= 2) { // per-level breakdown (stderr)
                vector<std::array<double, 5>> t(levels.size(), {0, 0, 0, 0, 0});
                for (auto &s : spans) {
                    HIPCHK(hipEventElapsedTime(&ms, ev[s.a], ev[s.b]));
                    t[s.level][s.kind] += ms;
                }
                fprintf(stderr, "[slu rank %d] lvl nsup diag trsm big small atomic  GFLOP  diag_ms trsm_ms big_ms small_ms comm_ms  TF/s wall_ms\n", iam);
                for (size_t L = 0; L < levels.size(); ++L) {
                    const LevelRange &R = levels[L];
                    double sch = t[L][2] + t[L][3];
                    float wall = 0;
                    HIPCHK(hipEventElapsedTime(&wall, ev[L ? lvl_end[L - 1] : e_start], ev[lvl_end[L]]));
                    fprintf(stderr, "[slu rank %d] %3zu %5zu %4d %5d %5d %5d %6d %7.2f %8.3f %7.3f %7.3f %7.3f %7.3f %6.2f %7.3f\n",
                            iam, L, bylev[L].size(), R.diag_n + R.df_n, R.lf_n + R.uf_n + R.tl_n + R.tu_n,
                            R.big_n, R.tile_n, R.atomic_tiles, R.schur_flops / 1e9, t[L][0], t[L][1], t[L][2], t[L][3],
                            t[L][4], sch > 0 ? R.schur_flops / sch / 1e9 : 0.0, (double)wall);
                }
            }
            for (auto e : ev) (void)hipEventDestroy(e);
        }
#ifdef SLU_SB_STAMP
        if (const char *fn = getenv("SLU_STAMP_OUT")) { // diagnostics build: per-tile stamps
            unsigned cnt = 0;
            HIPCHK(hipMemcpyFromSymbol(&cnt, HIP_SYMBOL(slu_stamp_n), sizeof cnt));
            cnt = std::min(cnt, SLU_STAMP_MAX);
            vector<uint64_t> h((size_t)cnt * 4);
            if (cnt) HIPCHK(hipMemcpyFromSymbol(h.data(), HIP_SYMBOL(slu_stamp), h.size() * 8));
            if (FILE *f = fopen(fn, "wb")) {
                fwrite(h.data(), 8, h.size(), f);
                fclose(f);
            }
        }
#endif
    }

    // ------------------------------------------------------- device solve
    // (1x1; solve.h).  Tables are built on the first call and kept.
    bool sv_ready = false;
    vector<int> sv_d_off, sv_l_off, sv_u_off; // per level: diag items, L chunks, U chunks
    DevBuf<SvDiag> d_sv_diag, d_sv_lvl;       // per supernode / in level order
    DevBuf<SvDiag> d_sv_pan;                  // per supernode: this rank's L rows below the diagonal block
    DevBuf<SvChunk> d_sv_lch, d_sv_uch;
    DevBuf<i64> d_sv_roff, d_sv_coff;
    DevBuf<int> d_sv_rows, d_sv_ncol, d_sv_gc;
    DevBuf<T> d_sv_x;

    void build_solve() {
        if (xmode) return build_solve_2d();
        vector<SvDiag> dg(nsupers), lvl;
        vector<i64> roff(nsupers), coff(nsupers, 0);
        vector<int> rows, ncol(nsupers, 0), gc;
        for (int k = 0; k < nsupers; ++k) {
            SLU_REQUIRE(lval_off[k] >= 0, "supernode %d has no L column block", k);
            SvDiag d{};
            d.voff = lval_off[k];
            d.ld = lval_ld[k];
            d.w = W(k);
            d.fst = (int)xsup[k];
            dg[k] = d;
            roff[k] = (i64)rows.size();
            const int_t *ix = lidx[k];
            i64 p = SLU_BC_HEADER;
            for (i64 b = 0; b < ix[0]; ++b) {
                const int gb = (int)ix[p], nr = (int)ix[p + 1];
                if (gb != k)
                    for (int i = 0; i < nr; ++i) rows.push_back((int)ix[p + 2 + i]);
                p += SLU_LB_DESCRIPTOR + nr;
            }
            SLU_REQUIRE((i64)rows.size() - roff[k] == d.ld - d.w, "supernode %d: panel rows", k);
            if (uval_off[k] >= 0 && urow_nblk[k] > 0) {
                coff[k] = ublk[urow_first[k]].coloff;
                for (int b = urow_first[k]; b < urow_first[k] + urow_nblk[k]; ++b) ncol[k] += W(ublk_jb[b]);
            }
        }
        gc.resize(ucol_voff.size());
        for (size_t b = 0; b < ublk.size(); ++b)
            for (int c = 0; c < W(ublk_jb[b]); ++c) gc[ublk[b].coloff + c] = ublk[b].fcol + c;
        vector<SvChunk> lch, uch;
        const int nl = (int)bylev.size();
        sv_d_off.assign(nl + 1, 0);
        sv_l_off.assign(nl + 1, 0);
        sv_u_off.assign(nl + 1, 0);
        for (int L = 0; L < nl; ++L) {
            sv_d_off[L] = (int)lvl.size();
            sv_l_off[L] = (int)lch.size();
            sv_u_off[L] = (int)uch.size();
            for (int k : bylev[L]) {
                lvl.push_back(dg[k]);
                for (int r0 = 0; r0 < dg[k].ld - dg[k].w; r0 += SV_THREADS) lch.push_back({k, r0});
                for (int c0 = 0; c0 < ncol[k]; c0 += SVU_COLS) uch.push_back({k, c0});
            }
        }
        sv_d_off[nl] = (int)lvl.size();
        sv_l_off[nl] = (int)lch.size();
        sv_u_off[nl] = (int)uch.size();
        d_sv_diag.upload(dg);
        {
            vector<SvDiag> pan(dg);
            for (auto &d : pan) {
                d.pad = d.ld - d.w;
                d.voff += d.w;
            }
            d_sv_pan.upload(pan);
        }
        d_sv_lvl.upload(lvl);
        d_sv_lch.upload(lch);
        d_sv_uch.upload(uch);
        d_sv_roff.upload(roff);
        d_sv_coff.upload(coff);
        d_sv_rows.upload(rows.empty() ? vector<int>(1, 0) : rows);
        d_sv_ncol.upload(ncol);
        d_sv_gc.upload(gc.empty() ? vector<int>(1, 0) : gc);
        d_sv_x.alloc(std::max(n, 1));
        HIPCHK(hipDeviceSynchronize()); // pageable table uploads landed (non-blocking streams)
        sv_ready = true;
    }

    // L and U sweeps over nr <= SV_NR device vectors xv (ld ldx, in place), on `stream`
    template <int NR> void sweep_nr(T *xv, i64 ldx, int nr) {
        const int nl = (int)bylev.size();
        for (int L = 0; L < nl; ++L) { // L y = b
            const int nd = sv_d_off[L + 1] - sv_d_off[L], nc = sv_l_off[L + 1] - sv_l_off[L];
            if (nd)
                hipLaunchKernelGGL((k_sv_ldiag<T, NR>), dim3(nd), dim3(SVD_THREADS), 0, stream,
                                   d_sv_lvl.p + sv_d_off[L], d_L.p, xv, ldx, nr);
            if (nc)
                hipLaunchKernelGGL((k_sv_lpanel<T, NR>), dim3(nc), dim3(SV_THREADS), 0, stream,
                                   d_sv_lch.p + sv_l_off[L], d_sv_pan.p, d_sv_roff.p,
                                   d_sv_rows.p, d_L.p, xv, ldx, nr);
        }
        for (int L = nl - 1; L >= 0; --L) { // U x = y
            const int nd = sv_d_off[L + 1] - sv_d_off[L], nc = sv_u_off[L + 1] - sv_u_off[L];
            if (nc)
                hipLaunchKernelGGL((k_sv_upanel<T, NR>), dim3(nc), dim3(SV_THREADS), 0, stream,
                                   d_sv_uch.p + sv_u_off[L], d_sv_diag.p, d_sv_coff.p,
                                   d_sv_ncol.p, d_ucol_voff.p, d_ucol_fst.p, d_sv_gc.p,
                                   d_U.p, xv, ldx, nr);
            if (nd)
                hipLaunchKernelGGL((k_sv_udiag<T, NR>), dim3(nd), dim3(SVD_THREADS), 0, stream,
                                   d_sv_lvl.p + sv_d_off[L], d_L.p, xv, ldx, nr);
        }
        HIPCHK(hipGetLastError());
    }
    void sweep(T *xv, i64 ldx = 0, int nr = 1) {
        if (nr == 1) sweep_nr<1>(xv, ldx, 1);
        else sweep_nr<SvNr<T>::v>(xv, ldx, nr);
    }

    // ---- 2D grids: the distributed supernodal solve of pdgstrs
    // (SRC/pdgstrs.c, pdgstrs_lsum.c), level-scheduled.  Block row k's partial
    // sums (lsum) live on its process row; per level they are sent to the
    // diagonal owner (k mod Pr, k mod Pc) along the row and added there; the
    // owner solves with the diagonal block; the solved piece goes down the
    // owner's process column to the ranks whose L(:,k) (forward) or U(:,k)
    // (backward) blocks use it, which push -L(i,k) y_k into their partial
    // sums of rows i (forward) or pull -U(i,k) x_k into rows i (backward).
    // b comes in and x goes out replicated on every rank (n values); each
    // rank starts from b on the block rows it owns and zero elsewhere.
    struct SvRed {                       // one partial-sum section of a level
        int k, c;                        // block row, sending process column
        i64 slot;                        // owner: offset of its slot in d_sv_slot
    };
    vector<vector<SvRed>> sv_red;        // per level, this rank's process row's sections
    vector<int> sv_add_off;              // per level: owner's slot-add items
    DevBuf<SvAdd> d_sv_add, d_sv_zero;
    DevBuf<T> d_sv_slot;
    vector<int> sv_own;                  // per supernode: this rank is the diagonal owner

    void build_solve_2d() {
        const int nl = (int)bylev.size();
        vector<SvDiag> dg(nsupers), pan(nsupers), lvl;
        vector<i64> roff(nsupers, 0), coff(nsupers, 0);
        vector<int> rows, ncol(nsupers, 0), gc;
        sv_own.assign(nsupers, 0);
        vector<SvAdd> zero;
        for (int k = 0; k < nsupers; ++k) {
            SvDiag d{};
            d.w = W(k);
            d.fst = (int)xsup[k];
            d.ld = 0;
            d.voff = 0;
            const bool lcol = k % Pc == mycol, own = lcol && k % Pr == myrow;
            sv_own[k] = own;
            if (!own) zero.push_back({(i64)xsup[k], -1, W(k), 0});
            SvDiag pd = d;
            pd.pad = 0;
            roff[k] = (i64)rows.size();
            if (lcol && lidx[k]) {
                const int ljb = k / Pc;
                SLU_REQUIRE(lval_off[ljb] >= 0, "supernode %d: no L column block", k);
                d.voff = lval_off[ljb];
                d.ld = lval_ld[ljb];
                int m = 0, r0 = 0;
                lrows(k, m, r0);
                SLU_REQUIRE(r0 == (own ? W(k) : 0), "supernode %d: diagonal block rows %d", k, r0);
                pd.voff = lval_off[ljb] + r0;
                pd.ld = lval_ld[ljb];
                pd.pad = m;
                const int_t *ix = lidx[k];
                i64 p = SLU_BC_HEADER;
                for (i64 b = 0; b < ix[0]; ++b) {
                    const int gb = (int)ix[p], nr = (int)ix[p + 1];
                    if (gb != k)
                        for (int i = 0; i < nr; ++i) rows.push_back((int)ix[p + 2 + i]);
                    p += SLU_LB_DESCRIPTOR + nr;
                }
            }
            dg[k] = d;
            pan[k] = pd;
            if (k % Pr == myrow) {
                const int lb = k / Pr;
                if (uval_off[lb] >= 0 && urow_nblk[lb] > 0) {
                    coff[k] = ublk[urow_first[lb]].coloff;
                    for (int b = urow_first[lb]; b < urow_first[lb] + urow_nblk[lb]; ++b)
                        ncol[k] += W(ublk_jb[b]);
                }
            }
        }
        gc.resize(ucol_voff.size());
        for (size_t b = 0; b < ublk.size(); ++b)
            for (int c = 0; c < W(ublk_jb[b]); ++c) gc[ublk[b].coloff + c] = ublk[b].fcol + c;
        vector<SvChunk> lch, uch;
        vector<SvAdd> adds;
        sv_d_off.assign(nl + 1, 0);
        sv_l_off.assign(nl + 1, 0);
        sv_u_off.assign(nl + 1, 0);
        sv_add_off.assign(nl + 1, 0);
        sv_red.assign(nl, {});
        i64 slot_max = 0;
        for (int L = 0; L < nl; ++L) {
            sv_d_off[L] = (int)lvl.size();
            sv_l_off[L] = (int)lch.size();
            sv_u_off[L] = (int)uch.size();
            sv_add_off[L] = (int)adds.size();
            i64 slot = 0;
            for (int k : bylev[L]) {
                if (sv_own[k]) lvl.push_back(dg[k]);
                for (int r0 = 0; r0 < pan[k].pad; r0 += SV_THREADS) lch.push_back({k, r0});
                for (int c0 = 0; c0 < ncol[k]; c0 += SVU_COLS) uch.push_back({k, c0});
                if (k % Pr != myrow) continue;
                if (sv_own[k] && Pc > 1) adds.push_back({(i64)xsup[k], slot, W(k), Pc - 1});
                for (int c = 0; c < Pc; ++c) {
                    if (c == k % Pc) continue;
                    SvRed r{k, c, -1};
                    if (sv_own[k]) {
                        r.slot = slot; // the Pc - 1 slots of k are consecutive
                        slot += W(k);
                    }
                    sv_red[L].push_back(r);
                }
            }
            slot_max = std::max(slot_max, slot);
        }
        sv_d_off[nl] = (int)lvl.size();
        sv_l_off[nl] = (int)lch.size();
        sv_u_off[nl] = (int)uch.size();
        sv_add_off[nl] = (int)adds.size();
        d_sv_diag.upload(dg);
        d_sv_pan.upload(pan);
        d_sv_lvl.upload(lvl.empty() ? vector<SvDiag>(1) : lvl);
        d_sv_lch.upload(lch.empty() ? vector<SvChunk>(1) : lch);
        d_sv_uch.upload(uch.empty() ? vector<SvChunk>(1) : uch);
        d_sv_roff.upload(roff);
        d_sv_coff.upload(coff);
        d_sv_rows.upload(rows.empty() ? vector<int>(1, 0) : rows);
        d_sv_ncol.upload(ncol);
        d_sv_gc.upload(gc.empty() ? vector<int>(1, 0) : gc);
        d_sv_add.upload(adds.empty() ? vector<SvAdd>(1) : adds);
        d_sv_zero.upload(zero.empty() ? vector<SvAdd>(1) : zero);
        d_sv_slot.alloc(std::max<i64>(slot_max, 1));
        d_sv_x.alloc(std::max(n, 1));
        HIPCHK(hipDeviceSynchronize()); // pageable table uploads landed (non-blocking streams)
        sv_ready = true;
    }

    // partial sums of the level's block rows to their owners, added there
    void sv_reduce(int L, T *xv) {
        for (const SvRed &r : sv_red[L]) {
            const int own_c = r.k % Pc;
            T *buf = mycol == r.c ? xv + xsup[r.k] : (mycol == own_c ? d_sv_slot.p + r.slot : nullptr);
            X.section(G_ROW, r.c, 1u << own_c, buf, (size_t)W(r.k) * sizeof(T));
        }
        X.phase = "solve: partial sums to the diagonal owners";
        X.level = L;
        X.flush();
        X.phase = "plan-time exchange";
        X.level = -1;
        const int na = sv_add_off[L + 1] - sv_add_off[L];
        if (na)
            hipLaunchKernelGGL(k_sv_add<T>, dim3(na), dim3(256), 0, stream, d_sv_add.p + sv_add_off[L],
                               xv, (const T *)d_sv_slot.p);
    }
    // the solved pieces of the level down their owners' process columns
    void sv_bcast(int L, T *xv, bool fwd) {
        const uint32_t all = Pr >= 32 ? ~0u : (1u << Pr) - 1;
        for (int k : bylev[L]) {
            if (k % Pc != mycol) continue;
            X.section(G_COL, k % Pr, fwd ? cmask(k) : all, xv + xsup[k], (size_t)W(k) * sizeof(T));
        }
        X.flush();
    }

    void sweep_2d(T *xv) {
        const int nl = (int)bylev.size();
        X.s = stream;
        const unsigned nz = (unsigned)(nsupers - std::accumulate(sv_own.begin(), sv_own.end(), 0));
        if (nz) hipLaunchKernelGGL(k_sv_add<T>, dim3(nz), dim3(256), 0, stream, d_sv_zero.p, xv, (const T *)nullptr);
        for (int L = 0; L < nl; ++L) { // L y = b
            sv_reduce(L, xv);
            const int nd = sv_d_off[L + 1] - sv_d_off[L], nc = sv_l_off[L + 1] - sv_l_off[L];
            if (nd)
                hipLaunchKernelGGL((k_sv_ldiag<T, 1>), dim3(nd), dim3(SVD_THREADS), 0, stream,
                                   d_sv_lvl.p + sv_d_off[L], d_L.p, xv, (i64)n, 1);
            sv_bcast(L, xv, true);
            if (nc)
                hipLaunchKernelGGL((k_sv_lpanel<T, 1>), dim3(nc), dim3(SV_THREADS), 0, stream,
                                   d_sv_lch.p + sv_l_off[L], d_sv_pan.p, d_sv_roff.p,
                                   d_sv_rows.p, d_L.p, xv, (i64)n, 1);
        }
        const bool fwd_only = getenv("SLU_SV_FWD_ONLY") != nullptr; // diagnostics: y = L^-1 b
        if (nz && !fwd_only) hipLaunchKernelGGL(k_sv_add<T>, dim3(nz), dim3(256), 0, stream, d_sv_zero.p, xv, (const T *)nullptr);
        for (int L = fwd_only ? -1 : nl - 1; L >= 0; --L) { // U x = y
            const int nd = sv_d_off[L + 1] - sv_d_off[L], nc = sv_u_off[L + 1] - sv_u_off[L];
            if (nc)
                hipLaunchKernelGGL((k_sv_upanel<T, 1>), dim3(nc), dim3(SV_THREADS), 0, stream,
                                   d_sv_uch.p + sv_u_off[L], d_sv_diag.p, d_sv_coff.p,
                                   d_sv_ncol.p, d_ucol_voff.p, d_ucol_fst.p, d_sv_gc.p,
                                   d_U.p, xv, (i64)n, 1);
            sv_reduce(L, xv);
            if (nd)
                hipLaunchKernelGGL((k_sv_udiag<T, 1>), dim3(nd), dim3(SVD_THREADS), 0, stream,
                                   d_sv_lvl.p + sv_d_off[L], d_L.p, xv, (i64)n, 1);
            sv_bcast(L, xv, false);
        }
        sv_gather(xv);
        HIPCHK(hipGetLastError());
    }
    // each diagonal owner's block rows of xv to every rank (xv replicated)
    void sv_gather(T *xv) {
        for (int k = 0; k < nsupers; ++k)
            X.section(G_WORLD, (k % Pr) * Pc + k % Pc, ~0u, xv + xsup[k], (size_t)W(k) * sizeof(T));
        X.flush();
    }

    // right-hand sides in batches of SvNr<T>: every factor element is read once
    // per batch and sweep
    void solve(void *b, int64_t ldb, int nrhs) override {
        SLU_REQUIRE(!zmode, "solve: 3D plans hold the factors spread over the layers (gather them to a 2D plan)");
        SLU_REQUIRE(vstate == 2, "solve: the device storage holds no factors (factor first)");
        if (!sv_ready) build_solve();
        if (xmode) {
            SLU_REQUIRE(ldb >= n && nrhs >= 0, "solve: ldb %lld < n %d", (long long)ldb, n);
            HIPCHK(hipStreamSynchronize(pstream));
            hipEvent_t e0, e1;
            HIPCHK(hipEventCreate(&e0));
            HIPCHK(hipEventCreate(&e1));
            float total = 0;
            for (int j = 0; j < nrhs; ++j) {
                HT *bj = (HT *)b + (i64)j * ldb;
                HIPCHK(hipMemcpyAsync(d_sv_x.p, bj, (size_t)n * sizeof(T), hipMemcpyHostToDevice, stream));
                HIPCHK(hipEventRecord(e0, stream));
                sweep_2d(d_sv_x.p);
                HIPCHK(hipEventRecord(e1, stream));
                HIPCHK(hipMemcpyAsync(bj, d_sv_x.p, (size_t)n * sizeof(T), hipMemcpyDeviceToHost, stream));
                HIPCHK(hipStreamSynchronize(stream));
                float ms = 0;
                HIPCHK(hipEventElapsedTime(&ms, e0, e1));
                total += ms;
            }
            (void)hipEventDestroy(e0);
            (void)hipEventDestroy(e1);
            stats.t_solve_ms = total;
            return;
        }
        SLU_REQUIRE(ldb >= n && nrhs >= 0, "solve: ldb %lld < n %d", (long long)ldb, n);
        constexpr int NB = SvNr<T>::v;
        if (nrhs > 1 && d_sv_x.n < (size_t)n * NB) d_sv_x.alloc((size_t)std::max(n, 1) * NB);
        hipEvent_t e0, e1;
        HIPCHK(hipEventCreate(&e0));
        HIPCHK(hipEventCreate(&e1));
        float total = 0;
        for (int r0 = 0; r0 < nrhs; r0 += NB) {
            const int nr = std::min(NB, nrhs - r0);
            for (int q = 0; q < nr; ++q)
                HIPCHK(hipMemcpyAsync(d_sv_x.p + (i64)q * n, (HT *)b + (i64)(r0 + q) * ldb,
                                      (size_t)n * sizeof(T), hipMemcpyHostToDevice, stream));
            HIPCHK(hipEventRecord(e0, stream));
            sweep(d_sv_x.p, n, nr);
            HIPCHK(hipEventRecord(e1, stream));
            for (int q = 0; q < nr; ++q)
                HIPCHK(hipMemcpyAsync((HT *)b + (i64)(r0 + q) * ldb, d_sv_x.p + (i64)q * n,
                                      (size_t)n * sizeof(T), hipMemcpyDeviceToHost, stream));
            HIPCHK(hipStreamSynchronize(stream));
            float ms = 0;
            HIPCHK(hipEventElapsedTime(&ms, e0, e1));
            total += ms;
        }
        (void)hipEventDestroy(e0);
        (void)hipEventDestroy(e1);
        stats.t_solve_ms = total;
    }

    // Iterative refinement on the device (SRC/pdgsrfs.c:197-253, 1x1 grid,
    // permuted coordinates): R = B - A X and S = |A||X| + |B| by rows of A
    // (k_resid), componentwise backward error berr = max |R_i| / S_i with the
    // SAFE1/SAFE2 guards (:219-230); while berr > eps, berr halves and fewer
    // than ITMAX = 20 steps: solve A dx = R with the device factors, X += dx.
    // A is the matrix of the last slu_plan_fill_a.
    DevBuf<i64> d_rp;
    DevBuf<int> d_rc;
    DevBuf<i64> d_re;
    const T *d_acur = nullptr;
    DevBuf<T> d_rf_b, d_rf_x, d_rf_r;
    DevBuf<unsigned long long> d_rf_berr;

    // 2D grids: the same loop with pdgsmv's distributed residual (solve.h
    // k_resid_part / k_resid_fin): partial rows from each rank's entries of
    // A, reduced along process rows to the diagonal owners, berr = the max
    // over the owners, R gathered to every rank, then the 2D solve.
    vector<RfRow> rf_rows_h;
    DevBuf<RfRow> d_rf_rows;
    DevBuf<double> d_rf_s, d_rf_ss;
    DevBuf<T> d_rf_sr;
    vector<std::array<i64, 3>> rf_secs; // (block row, sending column, owner slot)

    void build_refine_2d() {
        rf_rows_h.clear();
        rf_secs.clear();
        i64 slot = 0;
        for (int k = 0; k < nsupers; ++k) {
            if (k % Pr != myrow) continue;
            const bool own = k % Pc == mycol;
            if (own) rf_rows_h.push_back({(i64)xsup[k], slot, W(k), Pc - 1});
            for (int c = 0; c < Pc; ++c) {
                if (c == k % Pc) continue;
                rf_secs.push_back({k, c, own ? slot : -1});
                if (own) slot += W(k);
            }
        }
        d_rf_rows.upload(rf_rows_h.empty() ? vector<RfRow>(1) : rf_rows_h);
        d_rf_sr.alloc(std::max<i64>(slot, 1));
        d_rf_ss.alloc(std::max<i64>(slot, 1));
        d_rf_s.alloc(std::max(n, 1));
        HIPCHK(hipDeviceSynchronize());
    }

    double resid_2d(double safe1, double safe2) {
        const unsigned rb = (unsigned)((n + 255) / 256);
        X.s = stream;
        hipLaunchKernelGGL(k_resid_part<T>, dim3(rb), dim3(256), 0, stream, d_rp.p, d_rc.p, d_re.p,
                           a_fact, d_rf_x.p, d_rf_r.p, d_rf_s.p, n);
        for (const auto &q : rf_secs) {
            const int k = (int)q[0], c = (int)q[1], oc = k % Pc;
            const size_t w = (size_t)W(k);
            void *br = mycol == c ? (void *)(d_rf_r.p + xsup[k]) : mycol == oc ? (void *)(d_rf_sr.p + q[2]) : nullptr;
            void *bs = mycol == c ? (void *)(d_rf_s.p + xsup[k]) : mycol == oc ? (void *)(d_rf_ss.p + q[2]) : nullptr;
            X.section(G_ROW, c, 1u << oc, br, w * sizeof(T));
            X.section(G_ROW, c, 1u << oc, bs, w * sizeof(double));
        }
        X.flush();
        HIPCHK(hipMemsetAsync(d_rf_berr.p, 0, sizeof(unsigned long long), stream));
        if (!rf_rows_h.empty())
            hipLaunchKernelGGL(k_resid_fin<T>, dim3((unsigned)rf_rows_h.size()), dim3(256), 0, stream,
                               d_rf_rows.p, d_rf_b.p, d_rf_r.p, d_rf_s.p, d_rf_sr.p, d_rf_ss.p, safe1,
                               safe2, d_rf_berr.p);
        HIPCHK(hipGetLastError());
        unsigned long long bits = 0;
        HIPCHK(hipMemcpyAsync(&bits, d_rf_berr.p, sizeof bits, hipMemcpyDeviceToHost, stream));
        HIPCHK(hipStreamSynchronize(stream));
        // the max over the owners (bit patterns of non-negative doubles, NaN above +Inf)
        auto all = X.allgatherv(G_WORLD, vector<i64>(1, (i64)bits));
        unsigned long long m = 0;
        for (auto &v : all) m = std::max(m, (unsigned long long)v[0]);
        double be;
        memcpy(&be, &m, sizeof be);
        return be;
    }

    void refine(const void *b, void *x, int64_t ld, int nrhs, double *berr, int *steps) override {
        SLU_REQUIRE(!zmode, "refine: not on 3D plans");
        SLU_REQUIRE(vstate == 2, "refine: the device storage holds no factors (factor first)");
        SLU_REQUIRE(a_fact != nullptr,
                    "refine needs the values of A the factors came from (slu_plan_fill_a "
                    "before slu_plan_factor)");
        SLU_REQUIRE(ld >= n && nrhs >= 0, "refine: ld %lld < n %d", (long long)ld, n);
        if (!sv_ready) build_solve();
        const bool dbl = !std::is_same<T, float>::value;
        const double eps = dbl ? 0.5 * 2.220446049250313e-16 : 0.5 * 1.1920928955078125e-07;
        const double safmin = dbl ? 2.2250738585072014e-308 : 1.1754943508222875e-38;
        const double safe1 = (double)(n + 1) * safmin, safe2 = safe1 / eps;
        d_rf_b.alloc(std::max(n, 1));
        d_rf_x.alloc(std::max(n, 1));
        d_rf_r.alloc(std::max(n, 1));
        d_rf_berr.alloc(1);
        if (xmode && rf_rows_h.empty() && rf_secs.empty()) build_refine_2d();
        const unsigned rb = (unsigned)((n + 255) / 256);
        hipEvent_t e0, e1;
        HIPCHK(hipEventCreate(&e0));
        HIPCHK(hipEventCreate(&e1));
        HIPCHK(hipStreamSynchronize(pstream));
        HIPCHK(hipEventRecord(e0, stream));
        for (int j = 0; j < nrhs; ++j) {
            const HT *hb = (const HT *)b + (i64)j * ld;
            HT *hx = (HT *)x + (i64)j * ld;
            HIPCHK(hipMemcpyAsync(d_rf_b.p, hb, (size_t)n * sizeof(T), hipMemcpyHostToDevice, stream));
            HIPCHK(hipMemcpyAsync(d_rf_x.p, hx, (size_t)n * sizeof(T), hipMemcpyHostToDevice, stream));
            int count = 0;
            double lstres = 3.0, be = 0.0;
            while (true) {
                if (xmode) {
                    be = resid_2d(safe1, safe2);
                } else {
                    HIPCHK(hipMemsetAsync(d_rf_berr.p, 0, sizeof(unsigned long long), stream));
                    hipLaunchKernelGGL(k_resid<T>, dim3(rb), dim3(256), 0, stream, d_rp.p, d_rc.p, d_re.p,
                                       a_fact, d_rf_x.p, d_rf_b.p, d_rf_r.p, n, safe1, safe2, d_rf_berr.p);
                    HIPCHK(hipGetLastError());
                    unsigned long long bits = 0;
                    HIPCHK(hipMemcpyAsync(&bits, d_rf_berr.p, sizeof bits, hipMemcpyDeviceToHost, stream));
                    HIPCHK(hipStreamSynchronize(stream));
                    memcpy(&be, &bits, sizeof be);
                }
                if (!(be > eps && be * 2 <= lstres && count < 20)) break;
                if (xmode) {
                    sv_gather(d_rf_r.p); // R from its owners to every rank, then the 2D solve
                    sweep_2d(d_rf_r.p);
                } else {
                    sweep(d_rf_r.p);
                }
                hipLaunchKernelGGL(k_axpy1<T>, dim3(rb), dim3(256), 0, stream, d_rf_x.p, d_rf_r.p, n);
                lstres = be;
                ++count;
            }
            HIPCHK(hipMemcpyAsync(hx, d_rf_x.p, (size_t)n * sizeof(T), hipMemcpyDeviceToHost, stream));
            HIPCHK(hipStreamSynchronize(stream));
            if (berr) berr[j] = be;
            if (steps) steps[j] = count;
        }
        HIPCHK(hipEventRecord(e1, stream));
        HIPCHK(hipStreamSynchronize(stream));
        float ms = 0;
        HIPCHK(hipEventElapsedTime(&ms, e0, e1));
        (void)hipEventDestroy(e0);
        (void)hipEventDestroy(e1);
        stats.t_refine_ms = ms;
    }

    // ------------------------------------------------------- values of A
    // SamePattern_SameRowPerm refill (SRC/pddistribute.c:545-672) on the
    // device: the destination of every nonzero of A in this rank's L/U
    // storage is resolved once per pattern, with the reference's rules --
    // row block gb < column block jb goes to U(gb,jb) at the segment offset of
    // column j (:598-618), otherwise to L(:,jb) at the row's position in the
    // block column (:619-656); entries of other process rows / columns are
    // skipped (:587,596).
    DevBuf<i64> d_amap;
    DevBuf<T> d_aval;
    i64 a_nnz = -1;

    bool has_block(int gb, int jb) const { // this rank holds L(gb,jb) (gb >= jb) or U(gb,jb)
        const vector<int> &ids = gb < jb ? ublk_jb : lblk_ib;
        const int f = gb < jb ? urow_first[gb / Pr] : lcol_first[jb / Pc];
        const int nb = gb < jb ? urow_nblk[gb / Pr] : lcol_nblk[jb / Pc];
        return std::binary_search(ids.begin() + f, ids.begin() + f + nb, gb < jb ? jb : gb);
    }

    void set_a_pattern(int64_t ncol, const int64_t *xa, const int64_t *asub) override {
        SLU_REQUIRE(ncol == n, "A has %lld columns, the LU structure %d", (long long)ncol, n);
        SLU_REQUIRE(xa[0] == 0 && xa[n] >= 0, "A: bad column pointers");
        const int_t *supno = LU->Glu_persist->supno;
        const i64 nnz = xa[n];
        const bool aprof = getenv("SLU_PROFILE_PLAN") != nullptr;
        auto ta = std::chrono::steady_clock::now();
        auto atick = [&](const char *what) { // SLU_PROFILE_PLAN: phase times on stderr
            if (!aprof) return;
            fprintf(stderr, "[slu plan %d] a_pattern %-16s %7.1f ms\n", iam, what, ms_since(ta));
            ta = std::chrono::steady_clock::now();
        };
        vector<i64> map((size_t)nnz, -1);
        // columns on the host threads: each nonzero belongs to one column, so
        // the writes to map are disjoint
        parallel_for(n, [&](int j) {
            thread_local vector<std::pair<i64, i64>> col; // (destination, nonzero) of one column
            const int jb = (int)supno[j];
            SLU_REQUIRE(xa[j + 1] >= xa[j], "A: column pointers decrease at %d", j);
            if (jb % Pc != mycol) return;
            const int jc = (int)(j - xsup[jb]);
            col.clear();
            for (i64 e = xa[j]; e < xa[j + 1]; ++e) {
                const i64 irow = asub[e];
                SLU_REQUIRE(irow >= 0 && irow < n, "A(%lld,%d): row out of range", (long long)irow, j);
                const int gb = (int)supno[irow];
                if (gb % Pr != myrow) continue;
                i64 m;
                if (!has_block(gb, jb))
                    throw Error(fmt("A(%lld,%d) is outside the %c structure (no block (%d,%d))",
                                    (long long)irow, j, gb < jb ? 'U' : 'L', gb, jb));
                if (gb < jb) {
                    const UBlk &B = ublk[find_ublk(gb, jb)];
                    const i64 c = B.coloff + jc;
                    SLU_REQUIRE(irow >= ucol_fst[c], "A(%lld,%d) is outside the U structure",
                                (long long)irow, j);
                    m = 2 * (ucol_voff[c] + irow - ucol_fst[c]) + 1;
                } else {
                    const LBlk &B = lblk[find_lblk(gb, jb)];
                    const int pos = lmap[B.mapoff + irow - xsup[gb]];
                    SLU_REQUIRE(pos >= 0, "A(%lld,%d) is outside the L structure", (long long)irow, j);
                    m = 2 * (B.colvoff + (i64)jc * B.ld + pos);
                }
                col.push_back({m, e});
            }
            // a duplicated (row, column): the later entry wins, as in the SPA
            std::sort(col.begin(), col.end());
            for (size_t i = 0; i < col.size(); ++i)
                if (i + 1 == col.size() || col[i + 1].first != col[i].first)
                    map[col[i].second] = col[i].first;
        }, 512);
        atick("map");
        d_amap.upload(map.empty() ? vector<i64>(1, -1) : map);
        d_aval.alloc(std::max<i64>(nnz, 1));
        atick("map upload");
        a_nnz = nnz;
        d_acur = a_fact = snap_acur = nullptr; // the previous pattern's values are gone
        {   // rows of A for the refinement's residual (k_resid): all of A on a
            // 1x1 grid, this rank's entries (those of its blocks) on a 2D grid
            auto mine = [&](i64 e, int j) {
                return !xmode || ((int)supno[j] % Pc == mycol && (int)supno[asub[e]] % Pr == myrow);
            };
            // a counting sort by row on the host threads: the columns in NCH
            // chunks of about equal nnz, per (chunk, row) counts, then each
            // chunk fills its slice of every row (chunk order = column order,
            // so each row's entries come in column order, as serially)
            const int NCH = std::max(1, std::min(plan_threads(), (int)std::min<i64>(16, nnz / 65536 + 1)));
            SLU_REQUIRE(nnz < INT32_MAX, "A: %lld nonzeros", (long long)nnz);
            vector<int> cb(NCH + 1, 0);
            for (int c = 1; c < NCH; ++c)
                cb[c] = std::max(cb[c - 1], (int)(std::lower_bound(xa, xa + n + 1, nnz * c / NCH) - xa));
            cb[NCH] = n;
            vector<int32_t> cc((size_t)NCH * n, 0); // [chunk][row] counts, then fill cursors
            parallel_for(NCH, [&](int c) {
                int32_t *cnt = cc.data() + (size_t)c * n;
                for (int j = cb[c]; j < cb[c + 1]; ++j)
                    for (i64 e = xa[j]; e < xa[j + 1]; ++e)
                        if (mine(e, j)) ++cnt[asub[e]];
            }, 1);
            vector<i64> rp(n + 1, 0);
            const int NB = (n + 65535) / 65536;
            parallel_for(NB, [&](int t) {
                for (int i = t * 65536; i < std::min(n, (t + 1) * 65536); ++i) {
                    i64 tot = 0;
                    for (int c = 0; c < NCH; ++c) tot += cc[(size_t)c * n + i];
                    rp[i + 1] = tot;
                }
            }, 1);
            for (int i = 0; i < n; ++i) rp[i + 1] += rp[i];
            parallel_for(NB, [&](int t) {
                for (int i = t * 65536; i < std::min(n, (t + 1) * 65536); ++i) {
                    i64 pos = rp[i];
                    for (int c = 0; c < NCH; ++c) {
                        const int32_t k = cc[(size_t)c * n + i];
                        cc[(size_t)c * n + i] = (int32_t)pos;
                        pos += k;
                    }
                }
            }, 1);
            vector<i64> re((size_t)rp[n]);
            vector<int> rc((size_t)rp[n]);
            parallel_for(NCH, [&](int c) {
                int32_t *nx = cc.data() + (size_t)c * n;
                for (int j = cb[c]; j < cb[c + 1]; ++j)
                    for (i64 e = xa[j]; e < xa[j + 1]; ++e) {
                        if (!mine(e, j)) continue;
                        const i64 q = nx[asub[e]]++;
                        rc[q] = j;
                        re[q] = e;
                    }
            }, 1);
            atick("rows");
            d_rp.upload(rp);
            d_rc.upload(rc.empty() ? vector<int>(1, 0) : rc);
            d_re.upload(re.empty() ? vector<i64>(1, 0) : re);
            atick("rows upload");
            HIPCHK(hipDeviceSynchronize());
            atick("device sync");
        }
    }

    void fill_a(const void *a, int on_device) override {
        SLU_REQUIRE(a_nnz >= 0, "fill_a before set_a_pattern");
        const T *src = (const T *)a;
        if (!on_device) {
            if (a_nnz)
                HIPCHK(hipMemcpyAsync(d_aval.p, a, (size_t)a_nnz * sizeof(T), hipMemcpyHostToDevice, stream));
            src = d_aval.p;
        }
        d_acur = src;
        vstate = 1;
        host_current = false;
        hipEvent_t e0, e1;
        HIPCHK(hipEventCreate(&e0));
        HIPCHK(hipEventCreate(&e1));
        HIPCHK(hipStreamSynchronize(pstream));
        HIPCHK(hipEventRecord(e0, stream));
        if (d_L.n) HIPCHK(hipMemsetAsync(d_L.p, 0, d_L.bytes(), stream));
        if (d_U.n) HIPCHK(hipMemsetAsync(d_U.p, 0, d_U.bytes(), stream));
        if (a_nnz) {
            const i64 blocks = std::min<i64>((a_nnz + FILL_THREADS - 1) / FILL_THREADS, 65536);
            hipLaunchKernelGGL(k_fill_a<T>, dim3((unsigned)blocks), dim3(FILL_THREADS), 0, stream,
                               d_amap.p, src, a_nnz, d_L.p, d_U.p);
            HIPCHK(hipGetLastError());
        }
        HIPCHK(hipEventRecord(e1, stream));
        HIPCHK(hipStreamSynchronize(stream));
        float ms = 0;
        HIPCHK(hipEventElapsedTime(&ms, e0, e1));
        (void)hipEventDestroy(e0);
        (void)hipEventDestroy(e1);
        stats.t_fill_ms = ms;
    }
};

template <typename P> PlanBase *make_plan(void *LU, int n, int pr, int pc, int iam, slu_comm *c,
                                          const slu_engine_opts *o) {
    return new P((decltype(std::declval<P>().LU))LU, n, pr, pc, iam, c, o);
}


// ---------------------------------------------------------------- amalgamation
// A 1x1 plan over the coarse partition of csrc/amalg.h.  The inner plan is an
// ordinary Plan built on the coarse LUstruct's index arrays (held here, no
// host values); the caller's values travel in their own layout (d_oL / d_oU)
// and are relaid on the device: expand at upload (caller -> coarse), compress
// at download (coarse -> caller).  The device-resident state between upload
// and download -- what factor(), snapshot / restore, fill_a, solve and refine
// work on -- is the coarse layout.
template <typename T, typename HT, typename LocalLU, typename LUS>
struct AmalgPlan : PlanBase {
    using Inner = Plan<T, HT, LocalLU, LUS>;
    LUS *LU = nullptr;
    int n = 0, ns = 0;
    Amalg A;
    // the coarse LUstruct the inner plan reads (index arrays only)
    LUS mlu{};
    LocalLU mllu{};
    Glu_persist_t mglu{};
    vector<int_t *> mlidx, muidx;
    std::unique_ptr<Inner> in;
    slu_engine_opts opts{};
    // caller layout on the device, and the relayout programs
    DevBuf<T> d_oL, d_oU;
    DevBuf<LColX> d_lx;
    DevBuf<int32_t> d_lrow, d_ucd;
    DevBuf<uint16_t> d_ucl;
    DevBuf<UChunk> d_ur;
    DevBuf<i64> d_D;
    vector<i64> usrc; // caller U value offset per block row
    std::thread up_thread;
    std::string up_err;
    // the coarse L / U storage, allocated beside the analysis as soon as its
    // sizes are known (after pass 3a), adopted by the inner plan
    DevBuf<T> pre[2];
    std::thread alloc_thread;
    std::string alloc_err;
    std::mutex o_mu; // ensure_o: the upload thread or the D2H program build
    // fresh HBM is mapped at its first touch; the caller-layout buffers are
    // touched first thing on the upload thread (o_mapped), and the D2H warm-up
    // (pinned slots) waits for that
    std::mutex map_mu;
    std::condition_variable map_cv;
    bool o_mapped = false;
    double t_omap = 0;
    std::chrono::steady_clock::time_point t_born = std::chrono::steady_clock::now();
    void set_mapped() {
        std::lock_guard<std::mutex> lk(map_mu);
        o_mapped = true;
        map_cv.notify_all();
    }
    // the D2H's pinned slots and HBM staging slots, allocated and touched
    // (one DMA through each) beside the plan build: lazily, the first
    // factorization paid ~70 ms more D2H tail for them
    std::thread warm_thread;
    std::string warm_err;
    DevBuf<char> warm_stage;
    void warm_join() {
        if (warm_thread.joinable()) warm_thread.join();
        SLU_REQUIRE(warm_err.empty(), "%s", warm_err.c_str());
    }
    double up_ms = 0, h2d_bytes = 0;
    double t_amalg = 0, t_plan = 0, t_expand = 0, t_compress = 0, t_d2h = 0;
    bool coarse_current = false; // d_oL / d_oU stale: the coarse storage holds newer values

    static double ms_since(std::chrono::steady_clock::time_point t0) {
        return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0)
            .count();
    }

    // Returns nullptr when nothing merges (the caller then builds a Plan).
    static AmalgPlan *make(LUS *lu, int n_, const slu_engine_opts *o, double zero_frac, int maxw) {
        auto t0 = std::chrono::steady_clock::now();
        std::unique_ptr<AmalgPlan> P(new AmalgPlan);
        P->LU = lu;
        P->n = n_;
        if (o) P->opts = *o;
        const int_t *xsup = lu->Glu_persist->xsup;
        P->ns = (int)(lu->Glu_persist->supno[n_ - 1] + 1);
        LocalLU *L = lu->Llu;
        const int ns = P->ns;
        // caller value layout: contiguous per block column / row in supernode order
        i64 lv = 0, uv = 0;
        P->usrc.assign(ns + 1, 0);
        for (int s = 0; s < ns; ++s) {
            if (L->Lrowind_bc_ptr[s]) lv += (i64)L->Lrowind_bc_ptr[s][1] * (xsup[s + 1] - xsup[s]);
            if (L->Ufstnz_br_ptr[s]) uv += L->Ufstnz_br_ptr[s][1];
            P->usrc[s + 1] = uv;
        }
        const bool prof = getenv("SLU_PROFILE_PLAN") != nullptr;
        auto tk = t0;
        auto tick = [&](const char *what) { // SLU_PROFILE_PLAN: phase times on stderr
            if (!prof) return;
            fprintf(stderr, "[slu amalg plan] %-22s %7.1f ms\n", what, ms_since(tk));
            tk = std::chrono::steady_clock::now();
        };
        HIPCHK(hipSetDevice(0));
        tick("caller layout");
        P->o_lv = lv;
        P->o_uv = uv;
        // the caller-layout copies only where values cross PCIe: a plan fed
        // by fill_a and read by solve never allocates them (the upload thread
        // allocates them itself, beside the analysis)
        if (!P->opts.overlap_upload && P->opts.overlap_download) P->ensure_o();
        tick("caller-layout alloc");
        P->A.on_sizes = [raw = P.get()](int64_t lv2, int64_t uv2) {
            raw->alloc_thread = std::thread([raw, lv2, uv2] {
                try {
                    HIPCHK(hipSetDevice(0));
                    const auto ta = std::chrono::steady_clock::now();
                    const double at = ms_since(raw->t_born);
                    raw->pre[0].alloc_guarded(std::max<i64>(lv2, 1), SB_UGUARD);
                    raw->pre[1].alloc_guarded(std::max<i64>(uv2, 1), SB_UGUARD);
                    if (getenv("SLU_PROFILE_PLAN"))
                        fprintf(stderr, "[slu amalg plan]   (coarse storage %.1f GB mapped in %.1f ms, from %.1f ms)\n",
                                (lv2 + uv2) * sizeof(T) / 1e9, ms_since(ta), at);
                } catch (const std::exception &e) {
                    raw->alloc_err = e.what();
                }
            });
        };
        if (P->opts.overlap_upload) {
            AmalgPlan *raw = P.get();
            P->up_thread = std::thread([raw] {
                try {
                    HIPCHK(hipSetDevice(0));
                    raw->h2d();
                } catch (const std::exception &e) {
                    raw->up_err = e.what();
                }
                raw->set_mapped(); // (also on failure: the warm-up waits for it)
            });
        }
        if (P->opts.overlap_download) {
            AmalgPlan *raw = P.get();
            raw->warm_thread = std::thread([raw] {
                try {
                    HIPCHK(hipSetDevice(0));
                    // after the caller-layout buffers' mapping: beside it the
                    // pinned allocation made that mapping 102-274 instead of
                    // 34-37 ms (profiles/r04y)
                    if (raw->opts.overlap_upload) {
                        std::unique_lock<std::mutex> lk(raw->map_mu);
                        raw->map_cv.wait(lk, [raw] { return raw->o_mapped; });
                    }
                    i64 slot = 128ll << 20; // (Plan::D2H_SLOT, and its override as in build_d2h)
                    if (const char *e = getenv("SLU_D2H_SLOT_KB")) slot = std::max<i64>(16, atoll(e)) << 10;
                    constexpr int NS = Inner::D2H_NS;
                    std::lock_guard<std::mutex> in_use(pinned_pool(1).use);
                    std::vector<char *> slots = pinned_pool(1).get(NS, slot);
                    raw->warm_stage.alloc((size_t)NS * slot);
                    hipStream_t st = nullptr;
                    HIPCHK(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
                    HIPCHK(hipMemsetAsync(raw->warm_stage.p, 0, raw->warm_stage.bytes(), st));
                    for (int i = 0; i < NS; ++i)
                        HIPCHK(hipMemcpyAsync(slots[i], raw->warm_stage.p + (i64)i * slot, (size_t)slot,
                                              hipMemcpyDeviceToHost, st));
                    HIPCHK(hipStreamSynchronize(st));
                    HIPCHK(hipStreamDestroy(st));
                } catch (const std::exception &e) {
                    raw->warm_err = e.what();
                }
            });
        }
        try {
            vector<const int_t *> li(L->Lrowind_bc_ptr, L->Lrowind_bc_ptr + ns),
                ui(L->Ufstnz_br_ptr, L->Ufstnz_br_ptr + ns);
            const auto ta = std::chrono::steady_clock::now();
            P->A.defer_programs = true;
            if (!P->A.build(n_, ns, xsup, li.data(), ui.data(), zero_frac, maxw)) {
                if (P->up_thread.joinable()) P->up_thread.join();
                if (P->alloc_thread.joinable()) P->alloc_thread.join();
                if (P->warm_thread.joinable()) P->warm_thread.join();
                return nullptr;
            }
            SLU_REQUIRE(P->A.lval1 == lv && P->A.uval1 == uv, "amalgamation: value counts");
            P->t_amalg = ms_since(ta);
            tick("analysis");
            // the relayout programs (host pass 4; beside the coarse plan's
            // build it only slowed both down on the box's 16 cores).  Only an
            // upload or a download of the caller-layout values runs them: a
            // plan fed by fill_a whose factors stay in HBM (the device-
            // resident drop-in) builds them when one first happens
            const bool progs_now = P->opts.overlap_upload || P->opts.overlap_download;
            if (progs_now) {
                P->A.build_programs();
                tick("programs (host)");
            }
            P->build_inner();
            tick("coarse plan");
            if (progs_now) {
                P->build_programs();
                P->progs = true;
                tick("relayout programs");
            }
            if (P->opts.overlap_download) P->build_d2h();
            tick("d2h programs");
        } catch (...) {
            if (P->up_thread.joinable()) P->up_thread.join();
            if (P->alloc_thread.joinable()) P->alloc_thread.join();
            if (P->prog_thread.joinable()) P->prog_thread.join();
            if (P->warm_thread.joinable()) P->warm_thread.join();
            throw;
        }
        P->t_plan = ms_since(t0);
        P->sync_stats();
        return P.release();
    }

    void build_inner() {
        const int ns2 = A.ns2;
        mlidx.assign(ns2, nullptr);
        muidx.assign(ns2, nullptr);
        for (int J = 0; J < ns2; ++J) {
            if (A.Loff2[J] >= 0) mlidx[J] = A.Lidx2.data() + A.Loff2[J];
            if (A.Uoff2[J] >= 0) muidx[J] = A.Uidx2.data() + A.Uoff2[J];
        }
        mglu.xsup = A.xsup2.data();
        mglu.supno = A.supno2.data();
        mllu.Lrowind_bc_ptr = mlidx.data();
        mllu.Ufstnz_br_ptr = muidx.data();
        mlu.Glu_persist = &mglu;
        mlu.Llu = &mllu;
        slu_engine_opts io = opts;
        io.overlap_upload = io.overlap_download = 0;
        const auto tj = std::chrono::steady_clock::now();
        if (alloc_thread.joinable()) alloc_thread.join();
        if (getenv("SLU_PROFILE_PLAN"))
            fprintf(stderr, "[slu amalg plan]   (coarse storage: waited %.1f ms)\n", ms_since(tj));
        SLU_REQUIRE(alloc_err.empty(), "%s", alloc_err.c_str());
        in.reset(new Inner(&mlu, n, 1, 1, 0, nullptr, &io, pre));
    }

    // Programs in level order of the coarse plan (so the D2H can compress a
    // level as soon as its panels are done): lx / ublks items of the groups
    // of level L at [lx_lev[L], lx_lev[L+1]) / [ub_lev[L], ub_lev[L+1]).
    vector<int> lx_lev, ub_lev; // (ub_lev: U chunks)
    bool progs = false;         // the relayout programs are built
    void ensure_programs() {
        if (progs) return;
        // (the index pointer tables of the LUstruct as it is now: those
        // make() had are gone; the structure is the plan's by the cache key)
        LocalLU *L = LU->Llu;
        const vector<const int_t *> li(L->Lrowind_bc_ptr, L->Lrowind_bc_ptr + ns),
            ui(L->Ufstnz_br_ptr, L->Ufstnz_br_ptr + ns);
        A.set_index(li.data(), ui.data());
        A.build_programs();
        build_programs();
        progs = true;
    }
    void build_programs() {
        const int nl = (int)in->levels.size();
        auto lev = [&](int s) { return in->level_of[A.grp[s]]; };
        // L: column ranges of <= 64 K values per workgroup
        vector<vector<LColX>> bl(nl);
        for (int s = 0; s < ns; ++s) {
            const Amalg::LCol &C = A.lcols[s];
            if (!C.nsupr) continue;
            const int cpi = std::max(1, (int)(65536 / C.nsupr));
            for (int c0 = 0; c0 < C.w; c0 += cpi)
                bl[lev(s)].push_back({C.src, C.dst, C.map, C.nsupr, c0, std::min(C.w, c0 + cpi), C.ld2});
        }
        vector<LColX> lx;
        lx_lev.assign(nl + 1, 0);
        for (int L = 0; L < nl; ++L) {
            lx.insert(lx.end(), bl[L].begin(), bl[L].end());
            lx_lev[L + 1] = (int)lx.size();
        }
        // U: the original block rows in level order, in chunks of <= 64
        // non-empty columns (chunk counts in order, then the rows in parallel)
        ur_h.clear();
        {
            vector<vector<int>> rows(nl);
            for (int s = 0; s < ns; ++s)
                if (A.urows[s].nc) rows[lev(s)].push_back(s);
            vector<int> order;
            order.reserve(ns);
            vector<i64> first(ns + 1, 0);
            ub_lev.assign(nl + 1, 0);
            i64 nch = 0;
            for (int L = 0; L < nl; ++L) {
                for (int s : rows[L]) {
                    first[order.size()] = nch;
                    order.push_back(s);
                    nch += (A.urows[s].nc + 63) / 64;
                }
                ub_lev[L + 1] = (int)nch;
            }
            ur_h.resize(nch);
            parallel_for((int)order.size(), [&](int i) {
                const Amalg::URowX &R = A.urows[order[i]];
                i64 src = R.src, k = first[i];
                for (int c0 = 0; c0 < R.nc; c0 += 64) {
                    const int nc = std::min(64, R.nc - c0);
                    ur_h[k++] = {src, R.c0 + c0, nc, R.end};
                    for (int c = c0; c < c0 + nc; ++c) src += A.ucl[R.c0 + c] + 1;
                }
            }, 256);
        }
        nlx = (int)lx.size();
        if (lx.empty()) lx.push_back({0, 0, 0, 0, 0, 0, 0});
        if (ur_h.empty()) ur_h.resize(1);
        lx_h = std::move(lx);
        // the tables go up on a helper thread (1.5 GB at 100^3): the first
        // relayout joins it (programs_ready)
        prog_thread = std::thread([this] {
            try {
                HIPCHK(hipSetDevice(0));
                auto up = [](auto &d, const auto &h) { // (a 1-element buffer for an empty table)
                    if (h.empty()) d.alloc(1);
                    else d.upload(h.data(), h.size());
                };
                up(d_lx, lx_h);
                up(d_ur, ur_h);
                up(d_lrow, A.lrow);
                up(d_ucd, A.ucd);
                up(d_ucl, A.ucl);
                up(d_D, A.D);
            } catch (const std::exception &e) {
                prog_err = e.what();
            }
        });
    }
    vector<LColX> lx_h;
    vector<UChunk> ur_h;
    std::thread prog_thread;
    std::string prog_err;
    std::mutex prog_mu;
    void programs_ready() {
        std::lock_guard<std::mutex> lk(prog_mu);
        if (prog_thread.joinable()) prog_thread.join();
        SLU_REQUIRE(prog_err.empty(), "%s", prog_err.c_str());
    }
    int nlx = 0;

    // levels [L0, L1) of the relayout on stream st
    void relayout_levels(int dir, int L0, int L1, hipStream_t st) {
        ensure_programs();
        programs_ready();
        const int a = lx_lev[L0], b = lx_lev[L1];
        if (b > a)
            hipLaunchKernelGGL((k_amalg_l<T>), dim3(b - a), dim3(256), 0, st, d_lx.p + a, d_lrow.p,
                               d_oL.p, in->d_L.p, dir);
        const int u0 = ub_lev[L0], nr = ub_lev[L1] - u0;
        if (nr > 0)
            hipLaunchKernelGGL((k_amalg_u<T>), dim3((unsigned)((nr + 3) / 4)), dim3(256), 0, st,
                               d_ur.p + u0, nr, d_ucd.p, d_ucl.p, d_D.p, (i64)A.DL0, d_oU.p, in->d_L.p,
                               in->d_U.p, dir);
        HIPCHK(hipGetLastError());
    }

    // The overlapped D2H of the drop-in path (opts.overlap_download): the
    // inner plan's pinned-slot pipeline (run_d2h) with fills that carry the
    // caller's layout: a coarse group's members are consecutive supernodes,
    // so its values are one range of d_oL and one of d_oU; before a fill is
    // pushed, d2h_pre compresses every level up to the fill's into d_oL /
    // d_oU on the D2H stream.
    int compressed_to = 0;
    void build_d2h() {
        ensure_o(); // (the push programs address d_oL / d_oU)
        Inner &P = *in;
        warm_join();
        if (warm_stage.p) P.d_stage.swap(warm_stage);
        LocalLU *Llu = LU->Llu;
        const int_t *xsup = LU->Glu_persist->xsup;
        const int nl = (int)P.levels.size();
        if (const char *e = getenv("SLU_D2H_SLOT_KB")) { // as the plain plan
            P.D2H_SLOT = std::max<i64>(16, atoll(e)) << 10;
            P.D2H_MIN = P.D2H_SLOT / 4;
        }
        vector<i64> lsrc(ns + 1, 0);
        for (int s = 0; s < ns; ++s)
            lsrc[s + 1] = lsrc[s] + (Llu->Lrowind_bc_ptr[s] ? (i64)Llu->Lrowind_bc_ptr[s][1] * (xsup[s + 1] - xsup[s]) : 0);
        vector<int> g0(A.ns2 + 1, ns); // first original supernode of each group
        for (int s = ns - 1; s >= 0; --s) g0[A.grp[s]] = s;
        i64 fb = 0;
        int seg0 = 0, hs0 = 0;
        const i64 SLOT = P.D2H_SLOT, PIECE = Inner::D2H_PIECE;
        auto close = [&](int L) {
            if (fb == 0) return;
            P.d2h_fills.push_back({L, seg0, (int)P.h_push.size() - seg0, hs0, (int)P.h_unpack.size() - hs0, fb});
            seg0 = (int)P.h_push.size();
            hs0 = (int)P.h_unpack.size();
            fb = 0;
        };
        auto add = [&](const char *dev, char *host, i64 bytes, int L) {
            i64 done = 0;
            while (done < bytes) {
                const i64 take = std::min(bytes - done, SLOT - fb);
                for (i64 o = 0; o < take; o += PIECE)
                    P.h_push.push_back({dev + done + o, fb + o, (int)std::min(PIECE, take - o)});
                for (i64 o = 0; o < take; o += 4 * PIECE)
                    P.h_unpack.push_back({host + done + o, fb + o, std::min(4 * PIECE, take - o)});
                fb += (take + 15) & ~(i64)15;
                done += take;
                if (fb >= SLOT) close(L);
            }
        };
        // one piece per group and factor where the caller's arrays are
        // contiguous over the group's members (pddistribute's *_dat layout),
        // else one per member
        for (int L = 0; L < nl; ++L) {
            for (int J : P.bylev[L]) {
                for (int pass = 0; pass < 2; ++pass) {
                    const vector<i64> &off = pass ? usrc : lsrc;
                    const T *dbase = pass ? d_oU.p : d_oL.p;
                    auto hptr = [&](int s) -> char * {
                        if (pass) return Llu->Ufstnz_br_ptr[s] ? (char *)Llu->Unzval_br_ptr[s] : nullptr;
                        return Llu->Lrowind_bc_ptr[s] ? (char *)Llu->Lnzval_bc_ptr[s] : nullptr;
                    };
                    int a = g0[J];
                    while (a < g0[J + 1]) {
                        int b = a;
                        while (b < g0[J + 1] && (off[b + 1] == off[b] || !hptr(b))) ++b; // empty
                        if (b == g0[J + 1]) break;
                        char *h0 = hptr(b);
                        int e = b + 1;
                        while (e < g0[J + 1] && (off[e + 1] == off[e] ||
                                                 hptr(e) == h0 + (off[e] - off[b]) * (i64)sizeof(T)))
                            ++e;
                        add((const char *)(dbase + off[b]), h0, (off[e] - off[b]) * (i64)sizeof(T), L);
                        a = e;
                    }
                }
            }
            if (fb >= P.D2H_MIN || L + 1 == nl) close(L);
        }
        P.d_push.upload(P.h_push.empty() ? vector<PushSeg>(1) : P.h_push);
        P.d2h_pre = [this](int L, hipStream_t st) {
            if (L + 1 > compressed_to) {
                relayout_levels(1, compressed_to, L + 1, st);
                compressed_to = L + 1;
            }
        };
        P.opts.overlap_download = 1;
    }

    i64 o_lv = 0, o_uv = 0;
    void ensure_o() {
        std::lock_guard<std::mutex> lk(o_mu);
        if (d_oL.p) return;
        d_oL.alloc(std::max<i64>(o_lv, 1));
        d_oU.alloc(std::max<i64>(o_uv, 1));
    }
    // caller layout: host arrays <-> d_oL / d_oU
    vector<Xfer> xfers() {
        ensure_o();
        LocalLU *L = LU->Llu;
        vector<Xfer> xs;
        const int_t *xsup = LU->Glu_persist->xsup;
        i64 lo = 0;
        for (int s = 0; s < ns; ++s) {
            if (!L->Lrowind_bc_ptr[s]) continue;
            const i64 cnt = (i64)L->Lrowind_bc_ptr[s][1] * (xsup[s + 1] - xsup[s]);
            xs.push_back({(char *)(d_oL.p + lo), (char *)L->Lnzval_bc_ptr[s], (size_t)cnt * sizeof(T)});
            lo += cnt;
        }
        for (int s = 0; s < ns; ++s)
            if (L->Ufstnz_br_ptr[s])
                xs.push_back({(char *)(d_oU.p + usrc[s]), (char *)L->Unzval_br_ptr[s],
                              (size_t)(usrc[s + 1] - usrc[s]) * sizeof(T)});
        return merge_xfers(std::move(xs));
    }
    void h2d() {
        const auto t0 = std::chrono::steady_clock::now();
        vector<Xfer> xs = xfers();
        if (!o_mapped) {
            hipStream_t st = nullptr;
            HIPCHK(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
            HIPCHK(hipMemsetAsync(d_oL.p, 0, sizeof(T), st));
            HIPCHK(hipMemsetAsync(d_oU.p, 0, sizeof(T), st));
            HIPCHK(hipStreamSynchronize(st));
            HIPCHK(hipStreamDestroy(st));
            t_omap = ms_since(t0);
            if (getenv("SLU_PROFILE_PLAN"))
                fprintf(stderr, "[slu amalg plan]   (caller-layout storage %.1f GB mapped in %.1f ms, at %.1f ms)\n",
                        (d_oL.bytes() + d_oU.bytes()) / 1e9, t_omap, ms_since(t_born));
            set_mapped();
        }
        staged_h2d(xs, 0);
        h2d_bytes = 0;
        for (auto &x : xs) h2d_bytes += (double)x.bytes;
        up_ms = ms_since(t0);
    }

    void relayout(int dir) {
        ensure_o();
        hipStream_t st = in->stream;
        if (dir == 0) {
            HIPCHK(hipMemsetAsync(in->d_L.p, 0, in->d_L.bytes(), st));
            HIPCHK(hipMemsetAsync(in->d_U.p, 0, in->d_U.bytes(), st));
        }
        relayout_levels(dir, 0, (int)in->levels.size(), st);
        HIPCHK(hipStreamSynchronize(st));
    }

    void sync_stats() {
        stats = in->stats;
        // the caller's partition's algorithmic work (what the reference's
        // pdgstrf does on this LUstruct); the coarse partition's own counts
        // (explicit zeros included) stay in the kernel-level fields
        // (schur_big_flops, schur_flops_padded)
        const bool cp = sizeof(T) == 16;
        stats.schur_flops = A.fl_schur * (cp ? 4.0 : 1.0);
        stats.panel_flops = (cp ? 6 * A.fl_s1 + 10 * A.fl_w + 8 * A.fl_s2 : A.fl_s1 + 2 * A.fl_s2) +
                            (cp ? 4.0 : 1.0) * A.fl_trsm + A.fl_trsv;
        stats.nsupers_in = ns;
        stats.amalg_groups = A.n_merged_groups;
        stats.amalg_zeros = (double)A.zeros;
        stats.t_amalg_ms = t_amalg;
        stats.t_plan_ms = t_plan;
        stats.t_upload_ms = up_ms;
        stats.h2d_bytes = h2d_bytes;
        stats.t_expand_ms = t_expand;
        stats.t_compress_ms = t_compress;
        stats.t_d2h_ms = t_d2h;
        stats.d2h_bytes = (double)(d_oL.bytes() + d_oU.bytes());
    }

    void upload() override {
        const auto t0 = std::chrono::steady_clock::now();
        if (up_thread.joinable()) {
            up_thread.join();
            if (!up_err.empty()) {
                std::string e;
                e.swap(up_err);
                throw Error(e);
            }
        } else {
            h2d();
        }
        const auto t1 = std::chrono::steady_clock::now();
        relayout(0);
        t_expand = ms_since(t1);
        in->vstate = 1;
        in->d_acur = nullptr;
        in->host_current = false;
        coarse_current = false;
        host_done = false;
        sync_stats();
        stats.t_upload_wait_ms = std::chrono::duration<double, std::milli>(t1 - t0).count();
    }
    void adopt_factors() override {
        upload();
        in->sync();
        in->vstate = 2;
        coarse_current = true;
        host_done = true; // the caller's arrays hold these factors already
    }
    void factor(double anorm, int *info, int *tiny) override {
        compressed_to = 0;
        in->factor(anorm, info, tiny);
        // overlap_download: the caller's arrays already hold the factors
        coarse_current = !in->host_current;
        host_done = in->host_current;
        sync_stats();
        if (host_done) {
            stats.t_d2h_ms = in->stats.t_d2h_ms;
            stats.t_d2h_tail_ms = in->stats.t_d2h_tail_ms;
            stats.d2h_bytes = in->stats.d2h_bytes;
            stats.n_d2h_copies = in->stats.n_d2h_copies;
        }
    }
    bool host_done = false;
    void download() override {
        in->sync();
        if (host_done) return;
        if (coarse_current) {
            const auto t0 = std::chrono::steady_clock::now();
            relayout(1);
            t_compress = ms_since(t0);
            coarse_current = false;
        }
        const auto t0 = std::chrono::steady_clock::now();
        for (const Xfer &x : xfers()) HIPCHK(hipMemcpy(x.host, x.dev, x.bytes, hipMemcpyDeviceToHost));
        t_d2h = ms_since(t0);
        sync_stats();
    }
    void snapshot() override { in->snapshot(); }
    void restore() override {
        in->restore();
        coarse_current = true;
        host_done = false;
    }
    void sync() override { in->sync(); }
    void set_timing(int timing, int serial) override { in->set_timing(timing, serial); }
    void solve(void *b, int64_t ldb, int nrhs) override {
        in->solve(b, ldb, nrhs);
        sync_stats();
    }
    void set_a_pattern(int64_t ncol, const int64_t *xa, const int64_t *asub) override {
        in->set_a_pattern(ncol, xa, asub);
        sync_stats();
    }
    void fill_a(const void *a, int on_device) override {
        in->fill_a(a, on_device);
        coarse_current = true;
        host_done = false;
        sync_stats();
    }
    void refine(const void *b, void *x, int64_t ld, int nrhs, double *berr, int *steps) override {
        in->refine(b, x, ld, nrhs, berr, steps);
        sync_stats();
    }
    void check_exchange(int64_t *nsec, int64_t *nbytes) override { in->check_exchange(nsec, nbytes); }
    ~AmalgPlan() override {
        if (up_thread.joinable()) up_thread.join();
        if (alloc_thread.joinable()) alloc_thread.join();
        if (prog_thread.joinable()) prog_thread.join();
        if (warm_thread.joinable()) warm_thread.join();
    }
};

// ------------------------------------------------------------ grid amalgamation
// The coarse partition on a Pr x Pc grid (csrc/amalg.h, "grids"): the
// analysis runs on the ranks' supernode ranges, every fine block goes to
// the owner of its coarse block (structure once, values at every upload and
// back at download), and the inner Plan -- the ordinary grid plan -- runs on
// each rank's local coarse LUstruct with the caller's communicator.  The
// value relayout on the device: pack (k_amalg_l over the caller's L with a
// row map, k_ranges over its U blocks) into one send buffer ordered by
// destination, one section per ordered rank pair over the transport (RCCL
// send / receive on the world communicator, or the host transports), unpack
// (k_amalg_l / k_amalg_u) into the zeroed coarse storage; download runs the
// same programs backwards.
template <typename T, typename HT, typename LocalLU, typename LUS>
struct GridAmalgPlan : PlanBase {
    using Inner = Plan<T, HT, LocalLU, LUS>;
    LUS *LU = nullptr;
    int n = 0, ns = 0, Pr = 1, Pc = 1, iam = 0, P = 1;
    slu_comm *comm = nullptr;
    slu_engine_opts opts{};
    bool dry = false;
    GaFine f;
    vector<const int_t *> flidx, fuidx;
    GaChains ch;
    GaPartition g;
    GaRelay r;
    vector<vector<i64>> cnt; // cnt[p][q]: values rank p sends rank q
    // the coarse LUstruct the inner plan reads (index arrays only)
    LUS mlu{};
    LocalLU mllu{};
    Glu_persist_t mglu{};
    vector<int_t *> mlidx, muidx;
    std::unique_ptr<Inner> in;
    Xport X;
    hipStream_t xs = nullptr; // plan-time exchanges before the inner plan exists
    // device: caller layout, send / receive buffers, programs
    DevBuf<T> d_oL, d_oU, d_send, d_recv;
    DevBuf<LColX> d_pl, d_ul;
    DevBuf<int32_t> d_plrow, d_ulrow, d_uucd;
    DevBuf<uint16_t> d_uucl;
    DevBuf<GaSpan> d_pu;
    DevBuf<UChunk> d_uu;
    DevBuf<i64> d_D;
    double t_relay_plan = 0, t_expand = 0, t_compress = 0, t_h2d = 0, t_d2h = 0;
    bool coarse_current = false;

    static double ms_since(std::chrono::steady_clock::time_point t0) {
        return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
    }

    // nullptr when nothing merges (every rank decides the same: the
    // partition is all-gathered)
    static GridAmalgPlan *make(LUS *lu, int n_, int pr, int pc, int iam_, slu_comm *c,
                               const slu_engine_opts *o, double zero_frac, int maxw) {
        const auto t0 = std::chrono::steady_clock::now();
        std::unique_ptr<GridAmalgPlan> G(new GridAmalgPlan);
        G->LU = lu;
        G->n = n_;
        G->Pr = pr;
        G->Pc = pc;
        G->P = pr * pc;
        G->iam = iam_;
        G->comm = c;
        if (o) G->opts = *o;
        G->dry = G->opts.schedule_only != 0;
        SLU_REQUIRE(c && (c->world || c->host_fn || c->host_p2p), "a %dx%d grid needs a communicator", pr, pc);
        SLU_REQUIRE(G->P <= 32, "grid amalgamation: at most 32 ranks");
        if (!G->dry) {
            HIPCHK(hipSetDevice(c->device));
            HIPCHK(hipStreamCreateWithFlags(&G->xs, hipStreamNonBlocking));
        }
        G->X.c = c;
        G->X.s = G->xs;
        G->X.host_mem = G->dry;
        LocalLU *L = lu->Llu;
        GaFine &f = G->f;
        f.n = n_;
        f.ns = G->ns = (int)(lu->Glu_persist->supno[n_ - 1] + 1);
        f.Pr = pr;
        f.Pc = pc;
        f.myrow = iam_ / pc;
        f.mycol = iam_ % pc;
        f.xsup = lu->Glu_persist->xsup;
        G->flidx.assign(L->Lrowind_bc_ptr, L->Lrowind_bc_ptr + f.nlc());
        G->fuidx.assign(L->Ufstnz_br_ptr, L->Ufstnz_br_ptr + f.nlr());
        f.lidx = G->flidx.data();
        f.uidx = G->fuidx.data();
        // 1. structure to the analysis owners, chains of my range
        G->ch = ga_analyse(f, G->X.alltoallv(ga_structure_out(f)), zero_frac, maxw);
        // 2. the partition
        G->g = ga_partition(f, G->X.allgatherv(G_WORLD, G->ch.gstart));
        if (G->g.ns2 == G->ns) return nullptr;
        // 3. relayout: my pieces' structure to the coarse owners, my coarse
        // LUstruct and programs from what arrives; everybody's counts
        ga_send_side(f, G->g, G->r);
        ga_receive_side(f, G->g, G->X.alltoallv(G->r.sstruct), G->r);
        G->cnt = G->X.allgatherv(G_WORLD, G->r.scount);
        for (int p = 0; p < G->P; ++p)
            SLU_REQUIRE(G->cnt[p][iam_] == G->r.rcount[p], "grid amalgamation: counts %d -> %d", p, iam_);
        G->t_relay_plan = ms_since(t0);
        G->build_inner();
        if (!G->dry) G->build_programs();
        G->sync_stats();
        G->stats.t_plan_ms = ms_since(t0);
        return G.release();
    }

    void build_inner() {
        mlidx.assign(r.nlc2, nullptr);
        muidx.assign(r.nlr2, nullptr);
        for (int j = 0; j < r.nlc2; ++j)
            if (!r.Lidx2[j].empty()) mlidx[j] = r.Lidx2[j].data();
        for (int j = 0; j < r.nlr2; ++j)
            if (!r.Uidx2[j].empty()) muidx[j] = r.Uidx2[j].data();
        mglu.xsup = g.xsup2.data();
        mglu.supno = g.supno2.data();
        mllu.Lrowind_bc_ptr = mlidx.data();
        mllu.Ufstnz_br_ptr = muidx.data();
        mlu.Glu_persist = &mglu;
        mlu.Llu = &mllu;
        slu_engine_opts io = opts;
        io.overlap_upload = io.overlap_download = 0;
        in.reset(new Inner(&mlu, n, Pr, Pc, iam, comm, &io));
        if (!dry) X.s = in->stream; // the relayout's sections go on the kernels' stream
    }

    template <typename V> static void up(DevBuf<V> &d, const vector<V> &h) {
        if (h.empty()) d.upload(vector<V>(1));
        else d.upload(h);
    }
    void build_programs() {
        up(d_pl, r.pack_l);
        up(d_plrow, r.pack_lrow);
        up(d_pu, r.pack_u);
        up(d_ul, r.unpack_l);
        up(d_ulrow, r.unpack_lrow);
        up(d_uu, r.unpack_u);
        up(d_uucd, r.unpack_ucd);
        up(d_uucl, r.unpack_ucl);
        up(d_D, r.D);
        d_send.alloc(std::max<i64>(r.soff[P], 1));
        d_recv.alloc(std::max<i64>(r.received, 1));
    }
    void ensure_o() {
        if (d_oL.p) return;
        d_oL.alloc(std::max<i64>(r.lval, 1));
        d_oU.alloc(std::max<i64>(r.uval, 1));
    }
    // the caller's local values <-> d_oL / d_oU
    vector<Xfer> xfers() {
        ensure_o();
        LocalLU *L = LU->Llu;
        vector<Xfer> v;
        for (int j = 0; j < f.nlc(); ++j)
            if (L->Lrowind_bc_ptr[j] && r.lsrc[j + 1] > r.lsrc[j])
                v.push_back({(char *)(d_oL.p + r.lsrc[j]), (char *)L->Lnzval_bc_ptr[j],
                             (size_t)(r.lsrc[j + 1] - r.lsrc[j]) * sizeof(T)});
        for (int j = 0; j < f.nlr(); ++j)
            if (L->Ufstnz_br_ptr[j] && r.usrc[j + 1] > r.usrc[j])
                v.push_back({(char *)(d_oU.p + r.usrc[j]), (char *)L->Unzval_br_ptr[j],
                             (size_t)(r.usrc[j + 1] - r.usrc[j]) * sizeof(T)});
        return merge_xfers(std::move(v));
    }

    void launch_l(const DevBuf<LColX> &items, size_t nitems, const DevBuf<int32_t> &lrow, T *o, T *m, int dir,
                  hipStream_t st) {
        if (nitems)
            hipLaunchKernelGGL((k_amalg_l<T>), dim3((unsigned)nitems), dim3(256), 0, st, items.p, lrow.p, o, m, dir);
    }
    // the value all-to-all: forward p -> q from send to receive regions,
    // backward q -> p the other way; my own pair is a device copy
    void exchange(bool forward) {
        hipStream_t st = in->stream;
        const int me = iam;
        if (r.scount[me])
            HIPCHK(hipMemcpyAsync(forward ? d_recv.p + r.roff[me] : d_send.p + r.soff[me],
                                  forward ? d_send.p + r.soff[me] : d_recv.p + r.roff[me],
                                  (size_t)r.scount[me] * sizeof(T), hipMemcpyDeviceToDevice, st));
        for (int p = 0; p < P; ++p)
            for (int q = 0; q < P; ++q) {
                if (p == q || !cnt[p][q]) continue;
                const int root = forward ? p : q, dest = forward ? q : p;
                T *buf = nullptr;
                if (me == p) buf = d_send.p + r.soff[q];
                else if (me == q) buf = d_recv.p + r.roff[p];
                X.section(G_WORLD, root, 1u << dest, buf, (size_t)cnt[p][q] * sizeof(T));
            }
        X.phase = forward ? "grid amalgamation relayout (values to the coarse owners)"
                          : "grid amalgamation relayout (factors back to the caller layout)";
        X.flush();
        X.phase = "plan-time exchange";
    }

    void expand() { // caller layout (d_oL / d_oU) -> coarse
        const auto t0 = std::chrono::steady_clock::now();
        hipStream_t st = in->stream;
        launch_l(d_pl, r.pack_l.size(), d_plrow, d_send.p, d_oL.p, 1, st);
        if (!r.pack_u.empty())
            hipLaunchKernelGGL((k_ranges<T>), dim3((unsigned)((r.pack_u.size() + 255) / 256)), dim3(256), 0, st,
                               d_pu.p, (int)r.pack_u.size(), d_oU.p, d_send.p, 0);
        HIPCHK(hipGetLastError());
        exchange(true);
        HIPCHK(hipMemsetAsync(in->d_L.p, 0, in->d_L.bytes(), st));
        HIPCHK(hipMemsetAsync(in->d_U.p, 0, in->d_U.bytes(), st));
        launch_l(d_ul, r.unpack_l.size(), d_ulrow, d_recv.p, in->d_L.p, 0, st);
        if (!r.unpack_u.empty())
            hipLaunchKernelGGL((k_amalg_u<T>), dim3((unsigned)((r.unpack_u.size() + 3) / 4)), dim3(256), 0, st,
                               d_uu.p, (int)r.unpack_u.size(), d_uucd.p, d_uucl.p, d_D.p, (i64)r.DL0, d_recv.p, in->d_L.p,
                               in->d_U.p, 0);
        HIPCHK(hipGetLastError());
        HIPCHK(hipStreamSynchronize(st));
        t_expand = ms_since(t0);
    }
    void compress() { // coarse -> caller layout
        const auto t0 = std::chrono::steady_clock::now();
        hipStream_t st = in->stream;
        launch_l(d_ul, r.unpack_l.size(), d_ulrow, d_recv.p, in->d_L.p, 1, st);
        if (!r.unpack_u.empty())
            hipLaunchKernelGGL((k_amalg_u<T>), dim3((unsigned)((r.unpack_u.size() + 3) / 4)), dim3(256), 0, st,
                               d_uu.p, (int)r.unpack_u.size(), d_uucd.p, d_uucl.p, d_D.p, (i64)r.DL0, d_recv.p, in->d_L.p,
                               in->d_U.p, 1);
        HIPCHK(hipGetLastError());
        exchange(false);
        launch_l(d_pl, r.pack_l.size(), d_plrow, d_send.p, d_oL.p, 0, st);
        if (!r.pack_u.empty())
            hipLaunchKernelGGL((k_ranges<T>), dim3((unsigned)((r.pack_u.size() + 255) / 256)), dim3(256), 0, st,
                               d_pu.p, (int)r.pack_u.size(), d_oU.p, d_send.p, 1);
        HIPCHK(hipGetLastError());
        HIPCHK(hipStreamSynchronize(st));
        t_compress = ms_since(t0);
    }

    void sync_stats() {
        stats = in->stats;
        const bool cp = sizeof(T) == 16;
        const AmalgFlops &F = ch.fl; // my analysis range's share of the caller partition's work
        stats.schur_flops = F.schur * (cp ? 4.0 : 1.0);
        stats.panel_flops = (cp ? 6 * F.s1 + 10 * F.w + 8 * F.s2 : F.s1 + 2 * F.s2) +
                            (cp ? 4.0 : 1.0) * F.trsm + F.trsv;
        stats.nsupers_in = ns;
        i64 groups = 0;
        for (size_t i = 0; i < ch.gstart.size(); ++i) {
            const i64 e = i + 1 < ch.gstart.size() ? ch.gstart[i + 1]
                                                   : (i64)ga_range(ns, P, iam + 1);
            groups += e - ch.gstart[i] > 1;
        }
        stats.amalg_groups = groups;
        stats.t_amalg_ms = t_relay_plan;
        stats.t_expand_ms = t_expand;
        stats.t_compress_ms = t_compress;
        stats.t_upload_ms = t_h2d;
        stats.t_d2h_ms = t_d2h;
        stats.h2d_bytes = (double)(r.lval + r.uval) * sizeof(T);
        stats.d2h_bytes = stats.h2d_bytes;
    }

    void upload() override {
        const auto t0 = std::chrono::steady_clock::now();
        staged_h2d(xfers(), comm->device);
        t_h2d = ms_since(t0);
        expand();
        in->vstate = 1;
        in->d_acur = nullptr;
        in->host_current = false;
        coarse_current = false;
        sync_stats();
    }
    void adopt_factors() override {
        upload();
        in->sync();
        in->vstate = 2;
    }
    void factor(double anorm, int *info, int *tiny) override {
        in->factor(anorm, info, tiny);
        coarse_current = true;
        sync_stats();
    }
    void download() override {
        in->sync();
        if (coarse_current) {
            ensure_o();
            compress();
            coarse_current = false;
        }
        const auto t0 = std::chrono::steady_clock::now();
        for (const Xfer &x : xfers()) HIPCHK(hipMemcpy(x.host, x.dev, x.bytes, hipMemcpyDeviceToHost));
        t_d2h = ms_since(t0);
        sync_stats();
    }
    void snapshot() override { in->snapshot(); }
    void restore() override {
        in->restore();
        coarse_current = true;
    }
    void sync() override { in->sync(); }
    void set_timing(int timing, int serial) override { in->set_timing(timing, serial); }
    void solve(void *b, int64_t ldb, int nrhs) override {
        in->solve(b, ldb, nrhs);
        sync_stats();
    }
    void set_a_pattern(int64_t ncol, const int64_t *xa, const int64_t *asub) override {
        in->set_a_pattern(ncol, xa, asub);
        sync_stats();
    }
    void fill_a(const void *a, int on_device) override {
        in->fill_a(a, on_device);
        coarse_current = true;
        sync_stats();
    }
    void refine(const void *b, void *x, int64_t ld, int nrhs, double *berr, int *steps) override {
        in->refine(b, x, ld, nrhs, berr, steps);
        sync_stats();
    }
    void check_exchange(int64_t *nsec, int64_t *nbytes) override {
        in->check_exchange(nsec, nbytes);
        sync_stats();
    }
    ~GridAmalgPlan() override {
        in.reset();
        if (xs) (void)hipStreamDestroy(xs);
    }
};

// The plan for a caller's LUstruct: the amalgamated one when chains merge
// (1x1: AmalgPlan; 2D grids: GridAmalgPlan; SLU_AMALG=0 turns it off;
// SLU_AMALG_ZERO sets the explicit zero fraction, default 0.10), else the
// plain plan.  3D grids factor the caller's partition (its forests).
template <typename P> PlanBase *make_plan_any(void *LU, int n, int pr, int pc, int iam, slu_comm *c,
                                              const slu_engine_opts *o) {
    using A = AmalgPlan<typename P::value_type, typename P::host_type, typename P::local_type,
                        typename P::lus_type>;
    using GA = GridAmalgPlan<typename P::value_type, typename P::host_type, typename P::local_type,
                             typename P::lus_type>;
    const char *e = getenv("SLU_AMALG");
    const bool on = !(e && !strcmp(e, "0"));
    const char *z = getenv("SLU_AMALG_ZERO");
    const double zf = z ? atof(z) : 0.10;
    if (on && pr * pc == 1 && !(o && o->schedule_only) && !(c && c->npdep > 1)) {
        if (PlanBase *p = A::make((typename P::lus_type *)LU, n, o, zf, FAST_MAXW)) return p;
    } else if (on && pr * pc > 1 && !(c && c->npdep > 1)) {
        if (PlanBase *p = GA::make((typename P::lus_type *)LU, n, pr, pc, iam, c, o, zf, FAST_MAXW)) return p;
    }
    return make_plan<P>(LU, n, pr, pc, iam, c, o);
}

} // namespace slu

struct slu_plan {
    int dtype = 0;
    std::unique_ptr<slu::PlanBase> impl;
};

using namespace slu;

// Fills the whole LDS of every CU with NaN (test hook: a kernel that reads
// LDS it did not write, even to multiply it by zero, then fails every time
// instead of depending on what the previous kernel left there).
__global__ void __launch_bounds__(1024) k_poison_lds(double v, int bytes) {
    extern __shared__ double s_poison[];
    const int n = bytes / (int)sizeof(double);
    for (int i = threadIdx.x; i < n; i += blockDim.x) s_poison[i] = v;
    __syncthreads();
    if (s_poison[(threadIdx.x * 7) % n] != s_poison[(threadIdx.x * 7) % n] && threadIdx.x == 1u << 30)
        s_poison[0] = 0; // never true; keeps the stores
}

extern "C" {

int slu_debug_poison_lds(int device) {
    try {
        HIPCHK(hipSetDevice(device));
        // the whole 160 KB per workgroup where the runtime allows it, else 64 KB
        int bytes = 160 * 1024;
        if (hipFuncSetAttribute((const void *)k_poison_lds,
                                hipFuncAttributeMaxDynamicSharedMemorySize, bytes) != hipSuccess) {
            (void)hipGetLastError();
            bytes = 64 * 1024;
        }
        hipLaunchKernelGGL(k_poison_lds, dim3(4096), dim3(1024), bytes, 0, __builtin_nan(""), bytes);
        HIPCHK(hipGetLastError());
        HIPCHK(hipDeviceSynchronize());
        return 0;
    } catch (const std::exception &e) {
        set_last_error(e.what());
        return -1;
    }
}

const char *slu_last_error(void) { return g_last_error.c_str(); }

int slu_comm_unique_id(void *uid) {
    try {
        ncclUniqueId id;
        NCCLCHK(ncclGetUniqueId(&id));
        memcpy(uid, &id, sizeof id);
        return 0;
    } catch (const std::exception &e) {
        set_last_error(e.what());
        return -1;
    }
}

slu_comm *slu_comm_create(const void *uid, int nprow, int npcol, int iam, int device) {
    try {
        auto *c = new slu_comm;
        c->nprow = nprow;
        c->npcol = npcol;
        c->iam = iam;
        c->myrow = iam / npcol;
        c->mycol = iam % npcol;
        c->device = device;
        HIPCHK(hipSetDevice(device));
        if (nprow * npcol > 1) {
            SLU_REQUIRE(uid != nullptr, "uid required for a %dx%d grid", nprow, npcol);
            ncclUniqueId id;
            memcpy(&id, uid, sizeof id);
            NCCLCHK(ncclCommInitRank(&c->world, nprow * npcol, id, iam));
            NCCLCHK(ncclCommSplit(c->world, c->myrow, c->mycol, &c->row, nullptr));
            NCCLCHK(ncclCommSplit(c->world, c->mycol, c->myrow, &c->col, nullptr));
        }
        return c;
    } catch (const std::exception &e) {
        set_last_error(e.what());
        return nullptr;
    }
}

slu_comm *slu_comm_create3d(const void *uid, int nprow, int npcol, int npdep, int iam3d, int device) {
    try {
        const int P = nprow * npcol;
        SLU_REQUIRE(nprow > 0 && npcol > 0 && npdep > 0 && (npdep & (npdep - 1)) == 0,
                    "3D grid %dx%dx%d: Pz must be a power of two", nprow, npcol, npdep);
        SLU_REQUIRE(iam3d >= 0 && iam3d < P * npdep, "rank %d outside a %dx%dx%d grid", iam3d, nprow,
                    npcol, npdep);
        auto *c = new slu_comm;
        c->nprow = nprow;
        c->npcol = npcol;
        c->npdep = npdep;
        c->zlayer = iam3d / P;
        c->iam = iam3d % P;
        c->myrow = c->iam / npcol;
        c->mycol = c->iam % npcol;
        c->device = device;
        HIPCHK(hipSetDevice(device));
        if (P * npdep > 1) {
            SLU_REQUIRE(uid != nullptr, "uid required for a %dx%dx%d grid", nprow, npcol, npdep);
            ncclUniqueId id;
            memcpy(&id, uid, sizeof id);
            NCCLCHK(ncclCommInitRank(&c->all, P * npdep, id, iam3d));
            NCCLCHK(ncclCommSplit(c->all, c->zlayer, c->iam, &c->world, nullptr));
            NCCLCHK(ncclCommSplit(c->all, c->iam, c->zlayer, &c->zcomm, nullptr));
            NCCLCHK(ncclCommSplit(c->world, c->myrow, c->mycol, &c->row, nullptr));
            NCCLCHK(ncclCommSplit(c->world, c->mycol, c->myrow, &c->col, nullptr));
        }
        return c;
    } catch (const std::exception &e) {
        set_last_error(e.what());
        return nullptr;
    }
}

slu_comm *slu_comm_create_host_p2p3d(slu_host_p2p_fn fn, void *ctx, int nprow, int npcol, int npdep,
                                     int iam3d, int device) {
    try {
        SLU_REQUIRE(npdep > 0 && (npdep & (npdep - 1)) == 0, "Pz = %d is not a power of two", npdep);
        slu_comm *c = slu_comm_create_host_p2p(fn, ctx, nprow, npcol, iam3d % (nprow * npcol), device);
        if (!c) return nullptr;
        c->npdep = npdep;
        c->zlayer = iam3d / (nprow * npcol);
        return c;
    } catch (const std::exception &e) {
        set_last_error(e.what());
        return nullptr;
    }
}

slu_comm *slu_comm_create_host(slu_host_bcast_fn fn, void *ctx, int nprow, int npcol, int iam,
                               int device) {
    try {
        SLU_REQUIRE(fn != nullptr, "host transport needs a broadcast callback");
        auto *c = new slu_comm;
        c->nprow = nprow;
        c->npcol = npcol;
        c->iam = iam;
        c->myrow = iam / npcol;
        c->mycol = iam % npcol;
        c->device = device;
        c->host_fn = fn;
        c->host_ctx = ctx;
        HIPCHK(hipSetDevice(device));
        return c;
    } catch (const std::exception &e) {
        set_last_error(e.what());
        return nullptr;
    }
}

slu_comm *slu_comm_create_host_p2p(slu_host_p2p_fn fn, void *ctx, int nprow, int npcol, int iam,
                                   int device) {
    try {
        SLU_REQUIRE(fn != nullptr, "point-to-point host transport needs a callback");
        auto *c = new slu_comm;
        c->nprow = nprow;
        c->npcol = npcol;
        c->iam = iam;
        c->myrow = iam / npcol;
        c->mycol = iam % npcol;
        c->device = device;
        c->host_p2p = fn;
        c->host_ctx = ctx;
        if (device >= 0) HIPCHK(hipSetDevice(device)); // -1: schedule-only plans, no GPU
        return c;
    } catch (const std::exception &e) {
        set_last_error(e.what());
        return nullptr;
    }
}

int slu_comm_size(const slu_comm *c, int group) {
    if (!c) return -1;
    if (c->world || c->zcomm) { // what RCCL itself reports for the communicator
        int n = -1;
        ncclComm_t cm = group == 0 ? c->world : group == 1 ? c->row : group == 2 ? c->col : c->zcomm;
        if (!cm) return 1;
        if (ncclCommCount(cm, &n) != ncclSuccess) return -1;
        return n;
    }
    return group == 0 ? c->nprow * c->npcol : group == 1 ? c->npcol : group == 2 ? c->nprow : c->npdep;
}

void slu_comm_destroy(slu_comm *c) {
    if (!c) return;
    c->wd.reset(); // (its thread polls the communicators)
    if (c->row) ncclCommDestroy(c->row);
    if (c->col) ncclCommDestroy(c->col);
    if (c->world) ncclCommDestroy(c->world);
    if (c->zcomm) ncclCommDestroy(c->zcomm);
    if (c->all) ncclCommDestroy(c->all);
    delete c;
}

slu_plan *slu_plan_create(int dtype, void *LU, int n, int nprow, int npcol, int iam,
                          slu_comm *comm, const slu_engine_opts *opts, char *err, int errlen) {
    try {
        auto *p = new slu_plan;
        p->dtype = dtype;
        switch (dtype) {
        case SLU_D:
            p->impl.reset(make_plan_any<Plan<double, double, dLocalLU_t, dLUstruct_t>>(LU, n, nprow, npcol, iam, comm, opts));
            break;
        case SLU_S:
            p->impl.reset(make_plan_any<Plan<float, float, sLocalLU_t, sLUstruct_t>>(LU, n, nprow, npcol, iam, comm, opts));
            break;
        case SLU_Z:
            p->impl.reset(make_plan_any<Plan<zc, doublecomplex, zLocalLU_t, zLUstruct_t>>(LU, n, nprow, npcol, iam, comm, opts));
            break;
        default:
            throw Error(fmt("bad dtype %d", dtype));
        }
        return p;
    } catch (const std::exception &e) {
        set_last_error(e.what());
        if (err && errlen > 0) snprintf(err, errlen, "%s", e.what());
        return nullptr;
    }
}

int slu_plan_gather3d(slu_plan *p) {
    try {
        p->impl->gather_layers();
        return 0;
    } catch (const std::exception &e) {
        set_last_error(e.what());
        return -1;
    }
}

int slu_plan_adopt_factors(slu_plan *p) {
    try {
        p->impl->adopt_factors();
        return 0;
    } catch (const std::exception &e) {
        set_last_error(e.what());
        return -1;
    }
}

int slu_plan_upload(slu_plan *p) {
    try {
        p->impl->upload();
        return 0;
    } catch (const std::exception &e) {
        set_last_error(e.what());
        return -1;
    }
}

int slu_plan_factor(slu_plan *p, double anorm, int *info, int *tiny) {
    try {
        int i = 0, t = 0;
        p->impl->factor(anorm, &i, &t);
        if (info) *info = i;
        if (tiny) *tiny = t;
        return 0;
    } catch (const std::exception &e) {
        set_last_error(e.what());
        return -1;
    }
}

int slu_plan_solve(slu_plan *p, void *b, int64_t ldb, int nrhs) {
    try {
        p->impl->solve(b, ldb, nrhs);
        return 0;
    } catch (const std::exception &e) {
        set_last_error(e.what());
        return -1;
    }
}

int slu_plan_set_a_pattern(slu_plan *p, int64_t ncol, const int64_t *xa, const int64_t *asub) {
    try {
        p->impl->set_a_pattern(ncol, xa, asub);
        return 0;
    } catch (const std::exception &e) {
        set_last_error(e.what());
        return -1;
    }
}

int slu_plan_fill_a(slu_plan *p, const void *a, int on_device) {
    try {
        p->impl->fill_a(a, on_device);
        return 0;
    } catch (const std::exception &e) {
        set_last_error(e.what());
        return -1;
    }
}

int slu_plan_refine(slu_plan *p, const void *b, void *x, int64_t ld, int nrhs, double *berr,
                    int *steps) {
    try {
        p->impl->refine(b, x, ld, nrhs, berr, steps);
        return 0;
    } catch (const std::exception &e) {
        set_last_error(e.what());
        return -1;
    }
}

int slu_plan_download(slu_plan *p) {
    try {
        p->impl->download();
        return 0;
    } catch (const std::exception &e) {
        set_last_error(e.what());
        return -1;
    }
}

int slu_plan_snapshot(slu_plan *p) {
    try {
        p->impl->snapshot();
        return 0;
    } catch (const std::exception &e) {
        set_last_error(e.what());
        return -1;
    }
}

int slu_plan_restore(slu_plan *p) {
    try {
        p->impl->restore();
        return 0;
    } catch (const std::exception &e) {
        set_last_error(e.what());
        return -1;
    }
}

int slu_plan_check_exchange(slu_plan *p, int64_t *nsections, int64_t *nbytes) {
    try {
        p->impl->check_exchange(nsections, nbytes);
        return 0;
    } catch (const std::exception &e) {
        set_last_error(e.what());
        return -1;
    }
}

int slu_plan_set_timing(slu_plan *p, int timing, int serial) {
    try {
        p->impl->set_timing(timing, serial);
        return 0;
    } catch (const std::exception &e) {
        set_last_error(e.what());
        return -1;
    }
}

int slu_plan_sync(slu_plan *p) {
    try {
        p->impl->sync();
        return 0;
    } catch (const std::exception &e) {
        set_last_error(e.what());
        return -1;
    }
}

void slu_plan_destroy(slu_plan *p) { delete p; }

int slu_plan_get_stats(const slu_plan *p, slu_plan_stats *st) {
    *st = p->impl->stats;
    return 0;
}

} // extern "C"

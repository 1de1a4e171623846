// Drop-in C ABI: pdgstrf / psgstrf / pzgstrf and the scatter helpers the
// reference's pdgstrf.c.o exports.
//
// pxgstrf(options, m, n, anorm, LUstruct, grid, stat, info) keeps the
// reference contract (SRC/pdgstrf.c:242-402, 1927-1931):
//   * m < 0 -> info = -2, n < 0 -> info = -3, message as pxerr_dist, return -1;
//   * m == 0 || n == 0 -> return 0;
//   * factors are written back in place into LUstruct->Llu's host arrays;
//   * stat->ops[FACT] = algorithmic flops, stat->TinyPivots += replacements,
//     stat->num_look_aheads = clamp(options->num_lookaheads, 0, 49);
//   * *info = MIN over ranks of the rank's zero-pivot column (0 if none).
// It must be called by every rank of grid->comm.  On multi-rank grids MPI
// bootstraps RCCL (or, with several ranks per GPU, carries the host-staged
// panel broadcasts) and reduces info; its symbols are looked up in the host
// process at run time (this library has no link-time MPI dependency).  A 1x1
// grid makes no MPI call.
#include <dlfcn.h>
#include <execinfo.h>
#include <hip/hip_runtime.h>
#include <signal.h>
#include <sys/resource.h>
#include <unistd.h>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <map>
#include <future>
#include <mutex>
#include <set>
#include <thread>
#include <vector>

#include "common.h"
#include "slu_mi355x.h"

namespace {

using i64 = int64_t;

// MPI is resolved from the host process at run time (no link-time MPI).
struct Mpi {
    int (*bcast)(void *, int, MPI_Datatype, int, MPI_Comm) = nullptr;
    int (*allreduce)(const void *, void *, int, MPI_Datatype, MPI_Op, MPI_Comm) = nullptr;
    int (*allgather)(const void *, int, MPI_Datatype, void *, int, MPI_Datatype, MPI_Comm) = nullptr;
    int (*create_keyval)(MPI_Comm_copy_attr_function *, MPI_Comm_delete_attr_function *, int *,
                         void *) = nullptr;
    int (*set_attr)(MPI_Comm, int, void *) = nullptr;
    int (*get_attr)(MPI_Comm, int, void *, int *) = nullptr;
    int (*isend)(const void *, int, MPI_Datatype, int, int, MPI_Comm, MPI_Request *) = nullptr;
    int (*irecv)(void *, int, MPI_Datatype, int, int, MPI_Comm, MPI_Request *) = nullptr;
    int (*waitall)(int, MPI_Request *, MPI_Status *) = nullptr;
};

template <typename F> void mpi_sym(F &f, const char *name) {
    f = (F)dlsym(RTLD_DEFAULT, name);
    if (!f) throw slu::Error(slu::fmt("MPI symbol %s not found in the process", name));
}

const Mpi &mpi() {
    static Mpi m = [] {
        Mpi x;
        mpi_sym(x.bcast, "MPI_Bcast");
        mpi_sym(x.allreduce, "MPI_Allreduce");
        mpi_sym(x.allgather, "MPI_Allgather");
        mpi_sym(x.create_keyval, "MPI_Comm_create_keyval");
        mpi_sym(x.set_attr, "MPI_Comm_set_attr");
        mpi_sym(x.get_attr, "MPI_Comm_get_attr");
        mpi_sym(x.isend, "MPI_Isend");
        mpi_sym(x.irecv, "MPI_Irecv");
        mpi_sym(x.waitall, "MPI_Waitall");
        return x;
    }();
    return m;
}

// The HSA runtime seeds and draws libc rand() when it creates a queue (every
// HIP stream, RCCL's too).  The reference's pddistribute draws the seeds of
// its solve's broadcast / reduction trees from rand() on every rank
// (SRC/pddistribute.c:1557, 1729) and needs every rank to draw the same
// sequence: a rank whose sequence moved builds other trees than its peers,
// and pdgstrs then returns garbage on every later system in the process.
// Every entry point therefore runs on a private random() state and hands the
// caller's back untouched (tests/test_dropin.py, the grid life-cycle tests).
struct CallerRandState {
    char buf[256];
    char *prev;
    CallerRandState() : prev(initstate(1u, buf, sizeof buf)) {}
    ~CallerRandState() { setstate(prev); }
    CallerRandState(const CallerRandState &) = delete;
    CallerRandState &operator=(const CallerRandState &) = delete;
};

// SUPERLU_MI355X_SEGV_TRACE=1 (diagnostics): a host backtrace on SIGSEGV
void segv_trace(int sig) {
    void *fr[64];
    const int n = backtrace(fr, 64);
    static const char msg[] = "[slu] SIGSEGV, host backtrace:\n";
    (void)!write(2, msg, sizeof msg - 1);
    backtrace_symbols_fd(fr, n, 2);
    signal(sig, SIG_DFL);
    raise(sig);
}
void maybe_trace_segv() {
    const char *e = getenv("SUPERLU_MI355X_SEGV_TRACE");
    if (e && atoi(e) == 1) signal(SIGSEGV, segv_trace);
}

int pick_device(int iam) {
    const char *e = getenv("SUPERLU_DEVICE");
    if (e) return atoi(e);
    int nd = 0;
    if (hipGetDeviceCount(&nd) != hipSuccess || nd <= 0)
        throw slu::Error("no HIP device visible: the MI355X engine needs a GPU");
    const char *lr = getenv("MPI_LOCALRANKID");
    if (!lr) lr = getenv("OMPI_COMM_WORLD_LOCAL_RANK");
    if (!lr) lr = getenv("LOCAL_RANK");
    int r = lr ? atoi(lr) : iam;
    return r % nd;
}

// The engine's communicators for one gridinfo_t, cached on grid->comm as an
// MPI attribute: the delete callback runs when superlu_gridexit frees the
// communicator, so a later grid can never pick up a stale entry (MPICH
// reuses freed handle values).  Transport: RCCL when every rank drives its
// own GPU; MPI broadcasts of host-staged buffers on grid->comm / rscp / cscp
// (SRC/superlu_grid.c:158-172) when several ranks share one (RCCL refuses
// duplicate devices) or SUPERLU_MI355X_TRANSPORT=mpi.
struct GridComm {
    slu_comm *c = nullptr;
    int nprow = 0, npcol = 0, iam = -1;
    MPI_Comm comms[3]; // grid, process row, process column
    bool host = false;
    int64_t nbc[3] = {0, 0, 0}, nbytes[3] = {0, 0, 0}; // host broadcasts per group
};

int mpi_host_bcast(void *ctx, int group, int root, void *buf, int64_t bytes) {
    GridComm *g = (GridComm *)ctx;
    char *p = (char *)buf;
    ++g->nbc[group];
    g->nbytes[group] += bytes;
    while (bytes > 0) {
        const int n = (int)std::min<int64_t>(bytes, 1 << 30);
        if (mpi().bcast(p, n, MPI_BYTE, root, g->comms[group]) != MPI_SUCCESS) return 1;
        p += n;
        bytes -= n;
    }
    return 0;
}

void evict_for_comm(slu_comm *c); // (plan cache, below)

int grid_attr_delete(MPI_Comm, int, void *val, void *) {
    CallerRandState rs;
    GridComm *g = (GridComm *)val;
    evict_for_comm(g->c); // a cached plan must never outlive its transport
    slu_comm_destroy(g->c);
    delete g;
    return MPI_SUCCESS;
}

std::mutex g_mu;
int g_keyval = MPI_KEYVAL_INVALID;
std::map<int, slu_comm *> g_single; // 1x1 grids (no MPI at all), per device

slu_comm *comm_for_grid(gridinfo_t *grid) {
    std::lock_guard<std::mutex> lk(g_mu);
    const int nprow = (int)grid->nprow, npcol = (int)grid->npcol;
    if (nprow * npcol == 1) {
        const int dev = pick_device(0);
        auto it = g_single.find(dev);
        if (it != g_single.end()) return it->second;
        slu_comm *c = slu_comm_create(nullptr, 1, 1, 0, dev);
        if (!c) throw slu::Error(slu_last_error());
        return g_single[dev] = c;
    }
    const Mpi &M = mpi();
    if (g_keyval == MPI_KEYVAL_INVALID)
        M.create_keyval(MPI_COMM_NULL_COPY_FN, grid_attr_delete, &g_keyval, nullptr);
    void *val = nullptr;
    int flag = 0;
    M.get_attr(grid->comm, g_keyval, &val, &flag);
    if (flag) {
        GridComm *g = (GridComm *)val;
        if (g->nprow == nprow && g->npcol == npcol && g->iam == grid->iam) return g->c;
    }
    // collective from here on: every rank of grid->comm takes the same path
    const int dev = pick_device(grid->iam), P = nprow * npcol;
    std::vector<int> devs(P, -1);
    M.allgather(&dev, 1, MPI_INT, devs.data(), 1, MPI_INT, grid->comm);
    std::vector<int> sorted(devs);
    std::sort(sorted.begin(), sorted.end());
    bool host = std::adjacent_find(sorted.begin(), sorted.end()) != sorted.end();
    if (const char *t = getenv("SUPERLU_MI355X_TRANSPORT")) host = !strcmp(t, "mpi");
    auto *g = new GridComm;
    g->nprow = nprow;
    g->npcol = npcol;
    g->iam = grid->iam;
    g->comms[0] = grid->comm;
    g->comms[1] = grid->rscp.comm;
    g->comms[2] = grid->cscp.comm;
    g->host = host;
    if (host) {
        g->c = slu_comm_create_host(mpi_host_bcast, g, nprow, npcol, grid->iam, dev);
    } else {
        unsigned char uid[128] = {0};
        if (grid->iam == 0 && slu_comm_unique_id(uid) != 0) throw slu::Error(slu_last_error());
        M.bcast(uid, 128, MPI_BYTE, 0, grid->comm);
        g->c = slu_comm_create(uid, nprow, npcol, grid->iam, dev);
    }
    if (!g->c) {
        delete g;
        throw slu::Error(slu_last_error());
    }
    M.set_attr(grid->comm, g_keyval, g); // replaces (and deletes) a stale entry
    return g->c;
}

// SLU_BCAST_TRACE=1 (diagnostics): every rank's host-broadcast count and
// bytes per group so far, compared across each group's members
void trace_bcasts(gridinfo_t *grid, const char *where) {
    const char *e = getenv("SLU_BCAST_TRACE");
    if (!e || atoi(e) != 1 || grid->nprow * grid->npcol == 1) return;
    const Mpi &M = mpi();
    void *val = nullptr;
    int flag = 0;
    M.get_attr(grid->comm, g_keyval, &val, &flag);
    if (!flag) return;
    GridComm *g = (GridComm *)val;
    const char *gn[3] = {"grid", "row", "column"};
    for (int k = 0; k < 3; ++k) {
        int P = 0;
        int64_t mine[2] = {g->nbc[k], g->nbytes[k]};
        const int sz = k == 0 ? (int)(grid->nprow * grid->npcol) : k == 1 ? (int)grid->npcol : (int)grid->nprow;
        P = sz;
        std::vector<int64_t> all(2 * (size_t)P);
        M.allgather(mine, 2, MPI_LONG_LONG, all.data(), 2, MPI_LONG_LONG, g->comms[k]);
        bool same = true;
        for (int q = 1; q < P; ++q) same = same && all[2 * q] == all[0] && all[2 * q + 1] == all[1];
        fprintf(stderr, "[slu bcast %s] rank %d %s group: %lld broadcasts, %lld bytes%s\n", where, (int)grid->iam,
                gn[k], (long long)mine[0], (long long)mine[1], same ? "" : "  MISMATCH in this group");
    }
}

// The plan's HBM (the factors' device copy, index tables, staging) is
// released on a helper thread once the factors are back in the host arrays:
// hipFree of ~17 GB costs ~0.1 s that the caller's utime[FACT] need not pay.
// The next call, and process exit, wait for it.
std::mutex g_reap_mu;
std::thread g_reaper;
void reap_join() {
    std::lock_guard<std::mutex> lk(g_reap_mu);
    if (g_reaper.joinable()) g_reaper.join();
}
void reap_later(slu_plan *p) {
    static bool registered = false;
    std::lock_guard<std::mutex> lk(g_reap_mu);
    if (g_reaper.joinable()) g_reaper.join();
    if (!registered) {
        atexit(reap_join);
        registered = true;
    }
    int dev = 0;
    (void)hipGetDevice(&dev);
    g_reaper = std::thread([p, dev] {
        (void)hipSetDevice(dev);
        slu_plan_destroy(p);
    });
}

// ---- plan cache.  pdgssvx refactors one pattern with Fact = SamePattern /
// SamePattern_SameRowPerm (SRC/superlu_defs.h:577-598): the LUstruct's index
// arrays are the same, only the values differ.  The last plan is kept (with
// its HBM) and reused when the structure digest matches, so such a call pays
// upload + factor + download only; on a grid every rank reuses or every rank
// rebuilds (the digest covers grid->comm: the plan holds its transport).
// The digest hashes every index array, except under Fact =
// SamePattern_SameRowPerm: there the caller reuses "the L & U data structures
// set up from the previous factorization" (SRC/superlu_defs.h:590-598,
// pdgssvx skips symbfact and pddistribute only refills values,
// SRC/pddistribute.c:545-672), and a shallow digest (the LUstruct's tables,
// every block's pointers and header words) suffices.
// SUPERLU_MI355X_PLAN_CACHE=0 frees the plan after every call, as the
// reference frees its buffers.
struct CachedPlan {
    slu_plan *plan = nullptr;
    uint64_t digest = 0, shallow = 0;
    int dtype = -1, n = -1, replace_tiny = -1;
    const void *lu = nullptr; // the LUstruct the cached factors belong to (pdgstrs)
    struct Key {
        const void *lu, *llu, *lrow;
        bool operator==(const Key &o) const { return lu == o.lu && llu == o.llu && lrow == o.lrow; }
    } key{};
    bool a_pattern = false;   // the plan holds DevA's pattern (fill_a ready)
    uint64_t a_pattern_gen = 0; // ... of this DevA pattern generation
    bool host_factors = true; // the host L / U arrays hold these factors
    slu_comm *comm = nullptr; // the transport the plan was built with (grid->comm's)
};
CachedPlan g_cache;
std::mutex g_cache_mu;

// LUstructs whose factors lived only in the HBM of a cached plan that a later
// pdgstrf evicted (the host L / U arrays still hold A's values).  The plan
// cannot write them back at eviction: the caller may have destroyed the
// LUstruct by then (dDestroy_LU frees its arrays without telling this
// library).  A pdgstrs on such an LUstruct fails loudly instead of solving
// with A as if it were its factors; a new pdgstrf / pddistribute on it clears
// the mark.  Guarded by g_cache_mu.
using LuKey = CachedPlan::Key;
std::vector<LuKey> g_evicted;
template <typename LUS> LuKey lu_key(LUS *lu) {
    return {lu, lu->Llu, lu->Llu ? (const void *)lu->Llu->Lrowind_bc_ptr : nullptr};
}
void unmark_evicted(const LuKey &k) {
    g_evicted.erase(std::remove(g_evicted.begin(), g_evicted.end(), k), g_evicted.end());
}
// the cache entry goes: its plan is reaped, device-only factors are marked
void evict_cached() {
    if (!g_cache.plan) return;
    if (!g_cache.host_factors) g_evicted.push_back(g_cache.key);
    reap_later(g_cache.plan);
    g_cache.plan = nullptr;
}

// superlu_gridexit frees grid->comm, whose attribute delete callback destroys
// the engine communicators: a cached plan built on them goes first, and
// synchronously (a reaper thread could still be in the plan while the
// communicators are torn down).  Without this a later grid whose comm handle
// and LUstruct land on the same addresses would hit the cache and call into
// the freed transport.
void evict_for_comm(slu_comm *c) {
    slu_plan *p = nullptr;
    {
        std::lock_guard<std::mutex> lk(g_cache_mu);
        if (!g_cache.plan || g_cache.comm != c) return;
        if (!g_cache.host_factors) g_evicted.push_back(g_cache.key);
        p = g_cache.plan;
        g_cache.plan = nullptr;
    }
    reap_join();
    slu_plan_destroy(p);
}

// A in the LUstruct's coordinates (CSC), kept by this library's pddistribute
// for the pdgstrf that follows: the factor storage is then built on the
// device (zero + scatter of A's nnz values, the plan's fill_a) instead of
// copying the distributed L / U values over PCIe, and on a 1x1 grid the
// factors stay in HBM for this library's pdgstrs (the host L / U arrays keep
// A's values unless SUPERLU_MI355X_HOST_FACTORS=1).  Keyed by the LUstruct
// and its index tables, so an LUstruct distributed elsewhere never matches.
struct DevA {
    const void *lu = nullptr, *llu = nullptr, *lrow = nullptr;
    int dtype = -1;
    int64_t n = 0;
    std::vector<int64_t> xa, asub;
    std::vector<char> a; // nnz values of the dtype
    uint64_t gen = 0;         // bumps with every stash (values)
    uint64_t pattern_gen = 0; // bumps with every first-time distribute (pattern, perm_r)
};
DevA g_deva;
std::mutex g_deva_mu;
uint64_t g_deva_gen = 0;
// LocalLU_t of the LUstructs whose pddistribute left A's values out of the
// host arrays (SUPERLU_MI355X_DEFER_A, default on for fp64 unless
// SUPERLU_MI355X_HOST_FACTORS=1): their pdgstrf needs g_deva to hold their A
std::set<const void *> g_host_a_deferred;

inline uint64_t mix(uint64_t h, uint64_t v) {
    h ^= v + 0x9E3779B97F4A7C15ull + (h << 6) + (h >> 2);
    return h * 0xBF58476D1CE4E5B9ull;
}

// digest of this rank's structure: xsup and every local L / U index array
// (host threads), the grid, and where the values live
template <typename LUS> uint64_t structure_digest(LUS *lu, int n, const gridinfo_t *grid) {
    const int_t *xsup = lu->Glu_persist->xsup;
    const int ns = (int)(lu->Glu_persist->supno[n - 1] + 1);
    const int Pr = (int)grid->nprow, Pc = (int)grid->npcol;
    const int nlc = (ns + Pc - 1) / Pc, nlr = (ns + Pr - 1) / Pr, nb = std::max(nlc, nlr);
    std::vector<uint64_t> part(nb);
    auto idx = [](const int_t *ix, i64 len) {
        uint64_t h = 0x12345;
        for (i64 i = 0; i < len; ++i) h = mix(h, (uint64_t)ix[i]);
        return h;
    };
    slu::parallel_for(nb, [&](int j) {
        uint64_t h = (uint64_t)j;
        if (j < nlc)
            if (const int_t *ix = lu->Llu->Lrowind_bc_ptr[j]) {
                i64 p = SLU_BC_HEADER;
                for (i64 b = 0; b < ix[0]; ++b) p += SLU_LB_DESCRIPTOR + ix[p + 1];
                h = mix(h, idx(ix, p));
                // and where the values live: a plan keeps host pointers (the
                // D2H unpack targets), so another LUstruct of the same
                // pattern is a miss
                h = mix(h, (uint64_t)(uintptr_t)lu->Llu->Lnzval_bc_ptr[j]);
            }
        if (j < nlr)
            if (const int_t *ux = lu->Llu->Ufstnz_br_ptr[j]) {
                h = mix(h, idx(ux, ux[2]));
                h = mix(h, (uint64_t)(uintptr_t)lu->Llu->Unzval_br_ptr[j]);
            }
        part[j] = h;
    });
    uint64_t h = mix((uint64_t)n, (uint64_t)ns);
    for (int j = 0; j <= ns; ++j) h = mix(h, (uint64_t)xsup[j]); // every global xsup entry
    h = mix(h, (uint64_t)(uintptr_t)lu);
    h = mix(h, (uint64_t)(uintptr_t)lu->Llu);
    h = mix(h, ((uint64_t)Pr << 32) | (uint64_t)Pc);
    h = mix(h, (uint64_t)grid->iam);
    h = mix(h, (uint64_t)(uintptr_t)grid->comm); // (the plan holds this grid's transport)
    for (uint64_t v : part) h = mix(h, v);
    return h;
}

// the shallow digest: the tables, every local block's index / value pointers
// and header words, the grid (O(blocks), no index array is read through)
template <typename LUS> uint64_t shallow_digest(LUS *lu, int n, const gridinfo_t *grid) {
    const int_t *xsup = lu->Glu_persist->xsup;
    const int ns = (int)(lu->Glu_persist->supno[n - 1] + 1);
    const int Pr = (int)grid->nprow, Pc = (int)grid->npcol;
    const int nlc = (ns + Pc - 1) / Pc, nlr = (ns + Pr - 1) / Pr, nb = std::max(nlc, nlr);
    constexpr int CH = 4096;
    std::vector<uint64_t> part((nb + CH - 1) / CH);
    auto *L = lu->Llu;
    slu::parallel_for((int)part.size(), [&](int c) {
        uint64_t h = (uint64_t)c;
        for (int j = c * CH; j < std::min(nb, (c + 1) * CH); ++j) {
            if (j < nlc) {
                const int_t *ix = L->Lrowind_bc_ptr[j];
                h = mix(h, (uint64_t)(uintptr_t)ix);
                h = mix(h, (uint64_t)(uintptr_t)L->Lnzval_bc_ptr[j]);
                if (ix) h = mix(mix(h, (uint64_t)ix[0]), (uint64_t)ix[1]);
            }
            if (j < nlr) {
                const int_t *ux = L->Ufstnz_br_ptr[j];
                h = mix(h, (uint64_t)(uintptr_t)ux);
                h = mix(h, (uint64_t)(uintptr_t)L->Unzval_br_ptr[j]);
                if (ux) h = mix(mix(mix(h, (uint64_t)ux[0]), (uint64_t)ux[1]), (uint64_t)ux[2]);
            }
        }
        part[c] = h;
    }, 1);
    uint64_t h = mix(mix((uint64_t)n, (uint64_t)ns), 0x5A11u);
    for (int j = 0; j <= ns; ++j) h = mix(h, (uint64_t)xsup[j]); // every global xsup entry
    h = mix(h, (uint64_t)(uintptr_t)lu);
    h = mix(h, (uint64_t)(uintptr_t)L);
    h = mix(h, (uint64_t)(uintptr_t)L->Lrowind_bc_ptr);
    h = mix(h, (uint64_t)(uintptr_t)L->Ufstnz_br_ptr);
    h = mix(h, ((uint64_t)Pr << 32) | (uint64_t)Pc);
    h = mix(h, (uint64_t)grid->iam);
    h = mix(h, (uint64_t)(uintptr_t)grid->comm);
    for (uint64_t v : part) h = mix(h, v);
    return h;
}

// every rank of the grid reuses its cached plan, or none does (building a
// plan is collective)
bool all_ranks(bool mine, gridinfo_t *grid) {
    if (grid->nprow * grid->npcol == 1) return mine;
    int in = mine ? 1 : 0, out = 0;
    mpi().allreduce(&in, &out, 1, MPI_INT, MPI_MIN, grid->comm);
    return out == 1;
}

// process CPU time (all threads) and thread count, for SUPERLU_MI355X_TIMING
double process_cpu_ms() {
    struct rusage ru;
    getrusage(RUSAGE_SELF, &ru);
    return (ru.ru_utime.tv_sec + ru.ru_stime.tv_sec) * 1e3 + (ru.ru_utime.tv_usec + ru.ru_stime.tv_usec) * 1e-3;
}
int process_threads() {
    FILE *f = fopen("/proc/self/status", "r");
    if (!f) return -1;
    char line[256];
    int t = -1;
    while (fgets(line, sizeof line, f))
        if (!strncmp(line, "Threads:", 8)) t = atoi(line + 8);
    fclose(f);
    return t;
}

template <typename LUS>
int_t pxgstrf(int dtype, const char *name, superlu_dist_options_t *options, int m, int n,
              double anorm, LUS *LUstruct, gridinfo_t *grid, SuperLUStat_t *stat, int *info) {
    *info = 0;
    if (m < 0) *info = -2;
    else if (n < 0) *info = -3;
    if (*info) {
        printf("{%lld,%lld}: On entry to %6s, parameter number %lld had an illegal value\n",
               (long long)(grid->iam / grid->npcol), (long long)(grid->iam % grid->npcol), name,
               (long long)-*info);
        return -1;
    }
    if (m == 0 || n == 0) return 0;
    stat->ops[SLU_PHASE_FACT] = 0.0f;
    stat->current_buffer = stat->peak_buffer = stat->gpu_buffer = 0.0f;
    stat->num_look_aheads = std::max(0, std::min(options->num_lookaheads, SLU_MAX_LOOKAHEADS - 1));
    // SUPERLU_MI355X_FACTOR_SKIP=1 (test hook, no GPU needed): return at once,
    // the LUstruct untouched -- the distribute / destroy ownership test runs
    // the reference's p?gssvx around this library's p?distribute on the CPU
    if (const char *sk = getenv("SUPERLU_MI355X_FACTOR_SKIP"); sk && atoi(sk) == 1) {
        fprintf(stderr, "%s (MI355X library): SUPERLU_MI355X_FACTOR_SKIP=1 is set: test hook, the "
                        "LUstruct is NOT factored\n", name);
        return 0;
    }
    slu_plan *plan = nullptr;
    // SUPERLU_MI355X_TIMING=1: wall-clock breakdown of the call on stderr
    const char *tm = getenv("SUPERLU_MI355X_TIMING");
    const bool timing = tm && atoi(tm) == 1;
    using clk = std::chrono::steady_clock;
    clk::time_point tp[6];
    tp[0] = clk::now();
    try {
        const bool one = grid->nprow * grid->npcol == 1;
        const char *pc = getenv("SUPERLU_MI355X_PLAN_CACHE");
        const bool cache = !(pc && !strcmp(pc, "0"));
        const int rt = options->ReplaceTinyPivot == SLU_YES;
        uint64_t dg = 0, sdg = 0;
        // a miss on the shallow digest is a miss: the full digest is then
        // only stored with the new plan, and is computed beside the upload and
        // the factorization (beside the plan build it took memory bandwidth
        // and cores from the analysis passes)
        std::future<uint64_t> dg_later;
        bool dg_needed = false;
        // this grid's transport (collective only when it is created): a cached
        // plan is reused only on the communicators it was built with
        slu_comm *const gcomm = comm_for_grid(grid);
        if (cache) {
            sdg = shallow_digest(LUstruct, n, grid);
            bool hit;
            {
                std::lock_guard<std::mutex> lk(g_cache_mu);
                hit = g_cache.plan && g_cache.shallow == sdg && g_cache.key == lu_key(LUstruct) &&
                      g_cache.dtype == dtype && g_cache.n == n && g_cache.replace_tiny == rt &&
                      g_cache.comm == gcomm;
                if (hit) dg = g_cache.digest;
            }
            // Fact = SamePattern_SameRowPerm: the previous factorization's L & U
            // structures, by contract; otherwise every index array is hashed
            if (hit && options->Fact != SLU_SAMEPATTERN_SAMEROWPERM) {
                const uint64_t full = structure_digest(LUstruct, n, grid);
                hit = full == dg;
                dg = full;
            } else if (!hit) {
                dg_needed = true;
            }
            hit = all_ranks(hit, grid);
            std::lock_guard<std::mutex> lk(g_cache_mu);
            if (hit) {
                plan = g_cache.plan; // same structure: reuse (values are uploaded again below)
                g_cache.plan = nullptr;
            } else {
                evict_cached();
            }
        }
        {
            std::lock_guard<std::mutex> lk(g_cache_mu);
            unmark_evicted(lu_key(LUstruct)); // this call writes its factors anew
        }
        // built by this library's pddistribute: A is at hand for a device fill
        DevA *da = nullptr;
        {
            std::lock_guard<std::mutex> lk(g_deva_mu);
            if (g_deva.lu == LUstruct && g_deva.llu == LUstruct->Llu &&
                g_deva.lrow == LUstruct->Llu->Lrowind_bc_ptr && g_deva.dtype == dtype && g_deva.n == n)
                da = &g_deva;
        }
        if (!da) {
            std::lock_guard<std::mutex> lk(g_deva_mu);
            if (g_host_a_deferred.count(LUstruct->Llu))
                throw slu::Error("this LUstruct was distributed with A's values kept for the device fill "
                                 "(not placed in the host arrays), and another pddistribute has replaced "
                                 "that A since: call pddistribute again, or set SUPERLU_MI355X_DEFER_A=0");
        }
        const char *hf = getenv("SUPERLU_MI355X_HOST_FACTORS");
        const bool keep_on_device = one && da && cache && !(hf && atoi(hf) == 1);
        bool pattern_ready = false;
        const bool reused = plan != nullptr;
        tp[1] = clk::now();
        const double cpu1 = timing ? process_cpu_ms() : 0;
        if (plan && da) {
            // the plan's A-to-factor map holds for the pattern it was built
            // from: a new pddistribute (new perm_r, same index arrays) bumps
            // the pattern generation and the map is built again
            std::lock_guard<std::mutex> lk(g_cache_mu);
            pattern_ready = g_cache.a_pattern && g_cache.a_pattern_gen == da->pattern_gen;
        }
        if (!plan) {
            reap_join(); // the previous call's device memory is free again
            slu_comm *c = gcomm;
            slu_engine_opts eo{};
            eo.replace_tiny_pivot = rt;
            // utime[FACT] (SRC/pdgssvx.c:1174-1180) covers the copies too: the
            // H2D of the values runs beside the plan build, and each level's
            // finished factors go back to the host arrays while later levels
            // are factored (SUPERLU_MI355X_OVERLAP=0 turns both off).  With A
            // at hand nothing but A goes up, and on 1x1 nothing comes down.
            const char *ov = getenv("SUPERLU_MI355X_OVERLAP");
            const bool ovl = !(ov && !strcmp(ov, "0"));
            eo.overlap_upload = ovl && !da;
            eo.overlap_download = ovl && !keep_on_device;
            eo.timing = timing; // device-time breakdown for SUPERLU_MI355X_TIMING
            char err[512] = {0};
            plan = slu_plan_create(dtype, LUstruct, n, (int)grid->nprow, (int)grid->npcol,
                                   grid->iam, c, &eo, err, sizeof err);
            if (!plan) throw slu::Error(err);
        }
        if (dg_needed)
            dg_later = std::async(std::launch::async, [LUstruct, n, grid] {
                return structure_digest(LUstruct, n, grid);
            });
        int myinfo = 0, tiny = 0;
        tp[2] = clk::now();
        const double cpu2 = timing ? process_cpu_ms() : 0;
        if (da) {
            if (!pattern_ready &&
                slu_plan_set_a_pattern(plan, n, da->xa.data(), da->asub.data()))
                throw slu::Error(slu_last_error());
            pattern_ready = true;
            if (slu_plan_fill_a(plan, da->a.data(), 0)) throw slu::Error(slu_last_error());
        } else if (slu_plan_upload(plan)) {
            throw slu::Error(slu_last_error());
        }
        tp[3] = clk::now();
        if (slu_plan_factor(plan, anorm, &myinfo, &tiny)) throw slu::Error(slu_last_error());
        tp[4] = clk::now();
        if (!keep_on_device && slu_plan_download(plan)) throw slu::Error(slu_last_error());
        tp[5] = clk::now();
        slu_plan_stats st;
        slu_plan_get_stats(plan, &st);
        if (timing) {
            auto ms = [&](int a, int b) {
                return std::chrono::duration<double, std::milli>(tp[b] - tp[a]).count();
            };
            fprintf(stderr,
                    "[%s rank %d] digest %.1f ms, plan %s %.1f ms (amalg %.1f; process cpu %.0f ms, "
                    "%d threads), %s %.1f ms "
                    "(device fill %.1f, upload wait %.1f), factor %.1f ms (device %.1f: diag %.1f, "
                    "trsm %.1f, schur %.1f), download %.1f ms (tail %.1f)%s\n",
                    name, (int)grid->iam, ms(0, 1), reused ? "reused" : "built", ms(1, 2),
                    st.t_amalg_ms, cpu2 - cpu1, process_threads(), da ? "fill_a" : "upload", ms(2, 3), st.t_fill_ms,
                    st.t_upload_wait_ms, ms(3, 4), st.t_total_ms, st.t_diag_ms, st.t_trsm_ms,
                    st.t_schur_ms, ms(4, 5), st.t_d2h_tail_ms,
                    keep_on_device ? " [factors kept in HBM]" : "");
        }
        stat->ops[SLU_PHASE_FACT] = (float)(st.schur_flops + st.panel_flops);
        stat->TinyPivots += tiny;
        stat->gpu_buffer = (float)(st.lu_bytes + st.index_bytes);
        if (dg_later.valid()) dg = dg_later.get();
        if (cache) {
            std::lock_guard<std::mutex> lk(g_cache_mu);
            g_cache.plan = plan;
            g_cache.digest = dg;
            g_cache.shallow = sdg;
            g_cache.dtype = dtype;
            g_cache.n = n;
            g_cache.replace_tiny = rt;
            g_cache.lu = LUstruct;
            g_cache.a_pattern = pattern_ready;
            g_cache.a_pattern_gen = da ? da->pattern_gen : 0;
            g_cache.host_factors = !keep_on_device;
            g_cache.key = lu_key(LUstruct);
            g_cache.comm = gcomm;
        } else {
            reap_later(plan);
        }
        plan = nullptr;
        trace_bcasts(grid, name);
        int gi = myinfo ? myinfo : n + 1;
        if (grid->nprow * grid->npcol > 1) {
            int in = gi;
            mpi().allreduce(&in, &gi, 1, MPI_INT, MPI_MIN, grid->comm);
        }
        *info = gi == n + 1 ? 0 : gi;
        return 0;
    } catch (const std::exception &e) {
        if (plan) slu_plan_destroy(plan);
        fprintf(stderr, "%s (MI355X engine): %s\n", name, e.what());
        fflush(stderr);
        abort(); // the reference ABORTs on internal failures (SRC/util_dist.h ABORT)
    }
}

// ------------------------------------------------------------------ 3D
// pdgstrf3d (SRC/pdgstrf3d.c:121-392): the engine's 3D plan on
// each rank's LUstruct of its layer, with the caller's forest partition
// (trf3Dpartition->supernode2treeMap, built by dinitTrf3Dpartition, which
// also zeroed the ancestor blocks this layer does not own).  Communicators
// cached on grid3d->comm: RCCL when every rank drives its own GPU, else the
// point-to-point host transport over MPI_Isend / MPI_Irecv on the layer's
// grid2d.comm / rscp / cscp and on zscp (the same send / receive pairs the
// RCCL transport issues, host-staged).
struct Grid3Comm {
    slu_comm *c = nullptr;
    int nprow = 0, npcol = 0, npdep = 0, iam = -1;
    MPI_Comm comms[4]; // layer, process row, process column, z
};

int mpi_host_p2p(void *ctx, int nops, const slu_host_p2p_op *ops) {
    Grid3Comm *g = (Grid3Comm *)ctx;
    std::vector<MPI_Request> rq;
    for (int i = 0; i < nops; ++i) {
        char *p = (char *)ops[i].buf;
        int64_t left = ops[i].bytes;
        while (left > 0) { // pieces of <= 1 GiB, matched in order
            const int cnt = (int)std::min<int64_t>(left, 1 << 30);
            MPI_Request r;
            const MPI_Comm cm = g->comms[ops[i].group];
            const int rc = ops[i].send ? mpi().isend(p, cnt, MPI_BYTE, ops[i].peer, 7301, cm, &r)
                                       : mpi().irecv(p, cnt, MPI_BYTE, ops[i].peer, 7301, cm, &r);
            if (rc != MPI_SUCCESS) return 1;
            rq.push_back(r);
            p += cnt;
            left -= cnt;
        }
    }
    if (!rq.empty() && mpi().waitall((int)rq.size(), rq.data(), MPI_STATUSES_IGNORE) != MPI_SUCCESS)
        return 1;
    return 0;
}

int grid3_attr_delete(MPI_Comm, int, void *val, void *) {
    CallerRandState rs;
    Grid3Comm *g = (Grid3Comm *)val;
    slu_comm_destroy(g->c);
    delete g;
    return MPI_SUCCESS;
}
int g_keyval3 = MPI_KEYVAL_INVALID;

// SUPERLU_MI355X_SCHEDULE_ONLY=1 (test hook, no GPU needed): pdgstrf3d builds
// schedule-only plans over the MPI point-to-point transport, replays every
// exchange of the factorization with checked bytes (slu_plan_check_exchange)
// and returns without factoring.
bool schedule_only_3d() {
    const char *e = getenv("SUPERLU_MI355X_SCHEDULE_ONLY");
    return e && atoi(e) == 1;
}

slu_comm *comm_for_grid3d(gridinfo3d_t *g3) {
    std::lock_guard<std::mutex> lk(g_mu);
    const Mpi &M = mpi();
    if (g_keyval3 == MPI_KEYVAL_INVALID)
        M.create_keyval(MPI_COMM_NULL_COPY_FN, grid3_attr_delete, &g_keyval3, nullptr);
    const int nprow = (int)g3->nprow, npcol = (int)g3->npcol, npdep = (int)g3->npdep;
    void *val = nullptr;
    int flag = 0;
    M.get_attr(g3->comm, g_keyval3, &val, &flag);
    if (flag) {
        Grid3Comm *g = (Grid3Comm *)val;
        if (g->nprow == nprow && g->npcol == npcol && g->npdep == npdep && g->iam == g3->iam)
            return g->c;
    }
    SLU_REQUIRE(g3->rankorder == 0, "pdgstrf3d: only the default Z-major rank order");
    const int P = nprow * npcol * npdep;
    const bool dry = schedule_only_3d();
    const int dev = dry ? -1 : pick_device(g3->iam);
    std::vector<int> devs(P, -1);
    M.allgather(&dev, 1, MPI_INT, devs.data(), 1, MPI_INT, g3->comm);
    std::vector<int> sorted(devs);
    std::sort(sorted.begin(), sorted.end());
    bool host = dry || std::adjacent_find(sorted.begin(), sorted.end()) != sorted.end();
    if (const char *t = getenv("SUPERLU_MI355X_TRANSPORT")) host = host || !strcmp(t, "mpi");
    auto *g = new Grid3Comm;
    g->nprow = nprow;
    g->npcol = npcol;
    g->npdep = npdep;
    g->iam = g3->iam;
    g->comms[0] = g3->grid2d.comm;
    g->comms[1] = g3->grid2d.rscp.comm;
    g->comms[2] = g3->grid2d.cscp.comm;
    g->comms[3] = g3->zscp.comm;
    // the engine's 3D rank is layer * Pr * Pc + the rank in the layer's grid
    const int iam3 = g3->zscp.Iam * nprow * npcol + g3->grid2d.iam;
    if (host) {
        g->c = slu_comm_create_host_p2p3d(mpi_host_p2p, g, nprow, npcol, npdep, iam3, dev);
    } else {
        unsigned char uid[128] = {0};
        if (g3->iam == 0 && slu_comm_unique_id(uid) != 0) throw slu::Error(slu_last_error());
        M.bcast(uid, 128, MPI_BYTE, 0, g3->comm);
        g->c = slu_comm_create3d(uid, nprow, npcol, npdep, iam3, dev);
    }
    if (!g->c) {
        delete g;
        throw slu::Error(slu_last_error());
    }
    M.set_attr(g3->comm, g_keyval3, g);
    return g->c;
}

template <typename LUS>
int_t pxgstrf3d(int dtype, const char *name, superlu_dist_options_t *options, int m, int n,
                double anorm, dtrf3Dpartition_t *trf, LUS *LUstruct, gridinfo3d_t *g3,
                SuperLUStat_t *stat, int *info) {
    gridinfo_t *grid = &g3->grid2d;
    *info = 0;
    if (m < 0) *info = -2;
    else if (n < 0) *info = -3;
    if (*info) {
        printf("{%lld,%lld}: On entry to %6s, parameter number %lld had an illegal value\n",
               (long long)(grid->iam / grid->npcol), (long long)(grid->iam % grid->npcol), name,
               (long long)-*info);
        return -1;
    }
    if (m == 0 || n == 0) return 0;
    stat->ops[SLU_PHASE_FACT] = 0.0f;
    stat->current_buffer = stat->peak_buffer = stat->gpu_buffer = 0.0f;
    stat->num_look_aheads = std::max(0, std::min(options->num_lookaheads, SLU_MAX_LOOKAHEADS - 1));
    slu_plan *plan = nullptr;
    try {
        maybe_trace_segv();
        SLU_REQUIRE(trf && trf->supernode2treeMap, "%s: no trf3Dpartition", name);
        reap_join();
        slu_comm *c = comm_for_grid3d(g3);
        slu_engine_opts eo{};
        eo.replace_tiny_pivot = options->ReplaceTinyPivot == SLU_YES;
        eo.overlap_upload = 1;
        eo.forest_map = (const int64_t *)trf->supernode2treeMap;
        if (schedule_only_3d()) {
            eo.overlap_upload = 0;
            eo.schedule_only = 1;
            char err[512] = {0};
            plan = slu_plan_create(dtype, LUstruct, n, (int)g3->nprow, (int)g3->npcol, grid->iam,
                                   c, &eo, err, sizeof err);
            if (!plan) throw slu::Error(err);
            int64_t ns = 0, nb = 0;
            if (slu_plan_check_exchange(plan, &ns, &nb)) throw slu::Error(slu_last_error());
            slu_plan_stats st;
            slu_plan_get_stats(plan, &st);
            printf("[%s schedule] rank %d layer %lld: %lld supernodes factored in %lld levels, "
                   "%lld sections / %lld bytes received, exchange checked\n",
                   name, g3->iam, (long long)st.zlayer, (long long)st.nsupers,
                   (long long)st.nlevels, (long long)ns, (long long)nb);
            fflush(stdout);
            slu_plan_destroy(plan);
            plan = nullptr;
            return 0;
        }
        char err[512] = {0};
        plan = slu_plan_create(dtype, LUstruct, n, (int)g3->nprow, (int)g3->npcol, grid->iam, c,
                               &eo, err, sizeof err);
        if (!plan) throw slu::Error(err);
        int myinfo = 0, tiny = 0;
        if (slu_plan_upload(plan) || slu_plan_factor(plan, anorm, &myinfo, &tiny) ||
            slu_plan_download(plan))
            throw slu::Error(slu_last_error());
        slu_plan_stats st;
        slu_plan_get_stats(plan, &st);
        // reduceStat(FACT, ...) (SRC/util.c:1283-1296): the layers' sum on layer 0
        float mine = (float)(st.schur_flops + st.panel_flops), all = mine;
        mpi().allreduce(&mine, &all, 1, MPI_FLOAT, MPI_SUM, g3->zscp.comm);
        stat->ops[SLU_PHASE_FACT] = g3->zscp.Iam == 0 ? all : mine;
        stat->TinyPivots += tiny;
        stat->gpu_buffer = (float)(st.lu_bytes + st.index_bytes);
        reap_later(plan);
        plan = nullptr;
        *info = myinfo; // the engine's MIN over every layer and rank
        return 0;
    } catch (const std::exception &e) {
        if (plan) slu_plan_destroy(plan);
        fprintf(stderr, "%s (MI355X engine): %s\n", name, e.what());
        fflush(stderr);
        abort();
    }
}

// ------------------------------------------------------------------ solve
// pdgstrs (SRC/pdgstrs.c:1035-3139) on the device-resident factors: the
// plan the last pdgstrf on this LUstruct left in the cache (1x1 grids; its
// factors never left HBM), else a plan that adopts the LUstruct's host
// factors (grids: collective over grid->comm).  B holds rows fst_row ..
// fst_row + m_loc - 1 of the right-hand sides; as pdReDistribute_B_to_X /
// X_to_B (:59-72 of each), row i goes to position perm_c[perm_r[i]] of the
// LUstruct's coordinates, L U y = P b is solved (slu_plan_solve), and the
// same rows of y come back in B (pdgssvx undoes perm_c afterwards).
// Exported by libslu_mi355x_solve.so with p[dsz]Compute_Diag_Inv, which the
// device solve does not need (the reference's is empty without
// SLU_HAVE_LAPACK, SRC/pdgstrs.c:4550).  pdgsrfs stays the reference's and
// calls this pdgstrs for every refinement step.
struct Mpi2 {
    int (*allgatherv)(const void *, int, MPI_Datatype, void *, const int *, const int *,
                      MPI_Datatype, MPI_Comm) = nullptr;
};
const Mpi2 &mpi2() {
    static Mpi2 m = [] {
        Mpi2 x;
        mpi_sym(x.allgatherv, "MPI_Allgatherv");
        return x;
    }();
    return m;
}

template <typename LUS, typename HT>
void pxgstrs(int dtype, const char *name, int_t n, LUS *LU, xScalePermstruct_t *sp,
             gridinfo_t *grid, HT *B, int_t m_loc, int_t fst_row, int_t ldb, int nrhs,
             SuperLUStat_t *stat, int *info) {
    const auto t0 = std::chrono::steady_clock::now();
    *info = 0;
    if (n < 0) *info = -1;
    else if (nrhs < 0) *info = -9;
    if (*info) {
        printf("{%lld,%lld}: On entry to %6s, parameter number %lld had an illegal value\n",
               (long long)(grid->iam / grid->npcol), (long long)(grid->iam % grid->npcol), name,
               (long long)-*info);
        return;
    }
    if (n == 0 || nrhs == 0) return;
    slu_plan *plan = nullptr;
    bool cached = false;
    try {
        const bool one = grid->nprow * grid->npcol == 1;
        {
            // the plan of the last pdgstrf on this LUstruct still holds its
            // factors in HBM (grids too: its coarse storage); every rank of a
            // grid must agree, the solve is collective
            slu_comm *const gcomm = comm_for_grid(grid);
            bool hit;
            {
                std::lock_guard<std::mutex> lk(g_cache_mu);
                hit = g_cache.plan && g_cache.key == lu_key(LU) && g_cache.dtype == dtype && g_cache.n == n &&
                      g_cache.comm == gcomm;
            }
            if (all_ranks(hit, grid)) {
                std::lock_guard<std::mutex> lk(g_cache_mu);
                plan = g_cache.plan;
                cached = true;
            }
        }
        if (!plan) {
            reap_join(); // (nothing of an evicted plan still in flight if this aborts)
            {
                std::lock_guard<std::mutex> lk(g_cache_mu);
                const LuKey k = lu_key(LU);
                SLU_REQUIRE(std::find(g_evicted.begin(), g_evicted.end(), k) == g_evicted.end(),
                            "the factors of this LUstruct were kept only in GPU memory, and a later "
                            "pdgstrf on another LUstruct replaced them (its host L / U arrays still "
                            "hold A); factor it again, or set SUPERLU_MI355X_HOST_FACTORS=1 so that "
                            "pdgstrf writes the factors back");
            }
            slu_comm *c = comm_for_grid(grid);
            slu_engine_opts eo{};
            char err[512] = {0};
            plan = slu_plan_create(dtype, LU, (int)n, (int)grid->nprow, (int)grid->npcol, grid->iam,
                                   c, &eo, err, sizeof err);
            if (!plan) throw slu::Error(err);
            if (slu_plan_adopt_factors(plan)) throw slu::Error(slu_last_error());
        }
        // the whole right-hand side on every rank, in the LUstruct's order
        std::vector<HT> y((size_t)n * nrhs), bl;
        const int_t *pr = sp->perm_r, *pc = sp->perm_c;
        auto place = [&](const HT *src, int_t ld, int_t r0, int_t cnt) {
            for (int j = 0; j < nrhs; ++j)
                for (int_t i = 0; i < cnt; ++i) y[(size_t)j * n + pc[pr[r0 + i]]] = src[i + (size_t)j * ld];
        };
        if (one) {
            place(B, ldb, 0, n);
        } else {
            const int P = (int)(grid->nprow * grid->npcol);
            std::vector<int64_t> mine = {fst_row, m_loc}, all(2 * (size_t)P);
            mpi().allgather(mine.data(), 2, MPI_INT64_T, all.data(), 2, MPI_INT64_T, grid->comm);
            // rows go as bytes, one right-hand side at a time
            std::vector<int> cnt(P), dsp(P);
            for (int r = 0; r < P; ++r) {
                cnt[r] = (int)(all[2 * r + 1] * sizeof(HT));
                dsp[r] = (int)(all[2 * r] * sizeof(HT));
            }
            std::vector<HT> col(n), glob((size_t)n * nrhs);
            for (int j = 0; j < nrhs; ++j) {
                for (int_t i = 0; i < m_loc; ++i) col[i] = B[i + (size_t)j * ldb];
                mpi2().allgatherv(col.data(), (int)(m_loc * sizeof(HT)), MPI_BYTE,
                                  glob.data() + (size_t)j * n, cnt.data(), dsp.data(), MPI_BYTE,
                                  grid->comm);
            }
            place(glob.data(), n, 0, n);
        }
        if (slu_plan_solve(plan, y.data(), n, nrhs)) throw slu::Error(slu_last_error());
        for (int j = 0; j < nrhs; ++j)
            for (int_t i = 0; i < m_loc; ++i) B[i + (size_t)j * ldb] = y[(size_t)j * n + fst_row + i];
        slu_plan_stats st;
        slu_plan_get_stats(plan, &st);
        // reference accounting: 2 flops per stored factor entry per right-hand side
        const double vals = st.lu_bytes / (double)sizeof(HT);
        stat->ops[SLU_PHASE_SOLVE] = (float)(2.0 * vals * nrhs * (dtype == SLU_Z ? 4 : 1));
        if (!cached) reap_later(plan);
        plan = nullptr;
        stat->utime[SLU_PHASE_SOLVE] =
            std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
    } catch (const std::exception &e) {
        if (plan && !cached) slu_plan_destroy(plan);
        fprintf(stderr, "%s (MI355X engine): %s\n", name, e.what());
        fflush(stderr);
        abort();
    }
}

extern "C" void *slu_distribute_glu_deferred(int64_t n, const int_t *xsup, const int_t *supno,
                                             const int_t *xlsub, const int_t *lsub, const int_t *xusub,
                                             const int_t *usub, const int64_t *xa, const int64_t *asub,
                                             const double *a, int nprow, int npcol, int myrow, int mycol);

// ------------------------------------------------------------------ distribute
// pddistribute (SRC/pddistribute.c:327-2398) for callers that also take
// pdgstrs from this library (libslu_mi355x_solve.so).  The LU storage is the
// restated structural distribute (csrc/distribute.cpp: index arrays, block
// order, values, ToRecv / ToSendD / ToSendR and bufmax bit for bit with the
// reference's), built on host threads from Glu_persist + Glu_freeable and A
// -- the caller's NRformat_loc rows, row i going to perm_c[perm_r[i]] as in
// dReDistribute_A (:113-116; pdgssvx has already mapped the column indices
// through perm_c, SRC/pdgssvx.c:1140), gathered to every rank on grids.  The
// reference's triangular-solve metadata (trees, fmod / bmod, send lists,
// :1543-2236) is only read by the reference's pdgstrs, which the same library
// replaces; its fields are left as valid empty placeholders (every tree
// marked empty, the send lists allocated) so that dDestroy_LU frees them as
// usual.  Fact == SamePattern_SameRowPerm refills the values of the existing
// structure (:545-672).
template <typename T, typename LUS>
float pxdistribute(int dtype, const char *name, superlu_dist_options_t *options, int_t n,
                   SuperMatrix *A, xScalePermstruct_t *sp, Glu_freeable_t *glu, LUS *LU,
                   gridinfo_t *grid) {
    try {
        const NRformat_loc *As = (const NRformat_loc *)A->Store;
        const int_t *pr = sp->perm_r, *pc = sp->perm_c;
        const int Pr = (int)grid->nprow, Pc = (int)grid->npcol, P = Pr * Pc;
        const int myrow = grid->iam / Pc, mycol = grid->iam % Pc;
        // SLU_DIST_TIME=1: phase times on stderr (diagnostics)
        const bool dtime = getenv("SLU_DIST_TIME") != nullptr;
        auto dt0 = std::chrono::steady_clock::now();
        auto dtick = [&](const char *what) {
            if (!dtime) return;
            const auto t = std::chrono::steady_clock::now();
            fprintf(stderr, "[pxdistribute] %-26s %8.1f ms\n", what, std::chrono::duration<double, std::milli>(t - dt0).count());
            dt0 = t;
        };
        // ---- A in the LUstruct's coordinates, as CSC (every rank: all of it)
        const i64 nl = As->rowptr[As->m_loc] - As->rowptr[0];
        std::vector<int64_t> ri, ci;
        std::vector<T> vv;
        {
            std::vector<int64_t> r((size_t)nl), c((size_t)nl);
            std::vector<T> v((size_t)nl);
            const T *av = (const T *)As->nzval;
            // (rows in blocks on the host threads: entry e of row i is at
            // rowptr[i] - rowptr[0] + its position in the row)
            const i64 m_loc = As->m_loc, p0 = As->rowptr[0];
            const int nrb = (int)((m_loc + 16383) / 16384);
            slu::parallel_for(nrb, [&](int t) {
                for (i64 i = (i64)t * 16384; i < std::min<i64>(m_loc, (i64)(t + 1) * 16384); ++i) {
                    const int64_t gi = pc[pr[i + As->fst_row]];
                    for (i64 p = As->rowptr[i]; p < As->rowptr[i + 1]; ++p) {
                        r[p - p0] = gi;
                        c[p - p0] = As->colind[p];
                        v[p - p0] = av[p];
                    }
                }
            }, 1);
            if (P == 1) {
                ri.swap(r);
                ci.swap(c);
                vv.swap(v);
            } else {
                std::vector<int64_t> cnt(P);
                int64_t mine = nl;
                mpi().allgather(&mine, 1, MPI_INT64_T, cnt.data(), 1, MPI_INT64_T, grid->comm);
                i64 tot = 0;
                std::vector<int> bc(P), bd(P);
                for (int q = 0; q < P; ++q) tot += cnt[q];
                ri.resize(tot);
                ci.resize(tot);
                vv.resize(tot);
                auto gather = [&](const void *src, void *dst, int esz) {
                    i64 off = 0;
                    for (int q = 0; q < P; ++q) {
                        SLU_REQUIRE(cnt[q] * esz < (1ll << 31), "%s: rank %d holds too many entries", name, q);
                        bc[q] = (int)(cnt[q] * esz);
                        bd[q] = (int)std::min<i64>(off, (1ll << 31) - 1);
                        off += cnt[q] * esz;
                    }
                    SLU_REQUIRE(off < (1ll << 31), "%s: A too large to gather", name);
                    mpi2().allgatherv(src, (int)(mine * esz), MPI_BYTE, dst, bc.data(), bd.data(),
                                      MPI_BYTE, grid->comm);
                };
                gather(r.data(), ri.data(), 8);
                gather(c.data(), ci.data(), 8);
                gather(v.data(), vv.data(), (int)sizeof(T));
            }
        }
        dtick("A coordinates");
        std::vector<int64_t> xa(n + 1, 0), asub(ri.size());
        std::vector<T> aval(ri.size());
        const i64 ne = (i64)ri.size();
        // CSC by a counting sort; each column's entries in entry order (the
        // stash below compares the pattern with the previous call's).  On
        // the host threads: per (entry chunk, column) counts, then each chunk
        // fills its slice of every column
        const int NCH = std::max(1, std::min(slu::plan_threads(), (int)std::min<i64>(16, ne / 65536 + 1)));
        if (NCH > 1 && ne < INT32_MAX && (i64)NCH * n <= (1ll << 27)) {
            std::vector<int32_t> cc((size_t)NCH * n, 0); // counts, then fill cursors
            auto eb = [&](int c) { return ne * c / NCH; };
            slu::parallel_for(NCH, [&](int c) {
                int32_t *cnt = cc.data() + (size_t)c * n;
                for (i64 e = eb(c); e < eb(c + 1); ++e) cnt[ci[e]]++;
            }, 1);
            const int NB = (int)((n + 65535) / 65536);
            slu::parallel_for(NB, [&](int t) {
                for (i64 j = (i64)t * 65536; j < std::min<i64>(n, (i64)(t + 1) * 65536); ++j) {
                    i64 tot = 0;
                    for (int c = 0; c < NCH; ++c) tot += cc[(size_t)c * n + j];
                    xa[j + 1] = tot;
                }
            }, 1);
            for (i64 j = 0; j < n; ++j) xa[j + 1] += xa[j];
            slu::parallel_for(NB, [&](int t) {
                for (i64 j = (i64)t * 65536; j < std::min<i64>(n, (i64)(t + 1) * 65536); ++j) {
                    i64 pos = xa[j];
                    for (int c = 0; c < NCH; ++c) {
                        const int32_t k = cc[(size_t)c * n + j];
                        cc[(size_t)c * n + j] = (int32_t)pos;
                        pos += k;
                    }
                }
            }, 1);
            slu::parallel_for(NCH, [&](int c) {
                int32_t *f = cc.data() + (size_t)c * n;
                for (i64 e = eb(c); e < eb(c + 1); ++e) {
                    const i64 q = f[ci[e]]++;
                    asub[q] = ri[e];
                    aval[q] = vv[e];
                }
            }, 1);
        } else {
            for (int64_t c : ci) xa[c + 1]++;
            for (i64 j = 0; j < n; ++j) xa[j + 1] += xa[j];
            std::vector<int64_t> f(xa.begin(), xa.end() - 1);
            for (size_t e = 0; e < ri.size(); ++e) {
                const i64 q = f[ci[e]]++;
                asub[q] = ri[e];
                aval[q] = vv[e];
            }
        }
        dtick("A as CSC");
        // A's values go only to the stash (the device fill's source), not
        // into the host L / U arrays: their first touch is the 16.8 GB of
        // page zeroing that dominated pddistribute at 100^3, and nothing of
        // this library reads them before pdgstrf overwrites them (INTEGRATION
        // §1).  SUPERLU_MI355X_DEFER_A=0 or HOST_FACTORS=1: placed as the
        // reference does.
        const char *hfe = getenv("SUPERLU_MI355X_HOST_FACTORS"), *dfe = getenv("SUPERLU_MI355X_DEFER_A");
        const bool defer = dtype == SLU_D && !(hfe && atoi(hfe) == 1) && !(dfe && atoi(dfe) == 0);
        auto stash = [&](bool first_time) { // A for the device fill of the following pdgstrf
            std::lock_guard<std::mutex> lk(g_deva_mu);
            const bool same = g_deva.lu == LU && g_deva.llu == LU->Llu &&
                              g_deva.lrow == LU->Llu->Lrowind_bc_ptr && g_deva.dtype == dtype &&
                              g_deva.n == n && g_deva.xa == xa && g_deva.asub == asub;
            // a SamePattern_SameRowPerm refill keeps the pattern (and the
            // plan's map of it); anything else starts a new generation
            if (first_time || !same) g_deva.pattern_gen = ++g_deva_gen;
            g_deva.lu = LU;
            g_deva.llu = LU->Llu;
            g_deva.lrow = LU->Llu->Lrowind_bc_ptr;
            g_deva.dtype = dtype;
            g_deva.n = n;
            // (the last use of xa / asub: moved, not copied)
            g_deva.xa = std::move(xa);
            g_deva.asub = std::move(asub);
            g_deva.a.assign((const char *)aval.data(), (const char *)(aval.data() + aval.size()));
            g_deva.gen = ++g_deva_gen;
            if (defer) g_host_a_deferred.insert(LU->Llu);
            else g_host_a_deferred.erase(LU->Llu);
        };
        if (options->Fact == 2 /* SamePattern_SameRowPerm */) {
            if (!defer && slu_refill_values(dtype, LU, n, xa.data(), asub.data(), aval.data(), Pr, Pc, myrow,
                                            mycol))
                throw slu::Error(slu_last_error());
            dtick("refill");
            stash(false);
            dtick("stash");
            return 0.0f;
        }
        // ---- first-time branch: the restated structural distribute
        const Glu_persist_t *gp = LU->Glu_persist;
        LUS *tmp = defer ? (LUS *)slu_distribute_glu_deferred(n, gp->xsup, gp->supno, glu->xlsub, glu->lsub,
                                                              glu->xusub, glu->usub, xa.data(), asub.data(),
                                                              (const double *)aval.data(), Pr, Pc, myrow, mycol)
                         : (LUS *)slu_distribute_glu(dtype, n, gp->xsup, gp->supno, glu->xlsub, glu->lsub,
                                                     glu->xusub, glu->usub, xa.data(), asub.data(),
                                                     aval.data(), Pr, Pc, myrow, mycol);
        if (!tmp) throw slu::Error(slu_last_error());
        dtick("structural distribute");
        *LU->Llu = *tmp->Llu; // the arrays move over (malloc'ed: SUPERLU_FREE frees them)
        free(tmp->Glu_persist->xsup);
        free(tmp->Glu_persist->supno);
        free(tmp->Glu_persist);
        free(tmp->Llu);
        free(tmp);
        auto *Llu = LU->Llu;
        const i64 ns = gp->supno[n - 1] + 1, nlc = (ns + Pc - 1) / Pc, nlr = (ns + Pr - 1) / Pr;
        if (dtype != SLU_D) {
            // s / z: [sz]Destroy_LU (SRC/psutil.c, pzutil.c) frees every block
            // on its own -- their pddistribute mallocs each one (the d version
            // keeps them in the *_dat arrays and frees those)
            const int_t *xs = gp->xsup;
            for (i64 ljb = 0; ljb < nlc; ++ljb) {
                const int_t *ix = Llu->Lrowind_bc_ptr[ljb];
                if (!ix) continue;
                i64 p = SLU_BC_HEADER;
                for (i64 b = 0; b < ix[0]; ++b) p += SLU_LB_DESCRIPTOR + ix[p + 1];
                const i64 jb = ljb * Pc + mycol, nv = (i64)ix[1] * (xs[jb + 1] - xs[jb]);
                int_t *ni = (int_t *)malloc((size_t)p * sizeof(int_t));
                T *nv_ = (T *)malloc((size_t)std::max<i64>(nv, 1) * sizeof(T));
                SLU_REQUIRE(ni && nv_, "%s: out of host memory", name);
                memcpy(ni, ix, (size_t)p * sizeof(int_t));
                memcpy(nv_, Llu->Lnzval_bc_ptr[ljb], (size_t)nv * sizeof(T));
                Llu->Lrowind_bc_ptr[ljb] = ni;
                Llu->Lnzval_bc_ptr[ljb] = nv_;
            }
            for (i64 lb = 0; lb < nlr; ++lb) {
                const int_t *ix = Llu->Ufstnz_br_ptr[lb];
                if (!ix) continue;
                const i64 li = ix[2], nv = ix[1];
                int_t *ni = (int_t *)malloc((size_t)li * sizeof(int_t));
                T *nv_ = (T *)malloc((size_t)std::max<i64>(nv, 1) * sizeof(T));
                SLU_REQUIRE(ni && nv_, "%s: out of host memory", name);
                memcpy(ni, ix, (size_t)li * sizeof(int_t));
                memcpy(nv_, Llu->Unzval_br_ptr[lb], (size_t)nv * sizeof(T));
                Llu->Ufstnz_br_ptr[lb] = ni;
                Llu->Unzval_br_ptr[lb] = nv_;
            }
            free(Llu->Lrowind_bc_dat);
            free(Llu->Lnzval_bc_dat);
            free(Llu->Ufstnz_br_dat);
            free(Llu->Unzval_br_dat);
            free(Llu->Lrowind_bc_offset);
            free(Llu->Lnzval_bc_offset);
            free(Llu->Ufstnz_br_offset);
            free(Llu->Unzval_br_offset);
            Llu->Lrowind_bc_dat = nullptr;
            Llu->Lnzval_bc_dat = nullptr;
            Llu->Ufstnz_br_dat = nullptr;
            Llu->Unzval_br_dat = nullptr;
            Llu->Lrowind_bc_offset = Llu->Lnzval_bc_offset = nullptr;
            Llu->Ufstnz_br_offset = Llu->Unzval_br_offset = nullptr;
        }
        // per-block pointer tables the destroy routines walk (all empty)
        Llu->Lindval_loc_bc_ptr = (int_t **)calloc((size_t)std::max<i64>(nlc, 1), sizeof(int_t *));
        Llu->Linv_bc_ptr = (decltype(Llu->Linv_bc_ptr))calloc((size_t)std::max<i64>(nlc, 1), sizeof(void *));
        Llu->Uinv_bc_ptr = (decltype(Llu->Uinv_bc_ptr))calloc((size_t)std::max<i64>(nlc, 1), sizeof(void *));
        Llu->Urbs = (int_t *)calloc((size_t)std::max<i64>(nlc, 1), sizeof(int_t));
        Llu->Ucb_indptr = (decltype(Llu->Ucb_indptr))calloc((size_t)std::max<i64>(nlc, 1), sizeof(void *));
        Llu->Ucb_valptr = (int_t **)calloc((size_t)std::max<i64>(nlc, 1), sizeof(int_t *));
        auto trees = [](i64 cnt) {
            auto *t = (slu_ctree_mirror_t *)calloc((size_t)std::max<i64>(cnt, 1), sizeof(slu_ctree_mirror_t));
            for (i64 i = 0; i < cnt; ++i) t[i].empty_ = SLU_YES;
            return (C_Tree *)t;
        };
        Llu->LBtree_ptr = trees(nlc);
        Llu->UBtree_ptr = trees(nlc);
        Llu->LRtree_ptr = trees(nlr);
        Llu->URtree_ptr = trees(nlr);
        Llu->fsendx_plist = (int **)calloc(1, sizeof(int *));
        Llu->fsendx_plist[0] = (int *)calloc(1, sizeof(int));
        Llu->bsendx_plist = (int **)calloc(1, sizeof(int *));
        Llu->bsendx_plist[0] = (int *)calloc(1, sizeof(int));
        Llu->mod_bit = (int *)calloc((size_t)std::max<i64>(nlr, 1), sizeof(int));
        // ilsum / ldalsum as the reference sets them (:1530-1540): my block rows' offsets
        Llu->ilsum = (int_t *)malloc((size_t)(nlr + 1) * sizeof(int_t));
        Llu->ilsum[0] = 0;
        for (i64 lb = 0; lb < nlr; ++lb) {
            const i64 gb = lb * Pr + myrow;
            Llu->ilsum[lb + 1] = Llu->ilsum[lb] + (gb < ns ? gp->xsup[gb + 1] - gp->xsup[gb] : 0);
        }
        Llu->ldalsum = Llu->ilsum[nlr];
        {
            std::lock_guard<std::mutex> lk(g_cache_mu);
            unmark_evicted(lu_key(LU)); // new storage: A's values, no factors yet
        }
        dtick("placeholders");
        stash(true);
        dtick("stash");
        return (float)((double)Llu->Lnzval_bc_cnt * sizeof(T) + (double)Llu->Unzval_br_cnt * sizeof(T) +
                       (double)(Llu->Lrowind_bc_cnt + Llu->Ufstnz_br_cnt) * sizeof(int_t));
    } catch (const std::exception &e) {
        fprintf(stderr, "%s (MI355X library): %s\n", name, e.what());
        fflush(stderr);
        abort();
    }
}

// ------------------------------------------------------------------ scatter
// Host implementations with the reference prototypes and semantics of
// SRC/dscatter.c:28-277 (s/z are type substitutions).
template <typename T> inline void vsub(T &a, const T &b) { a -= b; }
inline void vsub(doublecomplex &a, const doublecomplex &b) { a.r -= b.r; a.i -= b.i; }

// dscatter_l_1 is defined with 32-bit usub / lsub (SRC/dscatter.c:29-43; it
// has no prototype in the headers), unlike dscatter_l / dscatter_u.
template <typename T>
void scatter_l_1(int ib, int ljb, int nsupc, int_t iukp, int_t *xsup, int klst, int nbrow,
                 int_t lptr, int temp_nbrow, int *usub, int *lsub, T *tempv,
                 int *indirect_thread, int_t **Lrowind_bc_ptr, T **Lnzval_bc_ptr) {
    int_t *index = Lrowind_bc_ptr[ljb];
    int_t ldv = index[1], lptrj = SLU_BC_HEADER, luptrj = 0;
    while (index[lptrj] != ib) {
        luptrj += index[lptrj + 1];
        lptrj += SLU_LB_DESCRIPTOR + index[lptrj + 1];
    }
    int_t fnz = xsup[ib], dest_nbrow = index[lptrj + 1];
    lptrj += SLU_LB_DESCRIPTOR;
    for (int_t i = 0; i < dest_nbrow; ++i) indirect_thread[index[lptrj + i] - fnz] = (int)i;
    T *nzval = Lnzval_bc_ptr[ljb] + luptrj;
    for (int jj = 0; jj < nsupc; ++jj) {
        int_t segsize = klst - usub[iukp + jj];
        if (segsize) {
            for (int i = 0; i < temp_nbrow; ++i)
                vsub(nzval[indirect_thread[lsub[lptr + i] - fnz]], tempv[i]);
            tempv += nbrow;
        }
        nzval += ldv;
    }
}

template <typename T>
void scatter_l(int ib, int ljb, int nsupc, int_t iukp, int_t *xsup, int klst, int nbrow,
               int_t lptr, int temp_nbrow, int_t *usub, int_t *lsub, T *tempv,
               int *indirect_thread, int *indirect2, int_t **Lrowind_bc_ptr, T **Lnzval_bc_ptr) {
    int_t *index = Lrowind_bc_ptr[ljb];
    int_t ldv = index[1], lptrj = SLU_BC_HEADER, luptrj = 0;
    while (index[lptrj] != ib) {
        luptrj += index[lptrj + 1];
        lptrj += SLU_LB_DESCRIPTOR + index[lptrj + 1];
    }
    int_t fnz = xsup[ib], dest_nbrow = index[lptrj + 1];
    lptrj += SLU_LB_DESCRIPTOR;
    for (int_t i = 0; i < dest_nbrow; ++i) indirect_thread[index[lptrj + i] - fnz] = (int)i;
    for (int i = 0; i < temp_nbrow; ++i) indirect2[i] = indirect_thread[lsub[lptr + i] - fnz];
    T *nzval = Lnzval_bc_ptr[ljb] + luptrj;
    for (int jj = 0; jj < nsupc; ++jj) {
        int_t segsize = klst - usub[iukp + jj];
        if (segsize) {
            for (int i = 0; i < temp_nbrow; ++i) vsub(nzval[indirect2[i]], tempv[i]);
            tempv += nbrow;
        }
        nzval += ldv;
    }
}

template <typename T>
void scatter_u(int ib, int jb, int nsupc, int_t iukp, int_t *xsup, int klst, int nbrow,
               int_t lptr, int temp_nbrow, int_t *lsub, int_t *usub, T *tempv,
               int_t **Ufstnz_br_ptr, T **Unzval_br_ptr, gridinfo_t *grid) {
    int_t ilst = xsup[ib + 1], lib = ib / grid->nprow;
    int_t *index = Ufstnz_br_ptr[lib];
    int_t iuip = SLU_BR_HEADER, ruip = 0;
    while (index[iuip] < jb) {
        ruip += index[iuip + 1];
        iuip += SLU_UB_DESCRIPTOR + (xsup[index[iuip] + 1] - xsup[index[iuip]]);
    }
    iuip += SLU_UB_DESCRIPTOR;
    for (int jj = 0; jj < nsupc; ++jj) {
        int_t segsize = klst - usub[iukp + jj];
        int_t fnz = index[iuip++];
        if (segsize) {
            T *ucol = &Unzval_br_ptr[lib][ruip];
            for (int i = 0; i < temp_nbrow; ++i) vsub(ucol[lsub[lptr + i] - fnz], tempv[i]);
            tempv += nbrow;
        }
        ruip += ilst - fnz;
    }
}

} // namespace

extern "C" {

int_t pdgstrf(superlu_dist_options_t *options, int m, int n, double anorm,
              dLUstruct_t *LUstruct, gridinfo_t *grid, SuperLUStat_t *stat, int *info) {
    CallerRandState rs;
    return pxgstrf(SLU_D, "PDGSTRF", options, m, n, anorm, LUstruct, grid, stat, info);
}
int_t psgstrf(superlu_dist_options_t *options, int m, int n, float anorm,
              sLUstruct_t *LUstruct, gridinfo_t *grid, SuperLUStat_t *stat, int *info) {
    CallerRandState rs;
    return pxgstrf(SLU_S, "PSGSTRF", options, m, n, (double)anorm, LUstruct, grid, stat, info);
}
int_t pzgstrf(superlu_dist_options_t *options, int m, int n, double anorm,
              zLUstruct_t *LUstruct, gridinfo_t *grid, SuperLUStat_t *stat, int *info) {
    CallerRandState rs;
    return pxgstrf(SLU_Z, "PZGSTRF", options, m, n, anorm, LUstruct, grid, stat, info);
}

int_t pdgstrf3d(superlu_dist_options_t *options, int m, int n, double anorm,
                dtrf3Dpartition_t *trf3Dpartition, SCT_t *, dLUstruct_t *LUstruct,
                gridinfo3d_t *grid3d, SuperLUStat_t *stat, int *info) {
    CallerRandState rs;
    return pxgstrf3d(SLU_D, "PDGSTRF3D", options, m, n, anorm, trf3Dpartition, LUstruct, grid3d,
                     stat, info);
}
int_t psgstrf3d(superlu_dist_options_t *options, int m, int n, float anorm,
                strf3Dpartition_t *trf3Dpartition, SCT_t *, sLUstruct_t *LUstruct,
                gridinfo3d_t *grid3d, SuperLUStat_t *stat, int *info) {
    CallerRandState rs;
    return pxgstrf3d(SLU_S, "PSGSTRF3D", options, m, n, (double)anorm, trf3Dpartition, LUstruct,
                     grid3d, stat, info);
}
int_t pzgstrf3d(superlu_dist_options_t *options, int m, int n, double anorm,
                ztrf3Dpartition_t *trf3Dpartition, SCT_t *, zLUstruct_t *LUstruct,
                gridinfo3d_t *grid3d, SuperLUStat_t *stat, int *info) {
    CallerRandState rs;
    return pxgstrf3d(SLU_Z, "PZGSTRF3D", options, m, n, anorm, trf3Dpartition, LUstruct, grid3d,
                     stat, info);
}

void pdgstrs(superlu_dist_options_t *, int_t n, dLUstruct_t *LUstruct,
             xScalePermstruct_t *ScalePermstruct, gridinfo_t *grid, double *B, int_t m_loc,
             int_t fst_row, int_t ldb, int nrhs, xSOLVEstruct_t *, SuperLUStat_t *stat,
             int *info) {
    CallerRandState rs;
    pxgstrs(SLU_D, "PDGSTRS", n, LUstruct, ScalePermstruct, grid, B, m_loc, fst_row, ldb, nrhs,
            stat, info);
}
void psgstrs(superlu_dist_options_t *, int_t n, sLUstruct_t *LUstruct,
             xScalePermstruct_t *ScalePermstruct, gridinfo_t *grid, float *B, int_t m_loc,
             int_t fst_row, int_t ldb, int nrhs, xSOLVEstruct_t *, SuperLUStat_t *stat,
             int *info) {
    CallerRandState rs;
    pxgstrs(SLU_S, "PSGSTRS", n, LUstruct, ScalePermstruct, grid, B, m_loc, fst_row, ldb, nrhs,
            stat, info);
}
void pzgstrs(superlu_dist_options_t *, int_t n, zLUstruct_t *LUstruct,
             xScalePermstruct_t *ScalePermstruct, gridinfo_t *grid, doublecomplex *B,
             int_t m_loc, int_t fst_row, int_t ldb, int nrhs, xSOLVEstruct_t *,
             SuperLUStat_t *stat, int *info) {
    CallerRandState rs;
    pxgstrs(SLU_Z, "PZGSTRS", n, LUstruct, ScalePermstruct, grid, B, m_loc, fst_row, ldb, nrhs,
            stat, info);
}
float pddistribute(superlu_dist_options_t *options, int_t n, SuperMatrix *A,
                   xScalePermstruct_t *ScalePermstruct, Glu_freeable_t *Glu_freeable,
                   dLUstruct_t *LUstruct, gridinfo_t *grid) {
    CallerRandState rs;
    return pxdistribute<double>(SLU_D, "PDDISTRIBUTE", options, n, A, ScalePermstruct, Glu_freeable,
                                LUstruct, grid);
}
float psdistribute(superlu_dist_options_t *options, int_t n, SuperMatrix *A,
                   xScalePermstruct_t *ScalePermstruct, Glu_freeable_t *Glu_freeable,
                   sLUstruct_t *LUstruct, gridinfo_t *grid) {
    CallerRandState rs;
    return pxdistribute<float>(SLU_S, "PSDISTRIBUTE", options, n, A, ScalePermstruct, Glu_freeable,
                               LUstruct, grid);
}
float pzdistribute(superlu_dist_options_t *options, int_t n, SuperMatrix *A,
                   xScalePermstruct_t *ScalePermstruct, Glu_freeable_t *Glu_freeable,
                   zLUstruct_t *LUstruct, gridinfo_t *grid) {
    CallerRandState rs;
    return pxdistribute<doublecomplex>(SLU_Z, "PZDISTRIBUTE", options, n, A, ScalePermstruct,
                                       Glu_freeable, LUstruct, grid);
}
void pdCompute_Diag_Inv(int_t, dLUstruct_t *, gridinfo_t *, SuperLUStat_t *, int *info) {
    if (info) *info = 0;
}
void psCompute_Diag_Inv(int_t, sLUstruct_t *, gridinfo_t *, SuperLUStat_t *, int *info) {
    if (info) *info = 0;
}
void pzCompute_Diag_Inv(int_t, zLUstruct_t *, gridinfo_t *, SuperLUStat_t *, int *info) {
    if (info) *info = 0;
}

#define SLU_SCATTER_EXPORTS(P, T)                                                              \
    void P##scatter_l_1(int ib, int ljb, int nsupc, int_t iukp, int_t *xsup, int klst,          \
                        int nbrow, int_t lptr, int temp_nbrow, int *usub, int *lsub,            \
                        T *tempv, int *indirect_thread, int_t **Lrowind_bc_ptr,                 \
                        T **Lnzval_bc_ptr, gridinfo_t *) {                                      \
        scatter_l_1<T>(ib, ljb, nsupc, iukp, xsup, klst, nbrow, lptr, temp_nbrow, usub, lsub,   \
                       tempv, indirect_thread, Lrowind_bc_ptr, Lnzval_bc_ptr);                  \
    }                                                                                          \
    void P##scatter_l(int ib, int ljb, int nsupc, int_t iukp, int_t *xsup, int klst,            \
                      int nbrow, int_t lptr, int temp_nbrow, int_t *usub, int_t *lsub,          \
                      T *tempv, int *indirect_thread, int *indirect2,                           \
                      int_t **Lrowind_bc_ptr, T **Lnzval_bc_ptr, gridinfo_t *) {                \
        scatter_l<T>(ib, ljb, nsupc, iukp, xsup, klst, nbrow, lptr, temp_nbrow, usub, lsub,     \
                     tempv, indirect_thread, indirect2, Lrowind_bc_ptr, Lnzval_bc_ptr);         \
    }                                                                                          \
    void P##scatter_u(int ib, int jb, int nsupc, int_t iukp, int_t *xsup, int klst, int nbrow,  \
                      int_t lptr, int temp_nbrow, int_t *lsub, int_t *usub, T *tempv,           \
                      int_t **Ufstnz_br_ptr, T **Unzval_br_ptr, gridinfo_t *grid) {             \
        scatter_u<T>(ib, jb, nsupc, iukp, xsup, klst, nbrow, lptr, temp_nbrow, lsub, usub,      \
                     tempv, Ufstnz_br_ptr, Unzval_br_ptr, grid);                                \
    }

SLU_SCATTER_EXPORTS(d, double)
SLU_SCATTER_EXPORTS(s, float)
SLU_SCATTER_EXPORTS(z, doublecomplex)

} // extern "C"

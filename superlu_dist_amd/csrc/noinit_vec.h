// std::vector storage that resize() leaves uninitialised (default- instead of
// value-initialised elements): the symbolic factorization's GB-sized index
// arrays are filled on the host threads or by a device copy right after, and
// the serial zeroing a plain vector does first cost as much as the fill.
#pragma once
#include <sys/mman.h>

#include <cstdint>
#include <cstdlib>
#include <new>
#include <memory>
#include <utility>
#include <vector>

namespace slu {

template <class T> struct NoInit : std::allocator<T> {
    using std::allocator<T>::allocator;
    template <class U> struct rebind {
        using other = NoInit<U>;
    };
    // arrays of 64 MB and more on 2 MB-aligned storage advised as huge pages:
    // their first touch (from the host threads) faults once per 2 MB, and the
    // symbolic search's random reads of the lists miss the TLB less (1.76 ->
    // 1.37-1.44 s of symbolic phase at 100^3 on the box, the following first
    // pdgstrf 816-840 -> 846-916 ms: profiles/r06thp/; SLU_NOINIT_THP=0 off)
    T *allocate(size_t n) {
        const size_t bytes = n * sizeof(T);
        static const bool thp = [] {
            const char *e = std::getenv("SLU_NOINIT_THP"); // (=0: plain allocation, A/B)
            return !(e && e[0] == '0');
        }();
        if (!thp || bytes < (size_t(64) << 20)) return std::allocator<T>::allocate(n);
        constexpr size_t HP = size_t(2) << 20;
        void *p = std::aligned_alloc(HP, (bytes + HP - 1) / HP * HP);
        if (!p) throw std::bad_alloc();
        madvise(p, (bytes + HP - 1) / HP * HP, MADV_HUGEPAGE);
        return (T *)p;
    }
    void deallocate(T *p, size_t n) {
        static const bool thp = [] {
            const char *e = std::getenv("SLU_NOINIT_THP");
            return !(e && e[0] == '0');
        }();
        if (!thp || n * sizeof(T) < (size_t(64) << 20)) std::allocator<T>::deallocate(p, n);
        else std::free(p);
    }
    template <class U, class... A> void construct(U *p, A &&...a) {
        if constexpr (sizeof...(A) == 0) ::new ((void *)p) U;
        else ::new ((void *)p) U(std::forward<A>(a)...);
    }
};
using i64_vec = std::vector<int64_t, NoInit<int64_t>>;

} // namespace slu

// std::vector storage that resize() leaves uninitialised (default- instead of
// value-initialised elements): the symbolic factorization's GB-sized index
// arrays are filled on the host threads or by a device copy right after, and
// the serial zeroing a plain vector does first cost as much as the fill.
#pragma once
#include <cstdint>
#include <memory>
#include <utility>
#include <vector>

namespace slu {

template <class T> struct NoInit : std::allocator<T> {
    using std::allocator<T>::allocator;
    template <class U> struct rebind {
        using other = NoInit<U>;
    };
    template <class U, class... A> void construct(U *p, A &&...a) {
        if constexpr (sizeof...(A) == 0) ::new ((void *)p) U;
        else ::new ((void *)p) U(std::forward<A>(a)...);
    }
};
using i64_vec = std::vector<int64_t, NoInit<int64_t>>;

} // namespace slu

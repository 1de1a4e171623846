// Error plumbing shared by the host files.  No exception leaves the C ABI:
// every extern "C" entry point catches slu::Error and stores the message
// for slu_last_error().
#pragma once
#include <cstdarg>
#include <cstdio>
#include <stdexcept>
#include <string>

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

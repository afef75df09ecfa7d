// common.h -- error plumbing shared by the C-ABI translation units.
#pragma once

#include <cstdarg>
#include <cstdio>
#include <string>

#include "../../include/chroma_amd.h"

namespace chr {

// thread-local last-error message (chr_last_error)
std::string &last_error();

// threads of the library's host OpenMP regions (host.cpp, chr_set_host_threads)
int host_threads();

inline int fail(int code, const char *fmt, ...) {
    char buf[1024];
    va_list ap;
    va_start(ap, fmt);
    std::vsnprintf(buf, sizeof(buf), fmt, ap);
    va_end(ap);
    last_error() = buf;
    return code;
}

}  // namespace chr

#define CHR_HIP_CHECK(expr)                                                                 \
    do {                                                                                    \
        hipError_t _e = (expr);                                                             \
        if (_e != hipSuccess)                                                               \
            return chr::fail(CHR_ERR_HIP, "%s failed at %s:%d: %s", #expr, __FILE__, __LINE__, \
                             hipGetErrorString(_e));                                        \
    } while (0)

// propagate a nonzero chr status
#define CHR_TRY(expr)                   \
    do {                                \
        const int _rc = (expr);         \
        if (_rc != CHR_OK) return _rc;  \
    } while (0)

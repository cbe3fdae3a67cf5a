// mlg_host.h -- host-side helpers of the C ABI: error capture, argument checks.
#pragma once
#include <hip/hip_runtime.h>

#include <cstdarg>
#include <cstdio>
#include <string>

namespace mlg {

inline std::string& last_error() {
    static thread_local std::string err;
    return err;
}

inline int fail(const char* fmt, ...) {
    char buf[1024];
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(buf, sizeof(buf), fmt, ap);
    va_end(ap);
    last_error() = buf;
    return 1;
}

inline int check_launch(const char* what) {
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return fail("%s: %s", what, hipGetErrorString(e));
    return 0;
}

}  // namespace mlg

#define MLG_REQUIRE(cond, ...)                  \
    do {                                        \
        if (!(cond)) return mlg::fail(__VA_ARGS__); \
    } while (0)

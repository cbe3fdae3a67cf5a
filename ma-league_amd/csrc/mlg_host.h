// mlg_host.h -- host-side helpers of the C ABI: error capture, argument checks.
#pragma once
#include <hip/hip_runtime.h>

#include <cstdarg>
#include <cstdio>
#include <mutex>
#include <string>

// largest batch (episodes) whose learner slot map travels as a kernel argument (MlgLearnerBufs / MlgRefilLearnerBufs
// .host_rows; mlg_qlearner_inline_rows)
constexpr int MLG_INLINE_ROWS = 64;

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

// A second stream on the device of the caller's stream `s`, for learner kernels that run beside the main chain (forked
// and joined with the events; one stream and four events per device, created on first use, never destroyed).
// nullptr -- the caller then runs everything on `s` -- when `s`'s device is not the current device (the side stream
// would land on the wrong device) or when creating the stream or its events fails (nothing half-built is published).
struct SideStream {
    hipStream_t s = nullptr;
    hipEvent_t ev[4] = {nullptr, nullptr, nullptr, nullptr};
};
inline SideStream* side_stream(hipStream_t caller) {
    static SideStream side[64];
    static std::mutex mu;
    int dev = 0;
    hipDevice_t sdev = 0;
    if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) return nullptr;
    if (hipStreamGetDevice(caller, &sdev) != hipSuccess || (int)sdev != dev) return nullptr;
    std::lock_guard<std::mutex> lk(mu);
    SideStream& ss = side[dev];
    if (!ss.s) {
        // the least priority (1 on this image; the caller's stream has the default 0): the side stream carries the
        // work off the critical path, so the main chain's workgroups are dispatched first when both have work
        // (REFIL learner 0.663 -> 0.658 ms; the greatest priority measured 0.677, profiles/r05/s47_side_prio_ab/)
        int least = 0, greatest = 0;
        if (hipDeviceGetStreamPriorityRange(&least, &greatest) != hipSuccess) return nullptr;
        SideStream fresh;
        for (auto& e : fresh.ev)
            if (hipEventCreateWithFlags(&e, hipEventDisableTiming) != hipSuccess) {
                for (auto& x : fresh.ev)
                    if (x) (void)hipEventDestroy(x);
                return nullptr;
            }
        if (hipStreamCreateWithPriority(&fresh.s, hipStreamNonBlocking, least) != hipSuccess) {
            for (auto& x : fresh.ev) (void)hipEventDestroy(x);
            return nullptr;
        }
        ss = fresh;  // published only once complete
    }
    return &ss;
}
// event `k` recorded on `from`, waited for by `to`
inline bool fork_join(SideStream* ss, int k, hipStream_t from, hipStream_t to) {
    return hipEventRecord(ss->ev[k], from) == hipSuccess && hipStreamWaitEvent(to, ss->ev[k], 0) == hipSuccess;
}

}  // namespace mlg

#define MLG_REQUIRE(cond, ...)                  \
    do {                                        \
        if (!(cond)) return mlg::fail(__VA_ARGS__); \
    } while (0)

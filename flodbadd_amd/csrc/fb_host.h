// fb_host.h -- host-side helpers shared by the C-ABI translation units (fb_capi.hip, fb_ring.hip).
#pragma once
#include <hip/hip_runtime.h>

#include "../../include/flodbadd_gpu.h"

namespace fbk {

// Sets the thread-local text fb_last_error() returns; returns `code`.
int set_err(int code, const char* fmt, ...);
// The device a context was created on.
int ctx_device(const fb_ctx* c);
// Record a nonzero device error word `e` of a call or ring batch: the context zeroes its launch
// scratch before the next launch; returns the matching fb_err (FB_ERR_TABLE_FULL / INTERNAL).
int ctx_report_error(fb_ctx* c, uint64_t e);

struct DeviceGuard {
    int prev = -1;
    explicit DeviceGuard(int dev) {
        if (hipGetDevice(&prev) != hipSuccess) prev = -1;
        if (prev != dev) (void)hipSetDevice(dev);
    }
    ~DeviceGuard() {
        int cur = -1;
        if (prev >= 0 && hipGetDevice(&cur) == hipSuccess && cur != prev) (void)hipSetDevice(prev);
    }
};

}  // namespace fbk

#define HIP_TRY(expr)                                                                         \
    do {                                                                                      \
        hipError_t _e = (expr);                                                               \
        if (_e != hipSuccess)                                                                 \
            return ::fbk::set_err(FB_ERR_HIP, "%s failed: %s", #expr, hipGetErrorString(_e)); \
    } while (0)

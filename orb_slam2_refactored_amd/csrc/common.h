// Shared host/device helpers for the gfx950 ORB / LocalBA library.
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <string>

#include "orbslam2_amd.h"

namespace orbamd {

// Thread-local error text behind orb_last_error().
void set_error(const std::string& msg);

#define ORB_HIP_TRY(expr)                                                                          \
    do {                                                                                           \
        hipError_t _e = (expr);                                                                    \
        if (_e != hipSuccess) {                                                                    \
            ::orbamd::set_error(std::string(#expr) + ": " + hipGetErrorString(_e));                \
            return ORB_EHIP;                                                                       \
        }                                                                                          \
    } while (0)

#define ORB_CHECK_ARG(cond, msg)                                                                   \
    do {                                                                                           \
        if (!(cond)) {                                                                             \
            ::orbamd::set_error(msg);                                                              \
            return ORB_EINVAL;                                                                     \
        }                                                                                          \
    } while (0)

// Device-side failure flags (written by kernels, read by the host after a sync).
enum DeviceFault : uint32_t {
    FAULT_NONE = 0,
    FAULT_QT_NODES = 1u << 0,     // quadtree node array capacity exceeded
    FAULT_QT_ROOT = 1u << 1,      // keypoint mapped outside the root nodes (CV_Assert :569)
    FAULT_CELL_CAP = 1u << 2,     // FAST cell slot overflow (cannot happen: strict NMS bound)
    FAULT_OUT_CAP = 1u << 3,      // per-level output capacity exceeded
    FAULT_BLOCK_SIZE = 1u << 4,   // a kernel launched with a block size other than the one it is written for
};

// Grow-only device buffer.
struct DevBuf {
    void* ptr = nullptr;
    size_t bytes = 0;
    int reserve(size_t need) {
        if (need <= bytes) return ORB_OK;
        if (ptr) (void)hipFree(ptr);
        ptr = nullptr;
        bytes = 0;
        hipError_t e = hipMalloc(&ptr, need);
        if (e != hipSuccess) {
            set_error(std::string("hipMalloc failed: ") + hipGetErrorString(e));
            return ORB_ENOMEM;
        }
        bytes = need;
        return ORB_OK;
    }
    void release() {
        if (ptr) (void)hipFree(ptr);
        ptr = nullptr;
        bytes = 0;
    }
    template <class T>
    T* as() const { return reinterpret_cast<T*>(ptr); }
};

inline size_t align_up(size_t v, size_t a) { return (v + a - 1) / a * a; }

}  // namespace orbamd

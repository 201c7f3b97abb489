// device_guard.hpp — host helper of the HIP translation units (engine.cpp,
// peer.cpp): make `device` current for a scope and restore the caller's.
#pragma once

#include <hip/hip_runtime.h>

namespace tsa {

// switches the calling thread to `device` (>= 0) for the scope, then back
struct DeviceGuard {
    int prev = -1;
    bool ok = true;
    explicit DeviceGuard(int device) {
        if (device < 0) return;
        if (hipGetDevice(&prev) != hipSuccess) { ok = false; prev = -1; return; }
        if (prev == device) { prev = -1; return; }
        if (hipSetDevice(device) != hipSuccess) { ok = false; prev = -1; }
    }
    ~DeviceGuard() {
        if (prev >= 0) (void)hipSetDevice(prev);
    }
};

}  // namespace tsa

// orbx_ws.h -- per-device workspace of the synchronous host entry points
// (the drop-in matchers, depth calls and per-frame helpers).
#pragma once

#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdint>
#include <cstring>
#include <mutex>

#include "../../include/orbx.h"
#include "orbx_device.h"

namespace orbx {

// Workspace of the synchronous host entry points (the drop-in matchers and
// depth calls): per device one grow-only device arena, one pinned staging
// arena, a stream and a mutex -- the reference calls its matchers from the
// Tracking, LocalMapping and LoopClosing threads concurrently.  A call packs
// its inputs into the staging arena, moves them with one copy, runs, and
// brings every output back with one copy.
struct CallWs {
    std::mutex mu;
    hipStream_t st = nullptr;
    uint8_t *dev = nullptr, *host = nullptr;
    uint8_t *host_d = nullptr;    // the pinned arena's device address (the HostTail copy writes there)
    uint32_t *flag = nullptr;     // pinned done flag the HostTail copy raises
    uint32_t *flag_d = nullptr;
    size_t cap = 0;
    int64_t proj_pool = 0;   // projection candidate-list entries the last calls needed
};

inline CallWs &call_ws(int device) {
    static CallWs ws[64];
    return ws[device & 63];
}

struct Layout {
    size_t size = 0;
    size_t add(size_t bytes) {
        const size_t o = size;
        size += (bytes + 255) & ~size_t(255);
        return o;
    }
};

// Ensures stream and capacity (caller holds ws.mu and has set the device).
inline int ws_reserve(CallWs &ws, size_t bytes) {
    if (!ws.st && hipStreamCreateWithFlags(&ws.st, hipStreamNonBlocking) != hipSuccess) return ORBX_EIO;
    if (!ws.flag) {
        if (hipHostMalloc(reinterpret_cast<void **>(&ws.flag), 64, hipHostMallocDefault) != hipSuccess) return ORBX_ENOMEM;
        if (hipHostGetDevicePointer(reinterpret_cast<void **>(&ws.flag_d), ws.flag, 0) != hipSuccess) ws.flag_d = nullptr;
    }
    if (ws.cap >= bytes) return ORBX_OK;
    (void)hipStreamSynchronize(ws.st);
    if (ws.dev) (void)hipFree(ws.dev);
    if (ws.host) (void)hipHostFree(ws.host);
    ws.dev = ws.host = nullptr;
    ws.cap = 0;
    const size_t cap = std::max(bytes, size_t(1) << 20) * 3 / 2;
    if (hipMalloc(reinterpret_cast<void **>(&ws.dev), cap) != hipSuccess) return ORBX_ENOMEM;
    if (hipHostMalloc(reinterpret_cast<void **>(&ws.host), cap, hipHostMallocDefault) != hipSuccess) {
        (void)hipFree(ws.dev);
        ws.dev = nullptr;
        return ORBX_ENOMEM;
    }
    if (hipHostGetDevicePointer(reinterpret_cast<void **>(&ws.host_d), ws.host, 0) != hipSuccess) ws.host_d = nullptr;
    ws.cap = cap;
    return ORBX_OK;
}

// Brings [off, off + bytes) of the device arena into the pinned arena after
// the call's last kernel, and waits for it: the last workgroup of that kernel
// to finish (HostTail, orbx_device.h) writes the bytes straight into the
// (device-visible) pinned buffer and then raises a flag the host polls,
// instead of a copy plus a stream synchronisation (about 10 us of wake-up for
// a call of ~50 us).  ws_tail prepares it before that launch (done_d: a
// device counter the inputs upload as zero; blocks: the kernel's workgroups;
// t.flag stays nullptr when the output takes the copy: large outputs, no
// device-visible pinned arena), ws_wait waits after.  Caller holds ws.mu.
void ws_tail(CallWs &ws, size_t off, size_t bytes, uint32_t *done_d, int blocks, HostTail &t);
int ws_wait(CallWs &ws, const HostTail &t, size_t off, size_t bytes);

template <typename T>
inline T *at(uint8_t *base, size_t off) { return reinterpret_cast<T *>(base + off); }

inline void put(CallWs &ws, size_t off, const void *src, size_t bytes) {
    if (bytes && src) std::memcpy(ws.host + off, src, bytes);
}
inline void get(CallWs &ws, size_t off, void *dst, size_t bytes) {
    if (bytes && dst) std::memcpy(dst, ws.host + off, bytes);
}


}  // namespace orbx

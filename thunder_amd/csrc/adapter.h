// adapter.h -- host-side helpers shared by the reference-shaped host adapters
// (interface.hip, recon_iface.hip): an RAII device buffer, a current-device
// guard and the per-device fan-out of an image batch.
#pragma once
#include <algorithm>
#include <string>
#include <thread>
#include <vector>

#include "common.h"

namespace thx {

// RAII device buffer on the device current at alloc(); errors surface as
// THX_ERR_NOMEM through THX_DALLOC.
struct DBuf {
    void* p = nullptr;
    int dev = -1;
    hipError_t alloc(size_t bytes)
    {
        (void)hipGetDevice(&dev);
        return hipMalloc(&p, bytes > 0 ? bytes : 1);
    }
    ~DBuf()
    {
        if (!p) return;
        int cur = 0;
        (void)hipGetDevice(&cur);
        if (dev >= 0 && dev != cur) (void)hipSetDevice(dev);
        (void)hipFree(p);
        if (dev >= 0 && dev != cur) (void)hipSetDevice(cur);
    }
    DBuf() = default;
    DBuf(const DBuf&) = delete;
    DBuf& operator=(const DBuf&) = delete;
    DBuf(DBuf&& o) noexcept : p(o.p), dev(o.dev) { o.p = nullptr; }
    template <typename T> T* as() const { return static_cast<T*>(p); }
};

#define THX_DALLOC(buf, bytes)                                                 \
    do {                                                                       \
        if ((buf).alloc(bytes) != hipSuccess) {                                \
            thx::set_error("device allocation of %zu bytes failed",           \
                           (size_t)(bytes));                                   \
            return THX_ERR_NOMEM;                                              \
        }                                                                      \
    } while (0)

// Restores the caller's current device when the adapter returns.
struct DeviceGuard {
    int dev = 0;
    DeviceGuard() { (void)hipGetDevice(&dev); }
    ~DeviceGuard() { (void)hipSetDevice(dev); }
};

// Runs fn(slot, device, l0, l1) for a contiguous image block per device, one
// host thread per device (each with its device current); the first failure's
// status and message come back to the caller's thread.
template <typename Fn>
int on_devices(const std::vector<int>& devs, int nImg, Fn&& fn)
{
    const int nd = (int)devs.size();
    std::vector<int> st(nd, THX_OK);
    std::vector<std::string> msg(nd);
    auto run = [&](int k) {
        const int per = (nImg + nd - 1) / nd;
        const int l0 = std::min(nImg, k * per), l1 = std::min(nImg, l0 + per);
        if (hipSetDevice(devs[k]) != hipSuccess) {
            st[k] = THX_ERR_HIP;
            msg[k] = "hipSetDevice failed";
            return;
        }
        st[k] = fn(k, devs[k], l0, l1);
        if (st[k] != THX_OK) msg[k] = thx_last_error();
    };
    if (nd == 1) {
        run(0);
    } else {
        std::vector<std::thread> th;
        for (int k = 0; k < nd; k++) th.emplace_back(run, k);
        for (auto& t : th) t.join();
    }
    for (int k = 0; k < nd; k++)
        if (st[k] != THX_OK) {
            thx::set_error("device %d: %s", devs[k], msg[k].c_str());
            return st[k];
        }
    return THX_OK;
}

}  // namespace thx

// Thread-local error reporting, per-device launch setup and the ABI version
// of the C-ABI (dfhip.h).
#include "common.h"

#include <stdarg.h>

#include <map>
#include <mutex>
#include <tuple>

namespace dfhip {

static thread_local char g_last_error[512] = "";

void set_error(const char *fmt, ...) {
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(g_last_error, sizeof(g_last_error), fmt, ap);
    va_end(ap);
}

int current_device() {
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess) dev = 0;
    return dev;
}

uint32_t device_cus() {
    int v = 0;
    if (hipDeviceGetAttribute(&v, hipDeviceAttributeMultiprocessorCount, current_device()) !=
            hipSuccess ||
        v <= 0)
        v = 256;
    return (uint32_t)v;
}

// Per-(kernel, device) launch facts.  The library keeps no mode state: these
// are caches of device properties, filled once per (kernel, device) under a
// lock, so two host threads or two devices in one process each get their own
// setup (a flag per process would skip the attribute on a second device).
namespace {
typedef std::tuple<const void *, int, int> LaunchKey;  // kernel, device, threads / bytes
std::mutex &launch_mutex() {
    static std::mutex m;
    return m;
}
std::map<LaunchKey, uint32_t> &launch_facts() {
    static std::map<LaunchKey, uint32_t> f;
    return f;
}
}  // namespace

void ensure_dynamic_lds(const void *kernel, int bytes) {
    const LaunchKey key{kernel, current_device(), -bytes};
    std::lock_guard<std::mutex> lock(launch_mutex());
    auto &f = launch_facts();
    if (f.count(key)) return;
    (void)hipFuncSetAttribute(kernel, hipFuncAttributeMaxDynamicSharedMemorySize, bytes);
    f[key] = 1;
}

uint32_t resident_blocks(const void *kernel, int threads, int fallback_per_cu) {
    const int dev = current_device();
    const LaunchKey key{kernel, dev, threads};
    {
        std::lock_guard<std::mutex> lock(launch_mutex());
        auto &f = launch_facts();
        auto it = f.find(key);
        if (it != f.end()) return it->second;
    }
    int per_cu = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, kernel, threads, 0) != hipSuccess ||
        per_cu <= 0)
        per_cu = fallback_per_cu;
    const uint32_t n = (uint32_t)per_cu * device_cus();
    std::lock_guard<std::mutex> lock(launch_mutex());
    launch_facts()[key] = n;
    return n;
}

}  // namespace dfhip

// A hash of include/dfhip.h, passed by the build (dfhip_build.abi_hash).
#ifndef DFHIP_ABI_HASH
#error "build with -DDFHIP_ABI_HASH=<hash of include/dfhip.h> (dfhip_build.py)"
#endif
extern "C" int dfhip_abi_version(void) { return DFHIP_ABI_HASH; }
extern "C" const char *dfhip_last_error(void) { return dfhip::g_last_error; }

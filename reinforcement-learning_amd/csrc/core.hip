// core.hip -- error channel and version of the rlgpu C ABI (include/rlgpu_core.h).
#include "common.hpp"

namespace rlgpu {
static thread_local std::string g_last_error;
void set_last_error(const std::string& msg) { g_last_error = msg; }
}  // namespace rlgpu

extern "C" const char* rlgpu_last_error(void) { return rlgpu::g_last_error.c_str(); }

extern "C" int rlgpu_abi_version(void) { return 100; }

extern "C" int rlgpu_device_count(void) {
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess) {
        (void)hipGetLastError();
        return 0;
    }
    return n;
}

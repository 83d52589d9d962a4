// common.hpp -- shared host helpers for the rlgpu C ABI implementation.
// Error handling mirrors the reference's throw-on-error (RG_ERR_CLOSE,
// GigaLearnCPP/RLGymCPP/src/RLGymCPP/Framework.h:16-21) but converts to the
// int-status + thread-local-message convention of include/rlgpu_core.h.
#pragma once
#include <hip/hip_runtime.h>
#include <cstdint>
#include <cstdio>
#include <stdexcept>
#include <string>

#include "../../include/rlgpu_core.h"

namespace rlgpu {

void set_last_error(const std::string& msg);

struct Error : std::runtime_error {
    int code;
    Error(int c, const std::string& m) : std::runtime_error(m), code(c) {}
};

#define RLGPU_CHECK_HIP(expr)                                                                \
    do {                                                                                     \
        hipError_t _e = (expr);                                                              \
        if (_e != hipSuccess)                                                                \
            throw ::rlgpu::Error(RLGPU_ERR_HIP, std::string(#expr " failed: ") +             \
                                                    hipGetErrorString(_e));                  \
    } while (0)

#define RLGPU_REQUIRE(cond, msg)                                                             \
    do {                                                                                     \
        if (!(cond)) throw ::rlgpu::Error(RLGPU_ERR_INVALID_ARG, std::string(msg));          \
    } while (0)

// Run a body, converting exceptions into a status code (no exception crosses the ABI).
template <class F>
inline int guarded(F&& f) {
    try {
        f();
        return RLGPU_OK;
    } catch (const Error& e) {
        set_last_error(e.what());
        return e.code;
    } catch (const std::bad_alloc&) {
        set_last_error("host allocation failed");
        return RLGPU_ERR_OOM;
    } catch (const std::exception& e) {
        set_last_error(e.what());
        return RLGPU_ERR_STATE;
    }
}

inline hipStream_t as_stream(void* s) { return reinterpret_cast<hipStream_t>(s); }

inline unsigned ceil_div(int64_t a, int64_t b) { return (unsigned)((a + b - 1) / b); }

}  // namespace rlgpu

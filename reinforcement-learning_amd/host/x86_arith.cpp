// x86_arith.cpp -- this host's rsqrtss table (include/rlgpu_arith.h).  Host code (g++).
//
// The reference's x86 Bullet normalises vectors with rsqrtss plus one Newton step
// (btVector3::normalize, btVector3.h:304-345).  rsqrtss is an approximation whose exact results are
// the CPU's own, so the kernels cannot compute it from a formula: the library executes the
// instruction once for every input of [1, 4) (2 x 2^23 values), finds the mantissa bits its result
// depends on, checks that every other exponent only rescales the result, checks the special inputs,
// and keeps the small table the kernels index (env.hip uploads it into EnvConst).
#include <algorithm>
#include <cmath>
#include <cstdint>
#include <cstring>
#include <mutex>
#include <string>
#include <vector>

#if defined(__x86_64__) || defined(__i386__)
#include <xmmintrin.h>
#define RLGPU_HAVE_RSQRTSS 1
#endif

#include "../../include/rlgpu_arith.h"
#include "../csrc/common.hpp"

namespace rlgpu {
namespace {

struct RsqrtTable {
    bool ok = false;
    int bits = 0;
    std::vector<uint32_t> t;  // [2 << bits]
    std::string why;
};

inline uint32_t fbits(float f) {
    uint32_t u;
    std::memcpy(&u, &f, 4);
    return u;
}
inline float bitsf(uint32_t u) {
    float f;
    std::memcpy(&f, &u, 4);
    return f;
}

#ifdef RLGPU_HAVE_RSQRTSS
// the instruction itself (noinline: the compiler never sees through it)
__attribute__((noinline)) float hw_rsqrtss(float x) { return _mm_cvtss_f32(_mm_rsqrt_ss(_mm_set_ss(x))); }
#endif

// The emulation the device runs (env_device.hpp x86_rsqrtss restates it): zero / denormal -> +-inf,
// +inf -> 0, NaN -> quiet NaN, negative -> the default NaN; a normal x = 2^(2q + p) * 1.m reads
// entry (p, top `bits` of m), the result of 2^p * 1.m, and scales it by 2^-q.
float emulate(const RsqrtTable& T, float x) {
    const uint32_t u = fbits(x);
    const uint32_t e = (u >> 23) & 0xffu, m = u & 0x7fffffu;
    if (e == 0u) return bitsf((u & 0x80000000u) | 0x7f800000u);
    if (e == 0xffu) {
        if (m) return bitsf(u | 0x400000u);
        return (u >> 31) ? bitsf(0xffc00000u) : 0.f;
    }
    if (u >> 31) return bitsf(0xffc00000u);
    const int E = (int)e - 127, p = E & 1, q = (E - p) / 2;
    const uint32_t r = T.t[((uint32_t)p << T.bits) | (m >> (23 - T.bits))];
    return bitsf((uint32_t)((int32_t)r - q * (1 << 23)));
}

RsqrtTable capture() {
    RsqrtTable T;
#ifndef RLGPU_HAVE_RSQRTSS
    T.why = "the host is not x86: no rsqrtss to read";
    return T;
#else
    // every input of [1, 4): index (p << 23) | mantissa
    std::vector<uint32_t> full((size_t)1 << 24);
    for (uint32_t i = 0; i < (1u << 24); i++) full[i] = fbits(hw_rsqrtss(bitsf(((127u + (i >> 23)) << 23) | (i & 0x7fffffu))));
    // the result may only change at multiples of 2^(23 - bits): OR the change points, keep their
    // common alignment
    uint32_t changes = 0;
    for (uint32_t i = 1; i < (1u << 24); i++)
        if ((i & 0x7fffffu) && full[i] != full[i - 1]) changes |= i & 0x7fffffu;
    const int align = changes ? __builtin_ctz(changes) : 23;
    T.bits = 23 - align;
    if (T.bits < 1) T.bits = 1;
    T.t.resize((size_t)2 << T.bits);
    for (uint32_t p = 0; p < 2; p++)
        for (uint32_t h = 0; h < (1u << T.bits); h++) T.t[(p << T.bits) | h] = full[(p << 23) | (h << (23 - T.bits))];
    // every exponent only rescales (a sample of the entries when the table is large)
    const uint32_t step = T.bits > 14 ? 1u << (T.bits - 14) : 1u;
    for (uint32_t e = 1; e < 255; e++) {
        const uint32_t p = (e - 127u) & 1u;
        for (uint32_t h = 0; h < (1u << T.bits); h += step) {
            for (uint32_t lo : {0u, (1u << (23 - T.bits)) - 1u}) {
                const float x = bitsf((e << 23) | (h << (23 - T.bits)) | lo);
                if (fbits(hw_rsqrtss(x)) != fbits(emulate(T, x))) {
                    T.why = "rsqrtss does not scale with the exponent as the emulation assumes (exponent " +
                            std::to_string(e) + ", parity " + std::to_string(p) + ")";
                    return T;
                }
            }
        }
    }
    // special inputs
    for (uint32_t u : {0x00000000u, 0x80000000u, 0x00000001u, 0x007fffffu, 0x80400000u, 0x7f800000u, 0xff800000u,
                       0x7fc00000u, 0x7fa00000u, 0xbf800000u, 0x00800000u, 0x7f7fffffu}) {
        const uint32_t a = fbits(hw_rsqrtss(bitsf(u))), b = fbits(emulate(T, bitsf(u)));
        const bool nan_a = (a & 0x7f800000u) == 0x7f800000u && (a & 0x7fffffu), nan_b = (b & 0x7f800000u) == 0x7f800000u && (b & 0x7fffffu);
        if (a != b && !(nan_a && nan_b)) {
            T.why = "rsqrtss special input " + std::to_string(u) + " differs from the emulation";
            return T;
        }
    }
    T.ok = true;
    return T;
#endif
}

}  // namespace

const RsqrtTable& rsqrt_table() {
    static RsqrtTable T;
    static std::once_flag once;
    std::call_once(once, [] { T = capture(); });
    return T;
}

// for env.hip: the table, or an RLGPU_ERR_UNSUPPORTED error naming why the host's cannot be used
const std::vector<uint32_t>& x86_rsqrt_table_or_throw(int* bits) {
    const RsqrtTable& T = rsqrt_table();
    if (!T.ok) throw Error(RLGPU_ERR_UNSUPPORTED, "x86 arithmetic modes need this host's rsqrtss table: " + T.why);
    *bits = T.bits;
    return T.t;
}

}  // namespace rlgpu

extern "C" int rlgpu_x86_rsqrt_table(uint32_t* h_table, int64_t cap, int32_t* bits) {
    return rlgpu::guarded([&] {
        RLGPU_REQUIRE(bits, "rlgpu_x86_rsqrt_table: null bits");
        int b = 0;
        const std::vector<uint32_t>& t = rlgpu::x86_rsqrt_table_or_throw(&b);
        *bits = b;
        if (h_table) {
            RLGPU_REQUIRE(cap >= (int64_t)t.size(), "rlgpu_x86_rsqrt_table: table needs 2 << bits entries");
            std::memcpy(h_table, t.data(), t.size() * sizeof(uint32_t));
        }
    });
}

extern "C" float rlgpu_x86_rsqrtss_emulated(float x) {
    const rlgpu::RsqrtTable& T = rlgpu::rsqrt_table();
    if (!T.ok) return 0.f / 0.f;
    return rlgpu::emulate(T, x);
}

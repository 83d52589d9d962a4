// Micro-benchmark of one box-triangle query on one lane (gjk.hpp): in-kernel clock64 cycles of the whole
// query, for a shallow (GJK only) and a deep (penetration solver) pose, LDS-first and HBM work sets.
// Built with different flags by tools/micro/run_gjk_micro.sh (experiments, not product code).
#include <hip/hip_runtime.h>
#include <cstdio>

__device__ long long g_trace[64];
__device__ int g_tid[64];
__device__ int g_ntrace;
#define RLGPU_GJK_TRACE(id) { if (__lane_id() == 0 && g_ntrace < 64) { g_tid[g_ntrace] = (id); g_trace[g_ntrace++] = clock64(); } }

#include "../../reinforcement-learning_amd/csrc/gjk.hpp"

using namespace rl;

__global__ void __launch_bounds__(64) k(int mode, float gap, unsigned long long* out, float* res, gjk::GjkScratch* hbm) {
    __shared__ char small[gjk::kSmallBytes];
    __shared__ int lock;
    lock = 0;
    if (mode < 2 && threadIdx.x != 0) return;  // mode 2: the whole wave runs the query (wave-mode EPA)
    const v3 impl = v3{1.1664109f, 0.8283349f, 0.3479319f};
    const float margin = 0.0386591f;
    // RLGPU_ARITH_SCALAR (2): no rsqrtss table on the device in this program
    gjk::Shape sh{impl, margin, v3{-50.f, -50.f, 0.f}, v3{50.f, -50.f, 0.f}, v3{0.f, 60.f, 0.f}, 2};
    const float c0 = 0.3f, s0 = 0.2f;  // a tilted box
    m3 R = m3{v3{1, 0, 0}, v3{0, c0 / sqrtf(c0 * c0 + s0 * s0), -s0 / sqrtf(c0 * c0 + s0 * s0)},
              v3{0, s0 / sqrtf(c0 * c0 + s0 * s0), c0 / sqrtf(c0 * c0 + s0 * s0)}};
    float ext = fabsf(R.r2.x) * (impl.x + margin) + fabsf(R.r2.y) * (impl.y + margin) + fabsf(R.r2.z) * (impl.z + margin);
    v3 c = v3{0.1f, 0.2f, ext + gap};
    gjk::Scr slow = gjk::hbm_view(hbm);
    gjk::Scr fast = gjk::lds_view(small);
    v3 n, p;
    float d = 0;
    int pen = 0;
    gjk::Scr wave = gjk::wave_view(small);
    if (threadIdx.x == 0) g_ntrace = 0;
    long long t0 = clock64();
    bool hit = mode == 2 ? gjk::box_triangle(R, c, sh, 0.02f, &wave, nullptr, slow, n, p, d, &pen, gjk::kPenWave)
                         : gjk::box_triangle(R, c, sh, 0.02f, mode ? &fast : nullptr, &lock, slow, n, p, d, &pen);
    if (threadIdx.x != 0) return;
    long long t1 = clock64();
    out[0] = (unsigned long long)(t1 - t0);
    out[1] = (unsigned long long)pen;
    out[2] = (unsigned long long)g_ntrace;
    out[3] = g_ntrace ? (unsigned long long)(g_trace[0] - t0) : 0;
    out[4] = g_ntrace > 1 ? (unsigned long long)((g_trace[g_ntrace - 1] - g_trace[0]) / (g_ntrace - 1)) : 0;
    out[5] = g_ntrace ? (unsigned long long)(t1 - g_trace[g_ntrace - 1]) : 0;
    res[0] = hit;
    res[1] = d;
}

int main() {
    unsigned long long* out;
    float* res;
    gjk::GjkScratch* hbm;
    hipMalloc(&out, 64);
    hipMalloc(&res, 8);
    hipMalloc(&hbm, sizeof(gjk::GjkScratch));
    for (int mode = 0; mode < 3; mode++)
        for (float gap : {0.01f, -0.02f, -0.1f, -0.3f}) {
            unsigned long long best = ~0ull, first = 0, o[8];
            float r[2];
            for (int rep = 0; rep < 5; rep++) {
                hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, mode, gap, out, res, hbm);
                hipError_t err = hipGetLastError();
                if (err == hipSuccess) err = hipDeviceSynchronize();
                if (err != hipSuccess) {
                    printf("launch failed: %s\n", hipGetErrorString(err));
                    return 1;
                }
                hipMemcpy(o, out, 64, hipMemcpyDeviceToHost);
                hipMemcpy(r, res, 8, hipMemcpyDeviceToHost);
                if (o[0] < best) best = o[0];
                if (rep == 0) first = o[0];
            }
            if (mode >= 1 && gap < -0.05f) {
                long long tr[64];
                int id[64], nt;
                hipMemcpyFromSymbol(tr, HIP_SYMBOL(g_trace), sizeof tr);
                hipMemcpyFromSymbol(id, HIP_SYMBOL(g_tid), sizeof id);
                hipMemcpyFromSymbol(&nt, HIP_SYMBOL(g_ntrace), sizeof nt);
                printf("  trace:");
                for (int k = 1; k < nt; k++) printf(" %d:%lld", id[k], tr[k] - tr[k - 1]);
                printf("\n");
            }
            printf("%s gap %+.2f: %8llu cycles (first run %llu) (pen-solver calls %llu, hit %.0f depth %+.5f) GJK iterations %llu: first %llu, "
                   "per iteration %llu, after the loop %llu\n", mode == 2 ? "wave-mode" : mode ? "LDS-first" : "HBM-only ", gap, best, first, o[1], r[0], r[1], o[2],
                   o[3], o[4], o[5]);
        }
    return 0;
}

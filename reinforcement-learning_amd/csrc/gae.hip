// gae.hip -- GAE on MI355X.
//
// Semantics follow GGL::GAE::Compute
// (GigaLearnCPP/src/private/GigaLearnCPP/PPO/GAE.cpp:7-208):
//   * rewards normalised by 1/returnStd when returnStd is not 0 or 1 (:74-76,104-167),
//     then clipped to +-clipRange (clipRange > 0);
//   * nextVal = 0 on NORMAL, truncValPreds[k] on the k-th TRUNCATED step (:86-96),
//     V[t+1] otherwise, 0 on the last step (:97-101);
//   * delta = r_hat + gamma*nextVal - V;  A_t = delta + gamma*lambda*nd_t*A_{t+1} (:177-190);
//   * returns use the RAW reward: R_t = r_t + R_{t+1}*gamma*nd_t (:183-185);
//   * target = V + A (:200); clip portion = (sum|n| - sum|clip(n)|)/max(sum|n|,1e-7) (:202-206).
//
// Two device layouts:
//   * rollout [T][N]: one lane per agent column walks t backwards in the reference's
//     operation order (compiled with -ffp-contract=off) -> bit-identical to the oracle;
//     memory access is coalesced across the agent dimension, so it is an HBM-streaming
//     kernel (21 B per agent-step algorithmic).
//   * flat (episode-concatenated, the reference's own input): A_t = d_t + c_t*A_{t+1} is a
//     composition of affine maps, (cL,dL)o(cR,dR) = (cL*cR, dL + cL*dR).  Terminals make c=0,
//     so one non-segmented reverse scan is exactly the segmented GAE.  Chunked 3-pass scan:
//     trunc counts -> chunk summaries -> chunk carries -> apply.  Within a chunk every lane
//     composes 8 contiguous elements, a 64-lane shuffle suffix-scan combines lanes and LDS
//     combines the 4 waves of a 256-thread workgroup.
#include "common.hpp"
#include "../../include/rlgpu_gae.h"

namespace {

constexpr int kThreads = 256;
constexpr int kPerThread = 8;
constexpr int kChunk = kThreads * kPerThread;  // 2048 elements per workgroup
constexpr int8_t kNormal = 1, kTruncated = 2;   // RLGC::TerminalType (TerminalCondition.h:6-11)

struct Aff {
    float c, d;
};
__device__ __forceinline__ Aff compose(Aff L, Aff R) { return {L.c * R.c, L.d + L.c * R.d}; }
__device__ __forceinline__ Aff shfl_down_aff(Aff a, int off) {
    return {__shfl_down(a.c, off, 64), __shfl_down(a.d, off, 64)};
}

// Per-element GAE parameters shared by the flat kernels.
struct GaeParams {
    const float* rews;
    const int8_t* terms;
    const float* vals;
    const float* trunc_vals;
    int64_t M;
    int64_t num_truncs;
    float gamma, gamma_lambda, inv_std;
    bool normalize, clip;
    float clip_range;
};

// Inclusive suffix scan over the 64 lanes of a wave: S_l = f_l o ... o f_63.
__device__ __forceinline__ Aff wave_suffix_inclusive(Aff a, int lane) {
#pragma unroll
    for (int off = 1; off < 64; off <<= 1) {
        Aff o = shfl_down_aff(a, off);
        if (lane + off < 64) a = compose(a, o);
    }
    return a;
}

// Exclusive forward prefix sum of an int over a 256-thread block.
__device__ __forceinline__ int block_excl_prefix_int(int v, int* smem4) {
    int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    int inc = v;
#pragma unroll
    for (int off = 1; off < 64; off <<= 1) {
        int o = __shfl_up(inc, off, 64);
        if (lane >= off) inc += o;
    }
    if (lane == 63) smem4[wave] = inc;
    __syncthreads();
    int base = 0;
    for (int w = 0; w < wave; ++w) base += smem4[w];
    __syncthreads();
    return base + inc - v;
}

// Block-wide exclusive suffix composition for two affine maps (adv + ret chains).
// Returns for this thread the composition of all threads to its right in the block.
__device__ __forceinline__ void block_suffix_excl(Aff& a, Aff& r, Aff* smem_a, Aff* smem_r) {
    int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    Aff sa = wave_suffix_inclusive(a, lane);
    Aff sr = wave_suffix_inclusive(r, lane);
    Aff ea = shfl_down_aff(sa, 1), er = shfl_down_aff(sr, 1);
    if (lane == 63) ea = er = Aff{1.f, 0.f};
    if (lane == 0) {
        smem_a[wave] = sa;
        smem_r[wave] = sr;
    }
    __syncthreads();
    Aff ta{1.f, 0.f}, tr{1.f, 0.f};
    for (int w = (kThreads / 64) - 1; w > wave; --w) {
        ta = compose(smem_a[w], ta);
        tr = compose(smem_r[w], tr);
    }
    __syncthreads();
    a = compose(ea, ta);
    r = compose(er, tr);
}

// Builds the 8 per-element maps of this thread.  trunc_base = global index of the first
// truncation at or after this thread's first element.
__device__ __forceinline__ void element_maps(const GaeParams& p, int64_t i0, int64_t trunc_base,
                                             Aff* fa, Aff* fr, float* nrew) {
    int64_t k = trunc_base;
#pragma unroll
    for (int j = 0; j < kPerThread; ++j) {
        int64_t i = i0 + j;
        if (i >= p.M) {
            fa[j] = fr[j] = Aff{1.f, 0.f};
            nrew[j] = 0.f;
            continue;
        }
        int8_t t = p.terms[i];
        float rew = p.rews[i];
        float n = rew;
        if (p.normalize) {
            n = rew * p.inv_std;
            if (p.clip) n = fminf(fmaxf(n, -p.clip_range), p.clip_range);
        }
        nrew[j] = n;
        float nd = (t == kNormal || t == kTruncated) ? 0.f : 1.f;
        float next;
        if (t == kNormal) next = 0.f;
        else if (t == kTruncated) next = (k < p.num_truncs) ? p.trunc_vals[k] : 0.f;
        else if (i < p.M - 1) next = p.vals[i + 1];
        else next = 0.f;
        if (t == kTruncated) ++k;
        float delta = (n + p.gamma * next) - p.vals[i];
        fa[j] = Aff{p.gamma_lambda * nd, delta};
        fr[j] = Aff{p.gamma * nd, rew};
    }
}

__global__ void __launch_bounds__(kThreads) k_trunc_count(const int8_t* terms, int64_t M, int* counts) {
    __shared__ int s[4];
    int64_t i0 = (int64_t)blockIdx.x * kChunk + (int64_t)threadIdx.x * kPerThread;
    int c = 0;
    for (int j = 0; j < kPerThread; ++j)
        if (i0 + j < M && terms[i0 + j] == kTruncated) ++c;
    int excl = block_excl_prefix_int(c, s);
    if (threadIdx.x == kThreads - 1) counts[blockIdx.x] = excl + c;
}

// Single workgroup: exclusive prefix of chunk trunc counts (sequential per thread segment).
__global__ void __launch_bounds__(kThreads) k_scan_counts(const int* counts, int nchunks, int64_t* offsets,
                                                          int64_t* total) {
    __shared__ int s[4];
    int per = (nchunks + kThreads - 1) / kThreads;
    int b0 = threadIdx.x * per;
    int local = 0;
    for (int b = b0; b < b0 + per && b < nchunks; ++b) local += counts[b];
    int base = block_excl_prefix_int(local, s);
    int64_t run = base;
    for (int b = b0; b < b0 + per && b < nchunks; ++b) {
        offsets[b] = run;
        run += counts[b];
    }
    if (threadIdx.x == kThreads - 1) *total = run;
}

// Pass 1: per-chunk composed maps (adv chain, return chain).
__global__ void __launch_bounds__(kThreads) k_chunk_summary(GaeParams p, const int64_t* trunc_offsets,
                                                            float4* summaries) {
    __shared__ int s_int[4];
    __shared__ Aff s_a[4], s_r[4];
    int64_t i0 = (int64_t)blockIdx.x * kChunk + (int64_t)threadIdx.x * kPerThread;
    int c = 0;
    for (int j = 0; j < kPerThread; ++j)
        if (i0 + j < p.M && p.terms[i0 + j] == kTruncated) ++c;
    int64_t tb = trunc_offsets[blockIdx.x] + block_excl_prefix_int(c, s_int);
    Aff fa[kPerThread], fr[kPerThread];
    float nrew[kPerThread];
    element_maps(p, i0, tb, fa, fr, nrew);
    Aff ta{1.f, 0.f}, tr{1.f, 0.f};
#pragma unroll
    for (int j = kPerThread - 1; j >= 0; --j) {
        ta = compose(fa[j], ta);
        tr = compose(fr[j], tr);
    }
    // Composition of the whole chunk = thread 0's map composed with everything to its right.
    Aff ea = ta, er = tr;
    block_suffix_excl(ea, er, s_a, s_r);
    if (threadIdx.x == 0) {
        Aff A = compose(ta, ea), R = compose(tr, er);
        summaries[blockIdx.x] = make_float4(A.c, A.d, R.c, R.d);
    }
}

// Pass 2 (single workgroup): carry-in value of each chunk = (chunks to the right)(0).
__global__ void __launch_bounds__(kThreads) k_chunk_carry(const float4* summaries, int nchunks, float2* carry) {
    __shared__ Aff s_a[4], s_r[4];
    int per = (nchunks + kThreads - 1) / kThreads;
    int b0 = threadIdx.x * per;
    Aff ta{1.f, 0.f}, tr{1.f, 0.f};
    for (int b = min(b0 + per, nchunks) - 1; b >= b0; --b) {
        float4 s = summaries[b];
        ta = compose(Aff{s.x, s.y}, ta);
        tr = compose(Aff{s.z, s.w}, tr);
    }
    Aff ea = ta, er = tr;
    block_suffix_excl(ea, er, s_a, s_r);
    // Value entering this thread's right edge: (everything right of it)(0).
    float va = ea.d, vr = er.d;
    for (int b = min(b0 + per, nchunks) - 1; b >= b0; --b) {
        carry[b] = make_float2(va, vr);
        float4 s = summaries[b];
        va = s.y + s.x * va;
        vr = s.w + s.z * vr;
    }
}

// Pass 3: apply carries and write A, target, R; accumulate clip-portion sums.
__global__ void __launch_bounds__(kThreads) k_apply(GaeParams p, const int64_t* trunc_offsets, const float2* carry,
                                                    float* adv, float* target, float* ret, float* clip_sums) {
    __shared__ int s_int[4];
    __shared__ Aff s_a[4], s_r[4];
    __shared__ float s_sum[2][4];
    int64_t i0 = (int64_t)blockIdx.x * kChunk + (int64_t)threadIdx.x * kPerThread;
    int c = 0;
    for (int j = 0; j < kPerThread; ++j)
        if (i0 + j < p.M && p.terms[i0 + j] == kTruncated) ++c;
    int64_t tb = trunc_offsets[blockIdx.x] + block_excl_prefix_int(c, s_int);
    Aff fa[kPerThread], fr[kPerThread];
    float nrew[kPerThread];
    element_maps(p, i0, tb, fa, fr, nrew);
    Aff ta{1.f, 0.f}, tr{1.f, 0.f};
#pragma unroll
    for (int j = kPerThread - 1; j >= 0; --j) {
        ta = compose(fa[j], ta);
        tr = compose(fr[j], tr);
    }
    Aff ea = ta, er = tr;
    block_suffix_excl(ea, er, s_a, s_r);
    float2 cin = carry[blockIdx.x];
    float xa = ea.d + ea.c * cin.x;
    float xr = er.d + er.c * cin.y;
    float sabs = 0.f, sclip = 0.f;
#pragma unroll
    for (int j = kPerThread - 1; j >= 0; --j) {
        int64_t i = i0 + j;
        xa = fa[j].d + fa[j].c * xa;
        xr = fr[j].d + fr[j].c * xr;
        if (i < p.M) {
            adv[i] = xa;
            ret[i] = xr;
            target[i] = p.vals[i] + xa;
            if (p.normalize) {
                float raw = p.rews[i] * p.inv_std;
                sabs += fabsf(raw);
                sclip += fabsf(nrew[j]);
            }
        }
    }
    if (clip_sums && p.normalize) {
        for (int off = 32; off > 0; off >>= 1) {
            sabs += __shfl_down(sabs, off, 64);
            sclip += __shfl_down(sclip, off, 64);
        }
        int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
        if (lane == 0) {
            s_sum[0][wave] = sabs;
            s_sum[1][wave] = sclip;
        }
        __syncthreads();
        if (threadIdx.x == 0) {
            atomicAdd(&clip_sums[0], s_sum[0][0] + s_sum[0][1] + s_sum[0][2] + s_sum[0][3]);
            atomicAdd(&clip_sums[1], s_sum[1][0] + s_sum[1][1] + s_sum[1][2] + s_sum[1][3]);
        }
    }
}

// Rollout layout: one lane per agent column, exact reference order (GAE.cpp:169-193).
__global__ void __launch_bounds__(256) k_gae_rollout(const float* __restrict__ rews, const int8_t* __restrict__ terms,
                                                     const float* __restrict__ vals, const float* __restrict__ trunc_vals,
                                                     const float* __restrict__ boot_vals, int T, int N, float gamma,
                                                     float gamma_lambda, float inv_std, int normalize, int clip,
                                                     float clip_range, float* __restrict__ adv,
                                                     float* __restrict__ target, float* __restrict__ ret,
                                                     float* clip_sums) {
    int n = blockIdx.x * blockDim.x + threadIdx.x;
    float sabs = 0.f, sclip = 0.f;
    if (n < N) {
        float prevLambda = 0.f, prevRet = 0.f;
        for (int t = T - 1; t >= 0; --t) {
            int64_t i = (int64_t)t * N + n;
            int8_t term = terms[i];
            float rew = rews[i];
            float cur = rew;
            if (normalize) {
                cur = rew * inv_std;
                sabs += fabsf(cur);
                if (clip) cur = fminf(fmaxf(cur, -clip_range), clip_range);
                sclip += fabsf(cur);
            }
            float done = (term == kNormal) ? 1.f : 0.f;
            float trunc = (term == kTruncated) ? 1.f : 0.f;
            float nd = (1.f - done) * (1.f - trunc);
            float nextVal;
            if (term == kNormal) nextVal = 0.f;
            else if (term == kTruncated) nextVal = trunc_vals ? trunc_vals[i] : 0.f;
            else if (t < T - 1) nextVal = vals[i + N];
            else nextVal = boot_vals ? boot_vals[n] : 0.f;
            float v = vals[i];
            float predReturn = cur + gamma * nextVal;
            float delta = predReturn - v;
            float curReturn = rew + prevRet * gamma * nd;
            ret[i] = curReturn;
            prevLambda = delta + gamma_lambda * nd * prevLambda;
            adv[i] = prevLambda;
            target[i] = v + prevLambda;
            prevRet = curReturn;
        }
    }
    if (clip_sums && normalize) {
        for (int off = 32; off > 0; off >>= 1) {
            sabs += __shfl_down(sabs, off, 64);
            sclip += __shfl_down(sclip, off, 64);
        }
        if ((threadIdx.x & 63) == 0) {
            atomicAdd(&clip_sums[0], sabs);
            atomicAdd(&clip_sums[1], sclip);
        }
    }
}

// One lane per complete trajectory of a flat batch (rlgpu_gae_segments): the same recursion as
// k_gae_rollout over rows off + len - 1 .. off, the segment's terminal bootstrapped from trunc_vals[tidx]
// (code 2) or 0 (code 1), prevLambda / prevRet starting at 0.
__global__ void __launch_bounds__(256) k_gae_segments(const float* __restrict__ rews, const int8_t* __restrict__ terms,
                                                      const float* __restrict__ vals, const float* __restrict__ trunc_vals,
                                                      const int64_t* __restrict__ seg_off, const int32_t* __restrict__ seg_len,
                                                      const int32_t* __restrict__ seg_tidx, int64_t K, float gamma,
                                                      float gamma_lambda, float inv_std, int normalize, int clip,
                                                      float clip_range, float* __restrict__ adv, float* __restrict__ target,
                                                      float* __restrict__ ret, float* clip_sums) {
    const int64_t k = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    float sabs = 0.f, sclip = 0.f;
    if (k < K) {
        const int64_t off = seg_off[k];
        const int L = seg_len[k], tidx = seg_tidx[k];
        float prevLambda = 0.f, prevRet = 0.f;
        for (int j = L - 1; j >= 0; --j) {
            const int64_t i = off + j;
            const int8_t term = terms[i];
            const float rew = rews[i];
            float cur = rew;
            if (normalize) {
                cur = rew * inv_std;
                sabs += fabsf(cur);
                if (clip) cur = fminf(fmaxf(cur, -clip_range), clip_range);
                sclip += fabsf(cur);
            }
            const float done = (term == kNormal) ? 1.f : 0.f;
            const float trunc = (term == kTruncated) ? 1.f : 0.f;
            const float nd = (1.f - done) * (1.f - trunc);
            float nextVal;
            if (term == kNormal) nextVal = 0.f;
            else if (term == kTruncated) nextVal = (trunc_vals && tidx >= 0) ? trunc_vals[tidx] : 0.f;
            else nextVal = vals[i + 1];  // a segment's non-final rows are never its last row
            const float v = vals[i];
            const float predReturn = cur + gamma * nextVal;
            const float delta = predReturn - v;
            const float curReturn = rew + prevRet * gamma * nd;
            ret[i] = curReturn;
            prevLambda = delta + gamma_lambda * nd * prevLambda;
            adv[i] = prevLambda;
            target[i] = v + prevLambda;
            prevRet = curReturn;
        }
    }
    if (clip_sums && normalize) {
        for (int o = 32; o > 0; o >>= 1) {
            sabs += __shfl_down(sabs, o, 64);
            sclip += __shfl_down(sclip, o, 64);
        }
        if ((threadIdx.x & 63) == 0) {
            atomicAdd(&clip_sums[0], sabs);
            atomicAdd(&clip_sums[1], sclip);
        }
    }
}

}  // namespace

extern "C" int rlgpu_gae_segments(const float* d_rews, const int8_t* d_terms, const float* d_vals, const float* d_trunc_vals,
                                  const int64_t* d_seg_off, const int32_t* d_seg_len, const int32_t* d_seg_tidx,
                                  int64_t num_segments, float gamma, float lambda, float return_std, float clip_range,
                                  float* d_adv, float* d_target, float* d_ret, float* d_clip_partials, void* stream) {
    return rlgpu::guarded([&] {
        RLGPU_REQUIRE(num_segments >= 0, "rlgpu_gae_segments: negative segment count");
        if (num_segments == 0) return;
        RLGPU_REQUIRE(d_rews && d_terms && d_vals && d_seg_off && d_seg_len && d_seg_tidx && d_adv && d_target && d_ret,
                      "rlgpu_gae_segments: null argument");
        hipStream_t s = rlgpu::as_stream(stream);
        const bool normalize = (return_std != 0.f && return_std != 1.f);  // GAE.cpp:47-49
        const float inv_std = normalize ? 1.f / return_std : 1.f;
        hipLaunchKernelGGL(k_gae_segments, dim3(rlgpu::ceil_div(num_segments, 256)), dim3(256), 0, s, d_rews, d_terms, d_vals,
                           d_trunc_vals, d_seg_off, d_seg_len, d_seg_tidx, num_segments, gamma, gamma * lambda, inv_std,
                           (int)normalize, (int)(clip_range > 0.f), clip_range, d_adv, d_target, d_ret, d_clip_partials);
        RLGPU_CHECK_HIP(hipGetLastError());
    });
}

extern "C" int rlgpu_gae_flat(const float* d_rews, const int8_t* d_terms, const float* d_vals,
                              const float* d_trunc_vals, int64_t num_returns, int64_t num_truncs, float gamma,
                              float lambda, float return_std, float clip_range, float* d_adv, float* d_target,
                              float* d_ret, float* h_clip_portion, void* stream) {
    return rlgpu::guarded([&] {
        RLGPU_REQUIRE(num_returns >= 0 && num_truncs >= 0, "rlgpu_gae_flat: negative size");
        if (num_returns == 0) {  // GAE.cpp:16-23
            if (h_clip_portion) *h_clip_portion = 0.f;
            return;
        }
        RLGPU_REQUIRE(d_rews && d_terms && d_vals && d_adv && d_target && d_ret, "rlgpu_gae_flat: null pointer");
        RLGPU_REQUIRE(num_truncs == 0 || d_trunc_vals, "rlgpu_gae_flat: trunc values missing");
        hipStream_t s = rlgpu::as_stream(stream);
        int nchunks = (int)rlgpu::ceil_div(num_returns, kChunk);
        // scratch: counts(int) | offsets(i64) | total(i64) | summaries(f4) | carry(f2) | clip sums(f2)
        size_t bytes = 0;
        auto take = [&](size_t n, size_t align) {
            bytes = (bytes + align - 1) / align * align;
            size_t off = bytes;
            bytes += n;
            return off;
        };
        size_t o_counts = take(sizeof(int) * nchunks, 16), o_offs = take(sizeof(int64_t) * nchunks, 16),
               o_total = take(sizeof(int64_t), 16), o_sum = take(sizeof(float4) * nchunks, 16),
               o_carry = take(sizeof(float2) * nchunks, 16), o_clip = take(sizeof(float) * 2, 16);
        char* scratch = nullptr;
        RLGPU_CHECK_HIP(hipMallocAsync((void**)&scratch, bytes, s));
        int* counts = (int*)(scratch + o_counts);
        int64_t* offs = (int64_t*)(scratch + o_offs);
        int64_t* total = (int64_t*)(scratch + o_total);
        float4* sums = (float4*)(scratch + o_sum);
        float2* carry = (float2*)(scratch + o_carry);
        float* clip = (float*)(scratch + o_clip);
        RLGPU_CHECK_HIP(hipMemsetAsync(clip, 0, sizeof(float) * 2, s));

        GaeParams p;
        p.rews = d_rews;
        p.terms = d_terms;
        p.vals = d_vals;
        p.trunc_vals = d_trunc_vals;
        p.M = num_returns;
        p.num_truncs = num_truncs;
        p.normalize = (return_std != 0.f && return_std != 1.f);  // GAE.cpp:73
        p.clip = clip_range > 0.f;                                  // GAE.cpp:74
        p.inv_std = p.normalize ? (1.0f / return_std) : 1.0f;
        p.gamma = gamma;
        p.gamma_lambda = gamma * lambda;
        p.clip_range = clip_range;

        hipLaunchKernelGGL(k_trunc_count, dim3(nchunks), dim3(kThreads), 0, s, d_terms, num_returns, counts);
        hipLaunchKernelGGL(k_scan_counts, dim3(1), dim3(kThreads), 0, s, counts, nchunks, offs, total);
        hipLaunchKernelGGL(k_chunk_summary, dim3(nchunks), dim3(kThreads), 0, s, p, offs, sums);
        hipLaunchKernelGGL(k_chunk_carry, dim3(1), dim3(kThreads), 0, s, sums, nchunks, carry);
        hipLaunchKernelGGL(k_apply, dim3(nchunks), dim3(kThreads), 0, s, p, offs, carry, d_adv, d_target, d_ret, clip);
        RLGPU_CHECK_HIP(hipGetLastError());
        int64_t h_total = 0;
        float h_clip[2] = {0.f, 0.f};
        RLGPU_CHECK_HIP(hipMemcpyAsync(&h_total, total, sizeof(int64_t), hipMemcpyDeviceToHost, s));
        RLGPU_CHECK_HIP(hipMemcpyAsync(h_clip, clip, sizeof(h_clip), hipMemcpyDeviceToHost, s));
        RLGPU_CHECK_HIP(hipFreeAsync(scratch, s));
        RLGPU_CHECK_HIP(hipStreamSynchronize(s));
        // GAE.cpp:196-197: truncation count must match the provided bootstrap values.
        if (num_truncs > 0 && h_total != num_truncs)
            throw rlgpu::Error(RLGPU_ERR_INVALID_ARG, "GAE: truncation count mismatch (" + std::to_string(h_total) +
                                                          "/" + std::to_string(num_truncs) + ")");
        if (h_clip_portion)
            *h_clip_portion = p.normalize ? (h_clip[0] - h_clip[1]) / fmaxf(h_clip[0], 1e-7f) : 0.f;
    });
}

extern "C" int rlgpu_gae_rollout(const float* d_rews, const int8_t* d_terms, const float* d_vals,
                                 const float* d_trunc_vals, const float* d_boot_vals, int32_t T, int32_t N,
                                 float gamma, float lambda, float return_std, float clip_range, float* d_adv,
                                 float* d_target, float* d_ret, float* d_clip_partials, void* stream) {
    return rlgpu::guarded([&] {
        RLGPU_REQUIRE(T >= 0 && N >= 0, "rlgpu_gae_rollout: negative size");
        if (T == 0 || N == 0) return;
        RLGPU_REQUIRE(d_rews && d_terms && d_vals && d_adv && d_target && d_ret, "rlgpu_gae_rollout: null pointer");
        hipStream_t s = rlgpu::as_stream(stream);
        bool normalize = (return_std != 0.f && return_std != 1.f);
        float inv_std = normalize ? (1.0f / return_std) : 1.0f;
        hipLaunchKernelGGL(k_gae_rollout, dim3(rlgpu::ceil_div(N, 256)), dim3(256), 0, s, d_rews, d_terms, d_vals,
                           d_trunc_vals, d_boot_vals, T, N, gamma, gamma * lambda, inv_std, (int)normalize,
                           (int)(clip_range > 0.f), clip_range, d_adv, d_target, d_ret, d_clip_partials);
        RLGPU_CHECK_HIP(hipGetLastError());
    });
}

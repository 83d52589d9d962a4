// learner_kernels.hip -- small device helpers of the C++ host Learner (host/learner.cpp):
// truncated-row compaction, index gathers / scatters, self-play row lists, fp64 moments.
#include <hipcub/hipcub.hpp>

#include "common.hpp"
#include "learner_kernels.hpp"

namespace lk {
namespace {

using rlgpu::ceil_div;

__global__ void k_gather_f32(const float* src, const int32_t* idx, int64_t n, float* dst) {
    int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) dst[i] = src[idx[i]];
}

__global__ void k_scatter_f32(const float* src, const int32_t* idx, int64_t n, float* dst) {
    int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) dst[idx[i]] = src[i];
}

__global__ void k_gather_rows(const float* src, int C, const int32_t* idx, int64_t n, float* dst) {
    int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (e >= n * C) return;
    int64_t r = e / C;
    int c = (int)(e % C);
    dst[e] = src[(int64_t)idx[r] * C + c];
}

__global__ void k_compose(const int32_t* rows, const int32_t* perm, int64_t n, int32_t* out) {
    int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) out[i] = rows[perm[i]];
}

__global__ void k_train_rows(int T, int P, int team, int32_t* out) {
    const int half = P / 2;
    int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= (int64_t)T * half) return;
    int t = (int)(i / half), q = (int)(i % half);
    out[i] = t * P + 2 * q + team;  // team of player p is p % 2 (cars 0, 2 blue; 1, 3 orange)
}

// one lane per player column: the last step t whose trajectory code is nonzero, -1 if none
__global__ void k_last_ends(const int8_t* terms, int T, int P, int32_t* out) {
    int p = blockIdx.x * blockDim.x + threadIdx.x;
    if (p >= P) return;
    int last = -1;
    for (int t = T - 1; t >= 0; --t)
        if (terms[(int64_t)t * P + p] != 0) {
            last = t;
            break;
        }
    out[p] = last;
}

__global__ void k_gather_samples(const float* src, const int64_t* idx, int n, float* dst) {
    int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) dst[i] = src[idx[i]];
}

// fp64 (sum, sum of squares) partials over a grid-stride range, then a fixed-order final sum:
// deterministic run to run
constexpr int kMomBlocks = 256;
__global__ void __launch_bounds__(256) k_moments_partial(const float* x, const int32_t* idx, int64_t n, double* part) {
    __shared__ double s1[256], s2[256];
    double a = 0, b = 0;
    for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256) {
        double v = idx ? x[idx[i]] : x[i];
        a += v;
        b += v * v;
    }
    s1[threadIdx.x] = a;
    s2[threadIdx.x] = b;
    __syncthreads();
    for (int o = 128; o > 0; o >>= 1) {
        if (threadIdx.x < o) {
            s1[threadIdx.x] += s1[threadIdx.x + o];
            s2[threadIdx.x] += s2[threadIdx.x + o];
        }
        __syncthreads();
    }
    if (threadIdx.x == 0) {
        part[2 * blockIdx.x] = s1[0];
        part[2 * blockIdx.x + 1] = s2[0];
    }
}
__global__ void k_moments_final(const double* part, int nb, int64_t n, double* out) {
    if (threadIdx.x != 0) return;
    double a = 0, b = 0;
    for (int k = 0; k < nb; k++) {
        a += part[2 * k];
        b += part[2 * k + 1];
    }
    out[0] = a;
    out[1] = b;
    out[2] = (double)n;
}

__global__ void k_stack_frames(const float* cur, const float* trunc, const int8_t* codes, float* hist, int K, int P,
                               int obs, float* out, float* out_trunc) {
    int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (e >= (int64_t)P * obs) return;
    const int p = (int)(e / obs), c = (int)(e % obs);
    const float x = cur[e];
    const int code = codes ? codes[p] : 1;
    const int64_t W = (int64_t)K * obs, plane = (int64_t)P * obs;
    float* o = out + p * W + c;
    if (code == 2 && out_trunc && trunc) {  // the ended trajectory's last stacked row
        float* ot = out_trunc + p * W + c;
        ot[0] = trunc[e];
        for (int k = 1; k < K; k++) ot[(int64_t)k * obs] = hist[(int64_t)(k - 1) * plane + e];
    }
    if (code != 0) {
        for (int k = 0; k < K; k++) o[(int64_t)k * obs] = x;
        for (int k = 0; k < K - 1; k++) hist[(int64_t)k * plane + e] = x;
        return;
    }
    float prev = x;
    o[0] = x;
    for (int k = 0; k < K - 1; k++) {  // read the old frame before overwriting it with the newer one
        const float h = hist[(int64_t)k * plane + e];
        o[(int64_t)(k + 1) * obs] = h;
        hist[(int64_t)k * plane + e] = prev;
        prev = h;
    }
}

// After a step hook (host plugins, Learner.cpp:780-861): one thread per (player, obs column).  The
// player's code becomes the arena's merged terminal (the hook's NORMAL-over-TRUNCATED merge of device and
// host conditions) or, where that is 0, the device's own code (the max-episode-length truncation); column 0
// also takes the step's (host-rebuilt) reward.  A code-2 row's pre-reset obs goes to the truncation rows.
__global__ void k_host_step_finish(const uint8_t* arena_terms, int8_t* codes, const float* rewards, float* rew_out,
                                   const float* obs, float* trunc_env, float* trunc_out, int P, int obs_w) {
    int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (e >= (int64_t)P * obs_w) return;
    const int p = (int)(e / obs_w), c = (int)(e % obs_w);
    const int m = arena_terms[p / 4];
    const int code = m ? m : codes[p];
    if (code == 2) {
        trunc_env[e] = obs[e];
        if (trunc_out) trunc_out[e] = obs[e];
    }
    if (c == 0) {  // idempotent: a thread of the row that reads codes[p] after this write computes the same code
        codes[p] = (int8_t)code;
        if (rew_out) rew_out[p] = rewards[p];
    }
}

// one workgroup walks the players in chunks of 1024: block-wide exclusive scans of the end /
// truncation flags give each ending trajectory its record slot, truncation slot and combined offset in
// (player) order after the records of earlier steps
constexpr int kTrajThreads = 1024;
__global__ void __launch_bounds__(kTrajThreads) k_traj_step(const int8_t* codes, int row, int Tmax, const uint8_t* track,
                                                            int P, int32_t* start, int32_t* len, TrajRecs R,
                                                            int64_t* cnt, int32_t* trnew) {
    typedef hipcub::BlockScan<int, kTrajThreads> Scan;
    typedef hipcub::BlockScan<int64_t, kTrajThreads> Scan64;
    __shared__ typename Scan::TempStorage ts;
    __shared__ typename Scan64::TempStorage ts64;
    __shared__ int64_t base[3];
    __shared__ int newtr;
    const int t = threadIdx.x;
    if (t == 0) {
        base[0] = cnt[kTcRecs];
        base[1] = cnt[kTcTruncs];
        base[2] = cnt[kTcSteps];
        newtr = 0;
    }
    __syncthreads();
    const int next = (row + 1) % Tmax;
    for (int c0 = 0; c0 < P; c0 += kTrajThreads) {
        const int p = c0 + t;
        const bool on = p < P && (!track || track[p]);
        const int code = on ? codes[p] : 0;
        const int l = on ? len[p] + 1 : 0;
        const int e = code != 0, tr = code == 2;
        int eo, to, etot, ttot;
        int64_t lo, ltot;
        Scan(ts).ExclusiveSum(e, eo, etot);
        __syncthreads();
        Scan(ts).ExclusiveSum(tr, to, ttot);
        __syncthreads();
        Scan64(ts64).ExclusiveSum(e ? (int64_t)l : (int64_t)0, lo, ltot);
        __syncthreads();
        if (e) {
            const int64_t k = base[0] + eo;
            R.p[k] = p;
            R.start[k] = start[p];
            R.len[k] = l;
            R.code[k] = code;
            R.tidx[k] = tr ? (int32_t)(base[1] + to) : -1;
            R.off[k] = base[2] + lo;
            if (tr) trnew[newtr + to] = p;
            start[p] = next;
            len[p] = 0;
        } else if (on) {
            len[p] = l;
        }
        __syncthreads();
        if (t == 0) {
            base[0] += etot;
            base[1] += ttot;
            base[2] += ltot;
            newtr += ttot;
        }
        __syncthreads();
    }
    if (t == 0) {
        cnt[kTcRecs] = base[0];
        cnt[kTcTruncs] = base[1];
        cnt[kTcSteps] = base[2];
        cnt[kTcNewTruncs] = newtr;
    }
}

__global__ void k_traj_trunc_copy(const float* src, int W, const int64_t* cnt, const int32_t* trnew, float* dst) {
    const int64_t nnew = cnt[kTcNewTruncs], first = cnt[kTcTruncs] - nnew;
    for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < nnew * W; e += (int64_t)gridDim.x * blockDim.x) {
        const int64_t j = e / W;
        const int c = (int)(e - j * W);
        dst[(first + j) * W + c] = src[(int64_t)trnew[j] * W + c];
    }
}

__global__ void k_traj_restart(const uint8_t* mask, int P, int row, int32_t* start, int32_t* len) {
    int p = blockIdx.x * blockDim.x + threadIdx.x;
    if (p < P && mask[p]) {
        start[p] = row;
        len[p] = 0;
    }
}

// one workgroup per record: its steps' rows, 16-byte vectors where the obs rows allow
__global__ void __launch_bounds__(256) k_traj_gather(TrajRecs R, int Tmax, int P, int W, int A, const float* obs,
                                                     const uint8_t* masks, const int32_t* acts, const float* logp,
                                                     const float* rews, const int8_t* terms, float* c_obs,
                                                     uint8_t* c_masks, int32_t* c_acts, float* c_logp, float* c_rews,
                                                     int8_t* c_terms) {
    const int64_t k = blockIdx.x;
    const int p = R.p[k], st = R.start[k], L = R.len[k];
    const int64_t off = R.off[k];
    for (int j = threadIdx.x; j < L; j += blockDim.x) {
        const int64_t src = (int64_t)((st + j) % Tmax) * P + p, dst = off + j;
        c_acts[dst] = acts[src];
        c_logp[dst] = logp[src];
        c_rews[dst] = rews[src];
        c_terms[dst] = terms[src];
    }
    for (int j = 0; j < L; j++) {
        const int64_t src = (int64_t)((st + j) % Tmax) * P + p, dst = off + j;
        const float* so = obs + src * W;
        float* d = c_obs + dst * W;
        for (int c = threadIdx.x; c < W; c += blockDim.x) d[c] = so[c];
        const uint8_t* sm = masks + src * A;
        uint8_t* dm = c_masks + dst * A;
        for (int c = threadIdx.x; c < A; c += blockDim.x) dm[c] = sm[c];
    }
}

struct IsTrunc {
    const int8_t* t;
    __device__ bool operator()(const int32_t& i) const { return t[i] == 2; }
};

}  // namespace

void gather_f32(const float* src, const int32_t* idx, int64_t n, float* dst, hipStream_t s) {
    if (n <= 0) return;
    hipLaunchKernelGGL(k_gather_f32, dim3(ceil_div(n, 256)), dim3(256), 0, s, src, idx, n, dst);
    RLGPU_CHECK_HIP(hipGetLastError());
}
void scatter_f32(const float* src, const int32_t* idx, int64_t n, float* dst, hipStream_t s) {
    if (n <= 0) return;
    hipLaunchKernelGGL(k_scatter_f32, dim3(ceil_div(n, 256)), dim3(256), 0, s, src, idx, n, dst);
    RLGPU_CHECK_HIP(hipGetLastError());
}
void gather_rows(const float* src, int C, const int32_t* idx, int64_t n, float* dst, hipStream_t s) {
    if (n <= 0) return;
    hipLaunchKernelGGL(k_gather_rows, dim3(ceil_div(n * C, 256)), dim3(256), 0, s, src, C, idx, n, dst);
    RLGPU_CHECK_HIP(hipGetLastError());
}
void compose(const int32_t* rows, const int32_t* perm, int64_t n, int32_t* out, hipStream_t s) {
    if (n <= 0) return;
    hipLaunchKernelGGL(k_compose, dim3(ceil_div(n, 256)), dim3(256), 0, s, rows, perm, n, out);
    RLGPU_CHECK_HIP(hipGetLastError());
}
void train_rows(int T, int P, int team, int32_t* out, hipStream_t s) {
    int64_t n = (int64_t)T * (P / 2);
    hipLaunchKernelGGL(k_train_rows, dim3(ceil_div(n, 256)), dim3(256), 0, s, T, P, team, out);
    RLGPU_CHECK_HIP(hipGetLastError());
}
void last_ends(const int8_t* terms, int T, int P, int32_t* out, hipStream_t s) {
    if (P <= 0) return;
    hipLaunchKernelGGL(k_last_ends, dim3(ceil_div(P, 256)), dim3(256), 0, s, terms, T, P, out);
    RLGPU_CHECK_HIP(hipGetLastError());
}
void gather_samples(const float* src, const int64_t* idx, int n, float* dst, hipStream_t s) {
    if (n <= 0) return;
    hipLaunchKernelGGL(k_gather_samples, dim3(ceil_div(n, 256)), dim3(256), 0, s, src, idx, n, dst);
    RLGPU_CHECK_HIP(hipGetLastError());
}
size_t moments_scratch_bytes() { return 2 * kMomBlocks * sizeof(double); }
void moments_f64(const float* x, const int32_t* idx, int64_t n, double* scratch, double* out3, hipStream_t s) {
    hipLaunchKernelGGL(k_moments_partial, dim3(kMomBlocks), dim3(256), 0, s, x, idx, n, scratch);
    hipLaunchKernelGGL(k_moments_final, dim3(1), dim3(64), 0, s, scratch, kMomBlocks, n, out3);
    RLGPU_CHECK_HIP(hipGetLastError());
}

void stack_frames(const float* cur, const float* trunc, const int8_t* codes, float* hist, int K, int P, int obs,
                  float* out, float* out_trunc, hipStream_t s) {
    const int64_t n = (int64_t)P * obs;
    hipLaunchKernelGGL(k_stack_frames, dim3(ceil_div(n, 256)), dim3(256), 0, s, cur, trunc, codes, hist, K, P, obs, out,
                       out_trunc);
    RLGPU_CHECK_HIP(hipGetLastError());
}

void host_step_finish(const uint8_t* arena_terms, int8_t* codes, const float* rewards, float* rew_out, const float* obs,
                      float* trunc_env, float* trunc_out, int P, int obs_w, hipStream_t s) {
    const int64_t n = (int64_t)P * obs_w;
    hipLaunchKernelGGL(k_host_step_finish, dim3(ceil_div(n, 256)), dim3(256), 0, s, arena_terms, codes, rewards, rew_out,
                       obs, trunc_env, trunc_out, P, obs_w);
    RLGPU_CHECK_HIP(hipGetLastError());
}

void traj_step(const int8_t* codes, int row, int Tmax, const uint8_t* track, int P, int32_t* start, int32_t* len,
               TrajRecs recs, int64_t* counters, int32_t* trnew, hipStream_t s) {
    hipLaunchKernelGGL(k_traj_step, dim3(1), dim3(kTrajThreads), 0, s, codes, row, Tmax, track, P, start, len, recs, counters,
                       trnew);
    RLGPU_CHECK_HIP(hipGetLastError());
}
void traj_trunc_copy(const float* src, int W, const int64_t* counters, const int32_t* trnew, float* dst, hipStream_t s) {
    hipLaunchKernelGGL(k_traj_trunc_copy, dim3(256), dim3(256), 0, s, src, W, counters, trnew, dst);
    RLGPU_CHECK_HIP(hipGetLastError());
}
void traj_restart(const uint8_t* mask, int P, int row, int32_t* start, int32_t* len, hipStream_t s) {
    hipLaunchKernelGGL(k_traj_restart, dim3(ceil_div(P, 256)), dim3(256), 0, s, mask, P, row, start, len);
    RLGPU_CHECK_HIP(hipGetLastError());
}
void traj_gather(TrajRecs recs, int64_t K, int Tmax, int P, int W, int A, const float* obs, const uint8_t* masks,
                 const int32_t* acts, const float* logp, const float* rews, const int8_t* terms, float* c_obs,
                 uint8_t* c_masks, int32_t* c_acts, float* c_logp, float* c_rews, int8_t* c_terms, hipStream_t s) {
    if (K <= 0) return;
    hipLaunchKernelGGL(k_traj_gather, dim3((unsigned)K), dim3(256), 0, s, recs, Tmax, P, W, A, obs, masks, acts, logp, rews,
                       terms, c_obs, c_masks, c_acts, c_logp, c_rews, c_terms);
    RLGPU_CHECK_HIP(hipGetLastError());
}

size_t select_trunc_scratch_bytes(int64_t n) {
    size_t bytes = 0;
    hipcub::CountingInputIterator<int32_t> it(0);
    RLGPU_CHECK_HIP(hipcub::DeviceSelect::If(nullptr, bytes, it, (int32_t*)nullptr, (int32_t*)nullptr, (int)n,
                                             IsTrunc{nullptr}, (hipStream_t)0));
    return bytes;
}
void select_trunc(const int8_t* terms, int64_t n, void* scratch, size_t scratch_bytes, int32_t* rows, int32_t* count,
                  hipStream_t s) {
    hipcub::CountingInputIterator<int32_t> it(0);
    RLGPU_CHECK_HIP(hipcub::DeviceSelect::If(scratch, scratch_bytes, it, rows, count, (int)n, IsTrunc{terms}, s));
}

}  // namespace lk

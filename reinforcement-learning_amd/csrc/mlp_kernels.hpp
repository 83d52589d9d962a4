// mlp_kernels.hpp -- MFMA GEMMs and row kernels of the PPO actor/critic (gfx950).
//
// GEMM convention: C[I,J] (+= over K) = sum_k A(i,k) * B(k,j), one 128x128 output tile per
// 256-thread workgroup (4 waves in 2x2, 64x64 per wave), K staged through LDS in steps of BK.
//   A layouts: A_IK  stored [I][lda], k contiguous (activations; optional row gather idx[i])
//              A_KI  stored [K][lda], i contiguous (dZ^T for weight gradients)
//   B layouts: B_JK  stored [J][ldb], k contiguous (Linear.weight [out,in] in the forward)
//              B_KJ  stored [K][ldb], j contiguous (weight in dX = dZ.W; activations in dW,
//                    optional row gather idx[k])
// fp32 path: v_mfma_f32_32x32x2_f32 (exact f32 products, f32 accumulate) -- training.
// bf16 path: v_mfma_f32_32x32x16_bf16 (fp32 accumulate, bf16 output) -- inference.
// Split-K (grid.z) writes per-split partial tiles; reduce_splits() sums them in a fixed
// order, so every result is deterministic run to run.
#pragma once
#include <hip/hip_bf16.h>
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace mlp {

#define DEV __device__ __forceinline__

typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef short bf16x8 __attribute__((ext_vector_type(8)));

enum { A_IK = 0, A_KI = 1 };
enum { B_JK = 0, B_KJ = 1 };

constexpr int BM = 128, BN = 128, BK = 32;
constexpr int KP = 4;  // pad of k-contiguous LDS rows ([m][BK + KP]: 144 B = 9 x 16 B, odd)
constexpr int MP = 4;  // pad of m-contiguous LDS rows ([k][BM + MP])

struct GemmArgs {
    const float* A;
    const float* B;
    float* C;
    const float* bias;     // [J] or null
    const int32_t* a_idx;  // row gather for A_IK (indexed by i + a_off)
    const int32_t* b_idx;  // row gather for B_KJ (indexed by k + b_off)
    int64_t a_off, b_off;
    int64_t lda, ldb, ldc;
    int I, J, K;
    int kchunk;            // K range per split (multiple of BK)
    int64_t c_split;       // element stride between split partials
    int a_vec, b_vec;      // 16-byte aligned rows (ld % 4 == 0, base aligned): float4 loads
};

DEV uint16_t f2bf(float f) {  // round-to-nearest-even (plain cast: NaN stays NaN)
    __hip_bfloat16 b = __float2bfloat16(f);
    return *reinterpret_cast<uint16_t*>(&b);
}
DEV float bf2f(uint16_t u) { return __uint_as_float((uint32_t)u << 16); }

// 4 consecutive elements p[c..c+3] of a row, zero outside [.., lim)
DEV float4 load4(const float* p, int c, int lim, bool vec) {
    if (!p) return make_float4(0.f, 0.f, 0.f, 0.f);
    if (vec && c + 3 < lim) return *reinterpret_cast<const float4*>(p + c);
    float4 v;
    v.x = c < lim ? p[c] : 0.f;
    v.y = c + 1 < lim ? p[c + 1] : 0.f;
    v.z = c + 2 < lim ? p[c + 2] : 0.f;
    v.w = c + 3 < lim ? p[c + 3] : 0.f;
    return v;
}

// One 128 x 32 tile of an operand, 4 float4 per thread.
//  KMAJ (global row = output index, k contiguous) -> LDS [row][BK + KP]
//  !KMAJ (global row = k, output index contiguous) -> LDS [k][BM + MP]
template <bool KMAJ>
DEV void tile_load(float4 (&r)[4], const float* base, int64_t ld, const int32_t* idx, int64_t off, int o0, int on, int k0,
                   int ke, bool vec) {
    const int t = threadIdx.x;
#pragma unroll
    for (int q = 0; q < 4; q++) {
        int e = t + 256 * q;
        if (KMAJ) {
            int row = e >> 3, c = (e & 7) * 4;
            int go = o0 + row;
            const float* p = nullptr;
            if (go < on) p = base + (idx ? (int64_t)idx[off + go] : (int64_t)go) * ld;
            r[q] = load4(p, k0 + c, ke, vec);
        } else {
            int kr = e >> 5, c = (e & 31) * 4;
            int k = k0 + kr;
            const float* p = nullptr;
            if (k < ke) p = base + (idx ? (int64_t)idx[off + k] : (int64_t)k) * ld;
            r[q] = load4(p, o0 + c, on, vec);
        }
    }
}

template <bool KMAJ>
DEV void tile_store(float* lds, const float4 (&r)[4]) {
    const int t = threadIdx.x;
#pragma unroll
    for (int q = 0; q < 4; q++) {
        int e = t + 256 * q;
        if (KMAJ) {
            int row = e >> 3, c = (e & 7) * 4;
            *reinterpret_cast<float4*>(lds + row * (BK + KP) + c) = r[q];
        } else {
            int kr = e >> 5, c = (e & 31) * 4;
            *reinterpret_cast<float4*>(lds + kr * (BM + MP) + c) = r[q];
        }
    }
}

// element (output index o, k) of an LDS tile
template <bool KMAJ>
DEV float tile_at(const float* lds, int o, int k) {
    return KMAJ ? lds[o * (BK + KP) + k] : lds[k * (BM + MP) + o];
}

// fp32 GEMM on v_mfma_f32_32x32x2_f32: each MFMA j of a BK step takes k = j (lanes 0-31) and
// k = 16 + j (lanes 32-63) so that k-contiguous tiles are read as 16-byte vectors.
template <int LA, int LB>
__global__ void __launch_bounds__(256, 2) gemm_f32(GemmArgs g) {
    constexpr bool AK = LA == A_IK, BKM = LB == B_JK;
    constexpr int ASZ = AK ? BM * (BK + KP) : BK * (BM + MP);
    constexpr int BSZ = BKM ? BN * (BK + KP) : BK * (BN + MP);
    __shared__ float As[ASZ];
    __shared__ float Bs[BSZ];
    const int t = threadIdx.x, lane = t & 63, w = t >> 6;
    const int wm = w >> 1, wn = w & 1;
    const int i0 = blockIdx.y * BM, j0 = blockIdx.x * BN;
    const int kb = blockIdx.z * g.kchunk;
    const int ke = min(g.K, kb + g.kchunk);
    const int h = lane >> 5, l32 = lane & 31;
    f32x16 acc[2][2];
    for (int a = 0; a < 2; a++)
        for (int b = 0; b < 2; b++)
            for (int r = 0; r < 16; r++) acc[a][b][r] = 0.f;
    float4 ra[4], rb[4];
    if (kb < ke) {
        tile_load<AK>(ra, g.A, g.lda, g.a_idx, g.a_off, i0, g.I, kb, ke, g.a_vec);
        tile_load<BKM>(rb, g.B, g.ldb, g.b_idx, g.b_off, j0, g.J, kb, ke, g.b_vec);
    }
    for (int k0 = kb; k0 < ke; k0 += BK) {
        tile_store<AK>(As, ra);
        tile_store<BKM>(Bs, rb);
        __syncthreads();
        if (k0 + BK < ke) {  // prefetch the next stage into registers while the MFMAs run
            tile_load<AK>(ra, g.A, g.lda, g.a_idx, g.a_off, i0, g.I, k0 + BK, ke, g.a_vec);
            tile_load<BKM>(rb, g.B, g.ldb, g.b_idx, g.b_off, j0, g.J, k0 + BK, ke, g.b_vec);
        }
        const int ma = wm * 64 + l32, nb = wn * 64 + l32;
#pragma unroll
        for (int j = 0; j < BK / 2; j++) {
            int kk = 16 * h + j;
            float a0 = tile_at<AK>(As, ma, kk), a1 = tile_at<AK>(As, ma + 32, kk);
            float b0 = tile_at<BKM>(Bs, nb, kk), b1 = tile_at<BKM>(Bs, nb + 32, kk);
            acc[0][0] = __builtin_amdgcn_mfma_f32_32x32x2f32(a0, b0, acc[0][0], 0, 0, 0);
            acc[0][1] = __builtin_amdgcn_mfma_f32_32x32x2f32(a0, b1, acc[0][1], 0, 0, 0);
            acc[1][0] = __builtin_amdgcn_mfma_f32_32x32x2f32(a1, b0, acc[1][0], 0, 0, 0);
            acc[1][1] = __builtin_amdgcn_mfma_f32_32x32x2f32(a1, b1, acc[1][1], 0, 0, 0);
        }
        __syncthreads();
    }
    float* C = g.C + (int64_t)blockIdx.z * g.c_split;
#pragma unroll
    for (int ti = 0; ti < 2; ti++)
#pragma unroll
        for (int tj = 0; tj < 2; tj++) {
            int j = j0 + wn * 64 + tj * 32 + l32;
            if (j >= g.J) continue;
            float bj = g.bias ? g.bias[j] : 0.f;
#pragma unroll
            for (int r = 0; r < 16; r++) {
                int i = i0 + wm * 64 + ti * 32 + (r & 3) + 8 * (r >> 2) + 4 * h;
                if (i < g.I) C[(int64_t)i * g.ldc + j] = acc[ti][tj][r] + bj;
            }
        }
}

// ---- bf16 inference GEMM: C[i,j] = bf16( sum_k A[i,k] W[j,k] + bias[j] ), A fp32 or bf16.
constexpr int HBK = 32, HPAD = 8;

struct HGemmArgs {
    const void* A;          // float* (a_f32) or uint16_t* (bf16)
    const uint16_t* B;      // [J][ldb] bf16
    const uint16_t* bias;   // [J] bf16 or null
    uint16_t* C;            // [I][ldc] bf16
    int64_t lda, ldb, ldc;
    int I, J, K;
};

template <bool A_F32>
__global__ void __launch_bounds__(256) gemm_bf16(HGemmArgs g) {
    __shared__ uint16_t As[BM][HBK + HPAD];
    __shared__ uint16_t Bs[BN][HBK + HPAD];
    const int t = threadIdx.x, lane = t & 63, w = t >> 6;
    const int wm = w >> 1, wn = w & 1;
    const int i0 = blockIdx.y * BM, j0 = blockIdx.x * BN;
    f32x16 acc[2][2];
    for (int a = 0; a < 2; a++)
        for (int b = 0; b < 2; b++)
            for (int r = 0; r < 16; r++) acc[a][b][r] = 0.f;
    for (int k0 = 0; k0 < g.K; k0 += HBK) {
        {
            int r = t >> 1, kh = (t & 1) * 16;
            int gi = i0 + r;
#pragma unroll
            for (int kk = 0; kk < 16; kk++) {
                int k = k0 + kh + kk;
                uint16_t v = 0;
                if (gi < g.I && k < g.K) {
                    if (A_F32)
                        v = f2bf(((const float*)g.A)[(int64_t)gi * g.lda + k]);
                    else
                        v = ((const uint16_t*)g.A)[(int64_t)gi * g.lda + k];
                }
                As[r][kh + kk] = v;
            }
            int gj = j0 + r;
#pragma unroll
            for (int kk = 0; kk < 16; kk++) {
                int k = k0 + kh + kk;
                Bs[r][kh + kk] = (gj < g.J && k < g.K) ? g.B[(int64_t)gj * g.ldb + k] : (uint16_t)0;
            }
        }
        __syncthreads();
#pragma unroll
        for (int ks = 0; ks < HBK / 16; ks++) {
            int kof = ks * 16 + 8 * (lane >> 5);
            bf16x8 a0 = *(const bf16x8*)&As[wm * 64 + (lane & 31)][kof];
            bf16x8 a1 = *(const bf16x8*)&As[wm * 64 + 32 + (lane & 31)][kof];
            bf16x8 b0 = *(const bf16x8*)&Bs[wn * 64 + (lane & 31)][kof];
            bf16x8 b1 = *(const bf16x8*)&Bs[wn * 64 + 32 + (lane & 31)][kof];
            acc[0][0] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a0, b0, acc[0][0], 0, 0, 0);
            acc[0][1] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a0, b1, acc[0][1], 0, 0, 0);
            acc[1][0] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a1, b0, acc[1][0], 0, 0, 0);
            acc[1][1] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a1, b1, acc[1][1], 0, 0, 0);
        }
        __syncthreads();
    }
#pragma unroll
    for (int ti = 0; ti < 2; ti++)
#pragma unroll
        for (int tj = 0; tj < 2; tj++) {
            int j = j0 + wn * 64 + tj * 32 + (lane & 31);
            if (j >= g.J) continue;
            float bj = g.bias ? bf2f(g.bias[j]) : 0.f;
#pragma unroll
            for (int r = 0; r < 16; r++) {
                int i = i0 + wm * 64 + ti * 32 + (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5);
                if (i < g.I) g.C[(int64_t)i * g.ldc + j] = f2bf(acc[ti][tj][r] + bj);
            }
        }
}

// out[e] (+)= sum_s part[s*stride + e], fixed order (deterministic split-K reduction)
__global__ void reduce_splits(const float* part, int splits, int64_t stride, int64_t n, float* out, int accumulate) {
    int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (e >= n) return;
    float s = 0.f;
    for (int k = 0; k < splits; k++) s += part[k * stride + e];
    out[e] = accumulate ? out[e] + s : s;
}

// ---------------------------------------------------------------- wave helpers
DEV float wave_sum(float v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
    return v;
}
DEV float wave_max(float v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
    return v;
}


// LayerNorm (eps 1e-5, biased variance) + LeakyReLU, training: one wave per row.
// Keeps xhat [R,H] and act [R,H] for the backward, rstd [R].
template <int MAXH>
__global__ void __launch_bounds__(256) ln_act_fwd_f32(const float* Z, const float* gamma, const float* beta, int R, int H,
                                                     float slope, int use_ln, float* xhat, float* act, float* rstd_out) {
    int row = blockIdx.x * 4 + (threadIdx.x >> 6), lane = threadIdx.x & 63;
    if (row >= R) return;
    const float* z = Z + (int64_t)row * H;
    float v[MAXH];
    constexpr int nper = MAXH;
    float s = 0.f;
    for (int q = 0; q < nper; q++) {
        int c = lane + 64 * q;
        v[q] = c < H ? z[c] : 0.f;
        s += v[q];
    }
    float* xo = xhat + (int64_t)row * H;
    float* ao = act + (int64_t)row * H;
    if (!use_ln) {
        for (int q = 0; q < nper; q++) {
            int c = lane + 64 * q;
            if (c < H) {
                xo[c] = v[q];
                ao[c] = v[q] > 0.f ? v[q] : v[q] * slope;
            }
        }
        return;
    }
    float mean = wave_sum(s) / (float)H;
    float s2 = 0.f;
    for (int q = 0; q < nper; q++) {
        int c = lane + 64 * q;
        float d = c < H ? v[q] - mean : 0.f;
        s2 += d * d;
    }
    float var = wave_sum(s2) / (float)H;
    float rs = 1.f / sqrtf(var + 1e-5f);
    for (int q = 0; q < nper; q++) {
        int c = lane + 64 * q;
        if (c < H) {
            float xh = (v[q] - mean) * rs;
            float h = xh * gamma[c] + beta[c];
            xo[c] = xh;
            ao[c] = h > 0.f ? h : h * slope;
        }
    }
    if (lane == 0) rstd_out[row] = rs;
}

// bf16 inference variant: Z bf16 in, bf16(LeakyReLU(bf16(LN(Z)))) out (torch bf16 module chain).
template <int MAXH>
__global__ void __launch_bounds__(256) ln_act_fwd_bf16(const uint16_t* Z, const uint16_t* gamma, const uint16_t* beta, int R,
                                                      int H, float slope, int use_ln, uint16_t* out) {
    int row = blockIdx.x * 4 + (threadIdx.x >> 6), lane = threadIdx.x & 63;
    if (row >= R) return;
    const uint16_t* z = Z + (int64_t)row * H;
    float v[MAXH];
    constexpr int nper = MAXH;
    float s = 0.f;
    for (int q = 0; q < nper; q++) {
        int c = lane + 64 * q;
        v[q] = c < H ? bf2f(z[c]) : 0.f;
        s += v[q];
    }
    uint16_t* o = out + (int64_t)row * H;
    float mean = 0.f, rs = 1.f;
    if (use_ln) {
        mean = wave_sum(s) / (float)H;
        float s2 = 0.f;
        for (int q = 0; q < nper; q++) {
            int c = lane + 64 * q;
            float d = c < H ? v[q] - mean : 0.f;
            s2 += d * d;
        }
        rs = 1.f / sqrtf(wave_sum(s2) / (float)H + 1e-5f);
    }
    for (int q = 0; q < nper; q++) {
        int c = lane + 64 * q;
        if (c < H) {
            float h = use_ln ? bf2f(f2bf((v[q] - mean) * rs * bf2f(gamma[c]) + bf2f(beta[c]))) : v[q];
            o[c] = f2bf(h > 0.f ? h : h * slope);
        }
    }
}

// Backward of LeakyReLU(LN(Z)): dZ from dA; per-block column partials of
// dbias = sum dZ, dgamma = sum dH*xhat, dbeta = sum dH -> part[blk][3][H] (the flat parameter
// order Linear.bias, LayerNorm.weight, LayerNorm.bias, so one reduction serves all three).
constexpr int LNB_ROWS = 128;
template <int MAXH>
__global__ void __launch_bounds__(256) ln_act_bwd(const float* dA, const float* xhat, const float* rstd, const float* gamma,
                                                 const float* beta, int R, int H, float slope, int use_ln, float* dZ,
                                                 float* part) {
    __shared__ float red[4][3][1024];
    int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
    constexpr int nper = MAXH;
    float pg[MAXH], pb[MAXH], pz[MAXH];
    for (int q = 0; q < nper; q++) pg[q] = pb[q] = pz[q] = 0.f;
    int r0 = blockIdx.x * LNB_ROWS;
    for (int rr = w; rr < LNB_ROWS; rr += 4) {
        int row = r0 + rr;
        if (row >= R) break;
        const float* da = dA + (int64_t)row * H;
        const float* xh = xhat + (int64_t)row * H;
        float dh[MAXH], x[MAXH];
        float s1 = 0.f, s2 = 0.f;
        for (int q = 0; q < nper; q++) {
            int c = lane + 64 * q;
            dh[q] = 0.f;
            x[q] = 0.f;
            if (c < H) {
                x[q] = xh[c];
                float h = use_ln ? x[q] * gamma[c] + beta[c] : x[q];
                dh[q] = h > 0.f ? da[c] : da[c] * slope;
                if (use_ln) {
                    float gg = dh[q] * gamma[c];
                    s1 += gg;
                    s2 += gg * x[q];
                }
            }
        }
        float* dz = dZ + (int64_t)row * H;
        if (use_ln) {
            float m1 = wave_sum(s1) / (float)H, m2 = wave_sum(s2) / (float)H;
            float rs = rstd[row];
            for (int q = 0; q < nper; q++) {
                int c = lane + 64 * q;
                if (c < H) {
                    float d = rs * (dh[q] * gamma[c] - m1 - x[q] * m2);
                    dz[c] = d;
                    pg[q] += dh[q] * x[q];
                    pb[q] += dh[q];
                    pz[q] += d;
                }
            }
        } else {
            for (int q = 0; q < nper; q++) {
                int c = lane + 64 * q;
                if (c < H) {
                    dz[c] = dh[q];
                    pz[q] += dh[q];
                }
            }
        }
    }
    for (int q = 0; q < nper; q++) {
        int c = lane + 64 * q;
        if (c < H) {
            red[w][0][c] = pz[q];
            red[w][1][c] = pg[q];
            red[w][2][c] = pb[q];
        }
    }
    __syncthreads();
    for (int e = threadIdx.x; e < 3 * H; e += 256) {
        int k = e / H, c = e % H;
        part[(int64_t)blockIdx.x * 3 * H + e] = red[0][k][c] + red[1][k][c] + red[2][k][c] + red[3][k][c];
    }
}

// NPER (columns per lane) dispatch: H <= 64 * NPER
#define RLGPU_NPER_DISPATCH(NAME)                                  \
    inline decltype(&NAME<16>) NAME##_any(int H) {                 \
        if (H <= 64) return &NAME<1>;                              \
        if (H <= 128) return &NAME<2>;                             \
        if (H <= 256) return &NAME<4>;                             \
        if (H <= 512) return &NAME<8>;                             \
        return &NAME<16>;                                          \
    }
RLGPU_NPER_DISPATCH(ln_act_fwd_f32)
RLGPU_NPER_DISPATCH(ln_act_fwd_bf16)
RLGPU_NPER_DISPATCH(ln_act_bwd)

// Per-block column partial sums of X [R, Cn] (Cn <= 1024): part[blk][Cn].
constexpr int CS_ROWS = 256;
__global__ void __launch_bounds__(256) colsum_partial(const float* X, int R, int Cn, float* part) {
    int r0 = blockIdx.x * CS_ROWS;
    for (int c = threadIdx.x; c < Cn; c += 256) {
        float s = 0.f;
        for (int r = r0; r < min(R, r0 + CS_ROWS); r++) s += X[(int64_t)r * Cn + c];
        part[(int64_t)blockIdx.x * Cn + c] = s;
    }
}

// grad[c] += sum_b part[b*stride + off + c] for c < n: 16 row groups x 64 columns per
// 1024-thread block, combined in LDS in a fixed order (deterministic).
__global__ void __launch_bounds__(1024) reduce_cols(const float* part, int nblk, int64_t stride, int64_t off, int n,
                                                   float* grad) {
    __shared__ float red[16][64];
    int cl = threadIdx.x & 63, gi = threadIdx.x >> 6;
    int c = blockIdx.x * 64 + cl;
    float s = 0.f;
    if (c < n)
        for (int b = gi; b < nblk; b += 16) s += part[(int64_t)b * stride + off + c];
    red[gi][cl] = s;
    __syncthreads();
    if (gi == 0 && c < n) {
        float tot = 0.f;
        for (int k = 0; k < 16; k++) tot += red[k][cl];
        grad[c] += tot;
    }
}

}  // namespace mlp

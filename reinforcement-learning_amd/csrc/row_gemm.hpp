// row_gemm.hpp -- full-row H3 GEMMs of the training path (gfx950): one workgroup owns 64 rows and ALL N output
// columns (N = 128 NBJ <= 512), so a row-wise epilogue -- LayerNorm + LeakyReLU forward -- runs on the GEMM's
// registers instead of in a second pass over the output.
//
//   z[i, j]   = sum_k A[i, k] W[j, k] + b[j]        (Linear.forward, Models.cpp:42-68; A fp32 [I][lda], W the
//                                                    layer's pre-split scaled fp16 planes, mlp::split_weight_h3)
//   act[i, :] = LeakyReLU(LayerNorm(z[i, :]) * gamma + beta),  stats[i] = (mean, rstd)   (EPI = ROW_LN)
//
// and the input-gradient GEMM of a hidden layer with the backward of its LayerNorm + LeakyReLU (EPI = ROW_LNB):
//   dA[i, c]  = sum_o dZ'[i, o] W'[o, c]              (the next layer's dX: dZ' its pre-activation gradient,
//                                                      W' its pre-split transposed planes)
//   dZ[i, :]  = rstd (dH g - mean(dH g) - xhat mean(dH g xhat)),  dH = dA * LeakyReLU'(h)   (mlp::ln_act_bwd's
//               formulas on xhat = (z - mean) rstd recomputed from this layer's z and stats)
//   part[blk] = per-column sums over the block's 64 rows of dZ, dH xhat, dH (the Linear.bias / LayerNorm.weight /
//               LayerNorm.bias gradient partials, ln_act_bwd's [blk][3][H] layout, reduced by mlp::reduce_batch)
//
// Arithmetic is the H3 scheme of mlp::gemm_x6 (A scaled by its tensor's power of two and split into fp16 h + l,
// products l.h, h.l, h.h into one f32 accumulator per 16-deep k step, the same epilogue scaling), so z is
// bit-identical to the 128 x 128 kernels'.  The LayerNorm reduces each row across the 4 waves (two passes: mean,
// then the biased variance of z - mean; eps 1e-5), in a fixed order: the sums differ in rounding order from the
// wave-per-row mlp::ln_act_fwd_f32, not in operations.
//
// Pipeline (gemm_h3r's): both operands travel global -> LDS by global_load_lds_dwordx4 into a ring of NS stages of
// RK k (A as fp32 rows, W as its two fp16 planes), NS - 1 stages in flight across the raw barriers; every wave
// splits the A fragments it reads (all 64 rows) and reads the W fragments of its own 32 NBJ columns.  Per 16-deep
// k step a wave issues 2 x NBJ x 3 MFMAs for 4 + 2 NBJ LDS reads (the 128 x 128 tile: 12 for 8).
#pragma once
#include "mlp_kernels.hpp"

namespace mlp {

constexpr int RM = 64;  // rows per workgroup
enum { ROW_PLAIN = 0, ROW_LN = 1, ROW_LNB = 2 };

struct RowArgs {
    const float* A;          // [I][lda] fp32, k contiguous
    int64_t lda;
    const uint16_t* B;       // pre-split planes [2][rows_pad][ldb] (rows = output columns j)
    int64_t ldb, bplane;
    const float* bscale;     // [N] inverse per-row scales of the planes
    const float* amax_a;     // 64 shards of max |A| (H3 operand scale)
    const float* bias;       // [N]
    float* C;                // z [I][ldc]
    int64_t ldc;
    int I, N, K;
    // ROW_LN / ROW_LNB
    const float* gamma;
    const float* beta;
    float slope;
    float* act;              // ROW_LN: [I][N]
    float2* stats;           // [I] (mean, rstd): ROW_LN writes them, ROW_LNB reads them
    float* amax_out;         // 64 shards of max |act| (ROW_LN) or |dZ| (ROW_LNB) for the next H3 GEMM, or null
    // ROW_LNB: this layer's pre-norm z [I][N] and the column partials [gridDim][3][N]; C receives dZ
    const float* Z;
    float* part;
};

template <int RK, int NBJ>
struct RowGeom {
    static constexpr int N = 128 * NBJ;
    static constexpr int AROW = RK * 4, BROW = RK * 2;  // bytes per LDS row
    static constexpr int ABYTES = RM * AROW, BPLANE = N * BROW;
    static constexpr int STAGE = ABYTES + 2 * BPLANE;
    static constexpr int AINS = ABYTES / 1024 / 4, BINS = 2 * BPLANE / 1024 / 4;  // 1 KB DMAs per wave and stage
    static constexpr int ARPI = 1024 / AROW, BRPI = 1024 / BROW;                 // rows per DMA
    static_assert(ABYTES % 4096 == 0 && (2 * BPLANE) % 4096 == 0, "whole DMA instructions per wave");
};

// sum over the 32 lanes of each half-wave (lanes l and l ^ o, o < 32): the lanes holding one row's columns
DEV float half_sum(float v) {
#pragma unroll
    for (int o = 1; o < 32; o <<= 1) v += __shfl_xor(v, o, 64);
    return v;
}

template <int RK, int NS, int NBJ, int EPI>
__global__ void __launch_bounds__(256, 1) gemm_row(RowArgs g) {
    using G = RowGeom<RK, NBJ>;
    static_assert(NS * G::STAGE + 4 * RM * 4 <= 160 * 1024, "ring exceeds the CU's LDS");
    constexpr int NV = (G::AINS + G::BINS) * (NS - 2);  // DMAs per wave allowed in flight at a stage's wait
    __shared__ __attribute__((aligned(16))) uint8_t ring[NS * G::STAGE];
    __shared__ float red[4][RM];  // per-wave row partials of the LayerNorm sums
    const int t = threadIdx.x, lane = t & 63, w = t >> 6;
    const int l32 = lane & 31, hk = lane >> 5;
    const int i0 = blockIdx.x * RM, cw0 = w * 32 * NBJ;  // this wave's first column
    const int K = g.K;
    const int pa = h3_pow(shard_max_bits(g.amax_a));
    const float sa = pow2f(pa);
    const float* zero = reinterpret_cast<const float*>(g_zero_row);
    const float* asrc[G::AINS];
    int akc[G::AINS];
#pragma unroll
    for (int q = 0; q < G::AINS; q++) {
        const int r = (w * G::AINS + q) * G::ARPI + lane / (G::AROW / 16);
        const int c = rswz<G::AROW>(r, lane % (G::AROW / 16));
        akc[q] = 4 * c;
        asrc[q] = (i0 + r < g.I) ? g.A + (int64_t)(i0 + r) * g.lda + 4 * c : nullptr;
    }
    const uint16_t* bsrc[G::BINS];
#pragma unroll
    for (int q = 0; q < G::BINS; q++) {
        constexpr int PER_PLANE = G::BPLANE / 1024;
        const int e = w * G::BINS + q, p = e / PER_PLANE;
        const int r = (e % PER_PLANE) * G::BRPI + lane / (G::BROW / 16);
        const int c = rswz<G::BROW>(r, lane % (G::BROW / 16));
        bsrc[q] = g.B + p * g.bplane + (int64_t)r * g.ldb + 8 * c;
    }
    const int nst = (K + RK - 1) / RK;
    auto issue = [&](int s) {
        uint8_t* dst = ring + (s % NS) * G::STAGE;
        const int k0 = s * RK;
        const bool live = s < nst;
#pragma unroll
        for (int q = 0; q < G::AINS; q++) {
            const bool ok = live && asrc[q] && (k0 + akc[q] < K);
            glds16(ok ? asrc[q] + k0 : zero, dst + (w * G::AINS + q) * 1024);
        }
#pragma unroll
        for (int q = 0; q < G::BINS; q++)
            glds16(live ? (const void*)(bsrc[q] + k0) : (const void*)zero, dst + G::ABYTES + (w * G::BINS + q) * 1024);
    };
    f32x16 acc[2][NBJ];
#pragma unroll
    for (int a = 0; a < 2; a++)
#pragma unroll
        for (int b = 0; b < NBJ; b++)
#pragma unroll
            for (int r = 0; r < 16; r++) acc[a][b][r] = 0.f;
#pragma unroll
    for (int s = 0; s < NS - 1; s++) issue(s);
    for (int it = 0; it < nst; it++) {
        asm volatile("s_waitcnt vmcnt(%0)\n\ts_waitcnt lgkmcnt(0)\n\ts_barrier" ::"n"(NV) : "memory");
        issue(it + NS - 1);
        const uint8_t* As = ring + (it % NS) * G::STAGE;
        const uint8_t* Bs = As + G::ABYTES;
#pragma unroll
        for (int ks = 0; ks < RK / 16; ks++) {
            h16x8 ah[2], al[2], bh[NBJ], bl[NBJ];
#pragma unroll
            for (int u = 0; u < 2; u++) {
                const int ra = 32 * u + l32, sa0 = ks * 4 + 2 * hk;
                f32x4_t v[2];
                v[0] = *(const f32x4_t*)(As + ra * G::AROW + rswz<G::AROW>(ra, sa0) * 16);
                v[1] = *(const f32x4_t*)(As + ra * G::AROW + rswz<G::AROW>(ra, sa0 + 1) * 16);
                u32x4_t h, l;
                split2h(v, sa, h, l);
                ah[u] = __builtin_bit_cast(h16x8, h);
                al[u] = __builtin_bit_cast(h16x8, l);
            }
#pragma unroll
            for (int tj = 0; tj < NBJ; tj++) {
                const int rb = cw0 + 32 * tj + l32;
                const int ob = rb * G::BROW + rswz<G::BROW>(rb, ks * 2 + hk) * 16;
                bh[tj] = *(const h16x8*)(Bs + ob);
                bl[tj] = *(const h16x8*)(Bs + G::BPLANE + ob);
            }
#pragma unroll
            for (int ti = 0; ti < 2; ti++)
#pragma unroll
                for (int tj = 0; tj < NBJ; tj++) {
                    f32x16 c = acc[ti][tj];
                    c = __builtin_amdgcn_mfma_f32_32x32x16_f16(al[ti], bh[tj], c, 0, 0, 0);  // l h
                    c = __builtin_amdgcn_mfma_f32_32x32x16_f16(ah[ti], bl[tj], c, 0, 0, 0);  // h l
                    acc[ti][tj] = __builtin_amdgcn_mfma_f32_32x32x16_f16(ah[ti], bh[tj], c, 0, 0, 0);  // h h
                }
        }
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the zero-row DMAs past the last stage
    // z = acc * (2^-pa / s_j) + b_j, gemm_x6's epilogue arithmetic; the 32 x 32 block layout: lane (l32, hk),
    // register r -> row 32 ti + (r & 3) + 8 (r >> 2) + 4 hk, column cw0 + 32 tj + l32
    float bj[NBJ];
#pragma unroll
    for (int tj = 0; tj < NBJ; tj++) {
        const int j = cw0 + 32 * tj + l32;
        const float csc = g.bscale[j];
        bj[tj] = g.bias ? g.bias[j] : 0.f;
#pragma unroll
        for (int ti = 0; ti < 2; ti++)
#pragma unroll
            for (int r = 0; r < 16; r++) acc[ti][tj][r] = ldexpf(acc[ti][tj][r] * csc, -pa) + bj[tj];
    }
    auto rowof = [&](int ti, int r) { return 32 * ti + (r & 3) + 8 * (r >> 2) + 4 * hk; };
    if constexpr (EPI != ROW_LNB) {
#pragma unroll
        for (int ti = 0; ti < 2; ti++)
#pragma unroll
            for (int r = 0; r < 16; r++) {
                const int i = i0 + rowof(ti, r);
                if (i < g.I) {
                    float* zr = g.C + (int64_t)i * g.ldc + cw0 + l32;
#pragma unroll
                    for (int tj = 0; tj < NBJ; tj++) zr[32 * tj] = acc[ti][tj][r];
                }
            }
    }
    if constexpr (EPI == ROW_LNB) {
        // acc holds dA.  Pass 1: dH = dA * LeakyReLU'(h) (kept in acc), row sums of dH g and dH g xhat; pass 2:
        // dZ, its column partials.  z is read twice (the second time from the cache), xhat recomputed with the
        // forward's operations.
        const float invN = 1.f / (float)G::N;
        float gj[NBJ], bt[NBJ];
#pragma unroll
        for (int tj = 0; tj < NBJ; tj++) {
            gj[tj] = g.gamma[cw0 + 32 * tj + l32];
            bt[tj] = g.beta[cw0 + 32 * tj + l32];
        }
        __shared__ float red2[4][RM];
#pragma unroll
        for (int ti = 0; ti < 2; ti++)
#pragma unroll
            for (int r = 0; r < 16; r++) {
                const int i = min(i0 + rowof(ti, r), g.I - 1);  // a row past I recomputes row I - 1 (not stored)
                const float2 st = g.stats[i];
                const float* zr = g.Z + (int64_t)i * G::N + cw0 + l32;
                float s1 = 0.f, s2 = 0.f;
#pragma unroll
                for (int tj = 0; tj < NBJ; tj++) {
                    const float xh = (zr[32 * tj] - st.x) * st.y;
                    const float h = xh * gj[tj] + bt[tj];
                    const float dh = h > 0.f ? acc[ti][tj][r] : acc[ti][tj][r] * g.slope;
                    acc[ti][tj][r] = dh;
                    const float gg = dh * gj[tj];
                    s1 += gg;
                    s2 += gg * xh;
                }
                s1 = half_sum(s1);
                s2 = half_sum(s2);
                if (l32 == 0) {
                    red[w][rowof(ti, r)] = s1;
                    red2[w][rowof(ti, r)] = s2;
                }
            }
        __syncthreads();
        float pz[NBJ], pg[NBJ], pb[NBJ];
#pragma unroll
        for (int tj = 0; tj < NBJ; tj++) pz[tj] = pg[tj] = pb[tj] = 0.f;
        uint32_t vmax = 0;
#pragma unroll
        for (int ti = 0; ti < 2; ti++)
#pragma unroll
            for (int r = 0; r < 16; r++) {
                const int row = rowof(ti, r), i = i0 + row;
                if (i >= g.I) continue;
                const float m1 = (((red[0][row] + red[1][row]) + red[2][row]) + red[3][row]) * invN;
                const float m2 = (((red2[0][row] + red2[1][row]) + red2[2][row]) + red2[3][row]) * invN;
                const float2 st = g.stats[i];
                const float* zr = g.Z + (int64_t)i * G::N + cw0 + l32;
                float* dz = g.C + (int64_t)i * g.ldc + cw0 + l32;
#pragma unroll
                for (int tj = 0; tj < NBJ; tj++) {
                    const float xh = (zr[32 * tj] - st.x) * st.y;
                    const float dh = acc[ti][tj][r];
                    const float d = st.y * (dh * gj[tj] - m1 - xh * m2);
                    dz[32 * tj] = d;
                    pz[tj] += d;
                    pg[tj] += dh * xh;
                    pb[tj] += dh;
                    const uint32_t b = abs_bits(d);
                    vmax = b > vmax ? b : vmax;
                }
            }
        // the two half-waves hold the same columns' other rows
        float* out = g.part + (int64_t)blockIdx.x * 3 * G::N + cw0 + l32;
#pragma unroll
        for (int tj = 0; tj < NBJ; tj++) {
            const float z2 = pz[tj] + __shfl_xor(pz[tj], 32, 64);
            const float g2 = pg[tj] + __shfl_xor(pg[tj], 32, 64);
            const float b2 = pb[tj] + __shfl_xor(pb[tj], 32, 64);
            if (hk == 0) {
                out[32 * tj] = z2;
                out[G::N + 32 * tj] = g2;
                out[2 * G::N + 32 * tj] = b2;
            }
        }
        if (g.amax_out) h3_amax_commit(g.amax_out, vmax);
    }
    if constexpr (EPI == ROW_LN) {
        const float invN = 1.f / (float)G::N;
        float mean[2][16], rs[2][16];
        // pass 1: row sums -> mean; pass 2: sums of (z - mean)^2 -> rstd
#pragma unroll
        for (int pass = 0; pass < 2; pass++) {
#pragma unroll
            for (int ti = 0; ti < 2; ti++)
#pragma unroll
                for (int r = 0; r < 16; r++) {
                    float s = 0.f;
#pragma unroll
                    for (int tj = 0; tj < NBJ; tj++) {
                        const float d = pass ? acc[ti][tj][r] - mean[ti][r] : acc[ti][tj][r];
                        s += pass ? d * d : d;
                    }
                    s = half_sum(s);
                    if (l32 == 0) red[w][rowof(ti, r)] = s;
                }
            __syncthreads();
#pragma unroll
            for (int ti = 0; ti < 2; ti++)
#pragma unroll
                for (int r = 0; r < 16; r++) {
                    const int row = rowof(ti, r);
                    const float tot = ((red[0][row] + red[1][row]) + red[2][row]) + red[3][row];
                    if (pass == 0) mean[ti][r] = tot * invN;
                    else rs[ti][r] = 1.f / sqrtf(tot * invN + 1e-5f);
                }
            __syncthreads();
        }
        float gj[NBJ], bt[NBJ];
#pragma unroll
        for (int tj = 0; tj < NBJ; tj++) {
            gj[tj] = g.gamma[cw0 + 32 * tj + l32];
            bt[tj] = g.beta[cw0 + 32 * tj + l32];
        }
        uint32_t vmax = 0;
#pragma unroll
        for (int ti = 0; ti < 2; ti++)
#pragma unroll
            for (int r = 0; r < 16; r++) {
                const int i = i0 + rowof(ti, r);
                if (i >= g.I) continue;
                float* ar = g.act + (int64_t)i * G::N + cw0 + l32;
#pragma unroll
                for (int tj = 0; tj < NBJ; tj++) {
                    const float xh = (acc[ti][tj][r] - mean[ti][r]) * rs[ti][r];
                    const float hv = xh * gj[tj] + bt[tj];
                    const float a = hv > 0.f ? hv : hv * g.slope;
                    ar[32 * tj] = a;
                    const uint32_t b = abs_bits(a);
                    vmax = b > vmax ? b : vmax;
                }
                if (w == 0 && l32 == 0) g.stats[i] = make_float2(mean[ti][r], rs[ti][r]);
            }
        if (g.amax_out) h3_amax_commit(g.amax_out, vmax);
    }
}

}  // namespace mlp

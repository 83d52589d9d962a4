// infer_kernels.hpp -- fused 16-bit MLP inference: one launch runs a whole actor / critic forward
// (obs f32 -> bf16, every Linear + LayerNorm + LeakyReLU, the output Linear) and then either samples
// the actions (InferActions, PPOLearner.cpp:114-184) or writes the f32 outputs (InferCritic,
// Learner.cpp:863-900; Model::Forward under RLGPU_INFER_BF16).
//
// The unfused path (ppo.hip forward_half: rows_to_bf16 -> gemm_bf16 -> ln_act_fwd_bf16 -> ... ->
// sample_actions) round-trips every activation through HBM and costs ~6 launches per step; here a
// workgroup keeps its IR = 64 rows resident in LDS for the whole network.  The arithmetic is the
// unfused path's, operation for operation: the same v_mfma_f32_32x32x16 instruction over the same K
// order (16-deep steps from k = 0), the same 16-bit rounding of (acc + bias), the same wave-per-row
// LayerNorm reduction (hcol column ownership, wave_sum order) and the same per-row sampler
// (ppo::sample_rows), so both paths produce the same bits.
//
// Layout.  LDS Xs[64][520] 16-bit holds the current layer input (the workgroup's rows, k contiguous,
// zero past the layer's width up to the next multiple of 16).  The weights come from a fragment-major
// copy (weight_to_frag): for 32-row tile jt and 16-deep step ks, the 64 lanes' MFMA B fragments are
// one contiguous 1 KB block, so every weight load of a wave is fully coalesced, and the copy is zero
// padded to whole tiles and steps.  8 waves: wave w owns the 32-column output tiles w and w + 8 of a
// hidden layer (<= 512 columns) for both 32-row halves, and column tile (w & 3) of row half (w >> 2)
// of the output layer (<= 128 columns).  A fragments come from LDS (shared by the waves); each wave
// streams its own weight tiles from L2 into registers one 64-deep K chunk ahead of its MFMAs.  After
// a layer's MFMAs the accumulators (+ bias, rounded) overwrite Xs in place, then LayerNorm + LeakyReLU
// and the sampler run with each wave on 8 rows interleaved, so their cross-lane reductions overlap.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "mlp_kernels.hpp"
#include "ppo_kernels.hpp"

namespace infer {

using mlp::bf16x8;
using mlp::f32x16;
using mlp::h2f;
using mlp::f2h;
using mlp::u32x4;

constexpr int IR = 64;             // rows per workgroup
constexpr int IW = 8;              // waves per workgroup
constexpr int IT = 64 * IW;        // threads
constexpr int IRW = IR / IW;       // rows per wave in the row-parallel phases
constexpr int IMAX = 512;          // widest layer input / hidden layer
constexpr int IPITCH = IMAX + 8;   // LDS row pitch (16-bit): 1040 B, rows 4 banks apart
// the sampler's probs (ppo::sample_rows) in each row of Xs past its <= kMaxA 16-bit logits
constexpr int kSampleProbs = 128;
static_assert(ppo::kMaxA <= kSampleProbs && kSampleProbs * 2 + ppo::kMaxA * 4 <= IPITCH * 2, "probs fit a row of Xs");
constexpr int IOUT = 128;          // widest output layer (4 x 32-column tiles)
constexpr int kMaxLinear = 9;      // RLGPU_MAX_LAYERS hidden + the output layer

// 16-bit weight copy in MFMA B-fragment order: element e of lane l of (tile jt, step ks) is
// W[jt * 32 + (l & 31)][ks * 16 + 8 (l >> 5) + e] (0 outside [out] x [in]), at ((jt * KS + ks) * 64 + l) * 8 + e.
inline int64_t frag_size(int out, int in) { return (int64_t)((out + 31) / 32) * ((in + 15) / 16) * 512; }
template <bool F16>
__global__ void weight_to_frag(const float* w, int out, int in, uint16_t* f) {
    const int KS = (in + 15) / 16, JT = (out + 31) / 32;
    const int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (e >= (int64_t)JT * KS * 512) return;
    const int el = (int)(e & 7), l = (int)((e >> 3) & 63);
    const int64_t blk = e >> 9;
    const int ks = (int)(blk % KS), jt = (int)(blk / KS);
    const int j = jt * 32 + (l & 31), k = ks * 16 + 8 * (l >> 5) + el;
    f[e] = (j < out && k < in) ? mlp::f2h<F16>(w[(int64_t)j * in + k]) : (uint16_t)0;
}

struct InferArgs {
    const float* X;                // [n][in] f32 obs
    int n, in;
    const uint16_t* P;             // padded 16-bit parameter copy (bias / LayerNorm vectors)
    const uint16_t* F;             // fragment-major 16-bit weights
    int nl;                        // Linear layers (hidden + output)
    int width[kMaxLinear + 1];     // width[0] = in, width[l + 1] = outputs of Linear l
    int64_t fw[kMaxLinear];        // offsets of the fragment weights in F
    int64_t hb[kMaxLinear], hg[kMaxLinear], hbe[kMaxLinear];  // offsets in P (-1: no LayerNorm)
    float slope;
    int use_ln;
    int mode;                      // 0: f32 outputs out_f [n][out]; 1: sample actions
    float* out_f;
    const uint8_t* masks;          // mode 1: [n][out]
    int det;
    uint64_t seed, step;
    int64_t row0;                  // global row number of X's row 0 (the sampler's Philox counter)
    int32_t* act;
    float* logp;                   // may be null
    const uint8_t* row_sel;        // mode 1, optional: only rows with (row_sel != 0) == sel are written
    int sel;
    unsigned long long* trace;     // optional: per-workgroup phase timestamps (wall clock), 16 per WG
};
#define INFER_MARK(p) \
    if (a.trace && threadIdx.x == 0) a.trace[blockIdx.x * 16 + (p)] = wall_clock64()

// acc[i][c] = Xs[row tile ti0 + i] . W[column tile jt[c]]^T over the layer's KS steps; column tiles
// c >= nc skip their MFMAs.  The weight loads are unconditional (clamped to the last step), so no
// branch sits between a load and its MFMA and the wait counts stay exact.
template <int NR, int NC, bool F16>
DEV void linear_tiles(const uint16_t (*Xs)[IPITCH], const uint16_t* F, int KS, const int (&jt)[NC], int ti0, int nc_act,
                      int lane, f32x16 (&acc)[NR][NC]) {
    const uint16_t* base[NC];
#pragma unroll
    for (int c = 0; c < NC; c++) base[c] = F + ((int64_t)jt[c] * KS * 64 + lane) * 8;
    const uint16_t* arow[NR];
#pragma unroll
    for (int i = 0; i < NR; i++) {
        arow[i] = Xs[(ti0 + i) * 32 + (lane & 31)] + 8 * (lane >> 5);
#pragma unroll
        for (int c = 0; c < NC; c++)
#pragma unroll
            for (int r = 0; r < 16; r++) acc[i][c][r] = 0.f;
    }
    const int nch = (KS + 3) / 4;  // 64-deep chunks
    auto load = [&](u32x4 (&b)[4][NC], int kc) {
#pragma unroll
        for (int s = 0; s < 4; s++) {
            const int ks = min(kc * 4 + s, KS - 1);
#pragma unroll
            for (int c = 0; c < NC; c++) b[s][c] = *reinterpret_cast<const u32x4*>(base[c] + ks * 512);
        }
    };
    auto step = [&](const u32x4 (&b)[4][NC], int kc) {
#pragma unroll
        for (int s = 0; s < 4; s++) {
            const int ks = kc * 4 + s;
            if (ks >= KS) break;
            bf16x8 av[NR];
#pragma unroll
            for (int i = 0; i < NR; i++) av[i] = *reinterpret_cast<const bf16x8*>(arow[i] + ks * 16);
#pragma unroll
            for (int c = 0; c < NC; c++) {
                if (c >= nc_act) break;
#pragma unroll
                for (int i = 0; i < NR; i++) acc[i][c] = mlp::mfma16<F16>(av[i], __builtin_bit_cast(bf16x8, b[s][c]), acc[i][c]);
            }
        }
    };
    u32x4 b0[4][NC], b1[4][NC];
    load(b0, 0);
    for (int kc = 0; kc < nch; kc += 2) {
        load(b1, kc + 1);
        step(b0, kc);
        load(b0, kc + 2);
        step(b1, kc + 1);
    }
}

// bf16(LeakyReLU(bf16(LN(z)))) in place on the rows w + IW g (g < IRW) of Xs, interleaved: the
// per-row arithmetic of mlp::ln_act_fwd_bf16<MAXH> (same sums in the same order, the centred value
// computed once and reused, LeakyReLU as max(h, slope h) when 0 <= slope <= 1 -- equal to the
// select for every h); FULL: H == 64 MAXH, no column masks.
template <int MAXH, bool FULL, bool F16>
DEV void ln_act_rows(uint16_t (*Xs)[IPITCH], const uint16_t* gamma, const uint16_t* beta, int H, float slope, int use_ln,
                     int w, int lane) {
    const bool vec = (H % 8 == 0) && (MAXH % 8 == 0);
    const bool maxform = slope >= 0.f && slope <= 1.f;
    auto in = [&](int q) { return FULL || mlp::hcol<MAXH>(lane, q) < H; };
    float g[MAXH], b[MAXH];
#pragma unroll
    for (int q = 0; q < MAXH; q++) {
        const int c = mlp::hcol<MAXH>(lane, q);
        g[q] = (use_ln && in(q)) ? h2f<F16>(gamma[c]) : 1.f;
        b[q] = (use_ln && in(q)) ? h2f<F16>(beta[c]) : 0.f;
    }
    float v[IRW][MAXH];
#pragma unroll
    for (int rg = 0; rg < IRW; rg++) {
        const uint16_t* z = Xs[w + IW * rg];
        if (vec) {
#pragma unroll
            for (int q = 0; q < MAXH; q += 8) {
                const int c = mlp::hcol<MAXH>(lane, q);
                u32x4 t = {0u, 0u, 0u, 0u};
                if (in(q)) t = *reinterpret_cast<const u32x4*>(z + c);
#pragma unroll
                for (int k = 0; k < 4; k++) {
                    v[rg][q + 2 * k] = h2f<F16>((uint16_t)(t[k] & 0xffffu));
                    v[rg][q + 2 * k + 1] = h2f<F16>((uint16_t)(t[k] >> 16));
                }
            }
        } else {
#pragma unroll
            for (int q = 0; q < MAXH; q++) {
                const int c = mlp::hcol<MAXH>(lane, q);
                v[rg][q] = in(q) ? h2f<F16>(z[c]) : 0.f;
            }
        }
    }
    if (use_ln) {
        float s[IRW];
#pragma unroll
        for (int rg = 0; rg < IRW; rg++) {
            s[rg] = 0.f;
#pragma unroll
            for (int q = 0; q < MAXH; q++) s[rg] += v[rg][q];
        }
#pragma unroll
        for (int rg = 0; rg < IRW; rg++) s[rg] = mlp::wave_sum_x(s[rg]);  // == mlp::wave_sum
#pragma unroll
        for (int rg = 0; rg < IRW; rg++) {
            const float mean = s[rg] / (float)H;
            float s2 = 0.f;
#pragma unroll
            for (int q = 0; q < MAXH; q++) {
                v[rg][q] = in(q) ? v[rg][q] - mean : 0.f;  // centred (masked columns are never stored)
                s2 += v[rg][q] * v[rg][q];
            }
            s[rg] = s2;
        }
#pragma unroll
        for (int rg = 0; rg < IRW; rg++) {
            s[rg] = mlp::wave_sum_x(s[rg]);
            const float rs = 1.f / sqrtf(s[rg] / (float)H + 1e-5f);
#pragma unroll
            for (int q = 0; q < MAXH; q++) v[rg][q] = h2f<F16>(f2h<F16>(v[rg][q] * rs * g[q] + b[q]));
        }
    }
#pragma unroll
    for (int rg = 0; rg < IRW; rg++) {
        uint16_t* z = Xs[w + IW * rg];
        uint16_t o[MAXH];
#pragma unroll
        for (int q = 0; q < MAXH; q++) {
            const float hv = v[rg][q];
            o[q] = f2h<F16>(maxform ? fmaxf(hv, hv * slope) : (hv > 0.f ? hv : hv * slope));
        }
        if (vec) {
#pragma unroll
            for (int q = 0; q < MAXH; q += 8) {
                const int c = mlp::hcol<MAXH>(lane, q);
                u32x4 t;
#pragma unroll
                for (int k = 0; k < 4; k++) t[k] = (uint32_t)o[q + 2 * k] | ((uint32_t)o[q + 2 * k + 1] << 16);
                if (in(q)) *reinterpret_cast<u32x4*>(z + c) = t;
            }
        } else {
#pragma unroll
            for (int q = 0; q < MAXH; q++) {
                const int c = mlp::hcol<MAXH>(lane, q);
                if (in(q)) z[c] = o[q];
            }
        }
    }
}

// accumulator element r of a lane: row ti * 32 + (r & 3) + 8 (r >> 2) + 4 (lane >> 5) of the tile
DEV int acc_row(int ti, int r, int lane) { return ti * 32 + (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5); }

template <bool F16>
__global__ void __launch_bounds__(IT, 1) mlp_infer(InferArgs a) {
    __shared__ uint16_t Xs[IR][IPITCH];
    __shared__ uint8_t Ms[IR * ppo::kMaxA];  // mode 1: the rows' action masks
    __shared__ uint8_t Sel[IR];              // mode 1: row is written (row_sel)
    __shared__ uint16_t Pv[kMaxLinear][3][IMAX];  // bias, LayerNorm weight, LayerNorm bias of each Linear
    const int t = threadIdx.x, lane = t & 63;
    const int w = __builtin_amdgcn_readfirstlane(t >> 6);
    const int r0 = blockIdx.x * IR;
    const int rows = min(IR, a.n - r0);
    INFER_MARK(0);
    // Prologue.  The global reads of the obs rows, the bias / LayerNorm vectors and the masks are all
    // issued (unconditionally, clamped in range) before the first LDS store waits on any of them, so
    // the workgroup pays one memory latency for the three.
    const float* xsrc = a.X + (int64_t)r0 * a.in;   // the workgroup's rows: one contiguous span of X
    const int xtot = rows * a.in;
    const bool xvec = (reinterpret_cast<uintptr_t>(xsrc) & 15) == 0;
    const int nv4 = xvec ? xtot / 4 : 0;            // whole float4s (vector path)
    constexpr int UO = 6, UP = 8, UM = 4;
    float4 ov[UO];
#pragma unroll
    for (int u = 0; u < UO; u++)
        if (nv4 > 0) ov[u] = *reinterpret_cast<const float4*>(xsrc + 4 * min(t + IT * u, nv4 - 1));
    int pre[kMaxLinear + 1];  // bias | LayerNorm weight | LayerNorm bias of Linear l: flat [pre[l], pre[l + 1])
    pre[0] = 0;
#pragma unroll
    for (int l = 0; l < kMaxLinear; l++)
        pre[l + 1] = pre[l] + (l < a.nl ? (a.hg[l] >= 0 ? 3 : 1) * a.width[l + 1] : 0);
    const int ptot = pre[kMaxLinear];
    // (layer l, index in its flat span, width) of flat position f; selects over constant indices keep
    // the per-lane lookups in registers
    struct PSlot {
        int64_t src;
        int idx, N, l;
    };
    auto pslot = [&](int f) {
        PSlot r{a.hb[0] + f, f, a.width[1], 0};
#pragma unroll
        for (int k = 1; k < kMaxLinear; k++)
            if (k < a.nl && f >= pre[k]) r = PSlot{a.hb[k] + (f - pre[k]), f - pre[k], a.width[k + 1], k};
        return r;
    };
    uint16_t pv[UP];
#pragma unroll
    for (int u = 0; u < UP; u++) pv[u] = a.P[pslot(min(t + IT * u, ptot - 1)).src];
    uint8_t selv = 1;  // row_sel of row t
    if (a.mode == 1 && a.row_sel) selv = (a.row_sel[r0 + min(t & (IR - 1), rows - 1)] != 0) == (a.sel != 0);
    const int A = a.width[a.nl];
    const uint8_t* msrc = a.masks + (int64_t)r0 * A;
    const int mtot = rows * A;
    const int nd = (a.mode == 1 && (reinterpret_cast<uintptr_t>(msrc) & 3) == 0) ? mtot / 4 : 0;
    uint32_t mv[UM];
#pragma unroll
    for (int u = 0; u < UM; u++)
        if (nd > 0) mv[u] = *reinterpret_cast<const uint32_t*>(msrc + 4 * min(t + IT * u, nd - 1));
    // obs -> 16-bit (mlp::rows_to_bf16)
    auto put4 = [&](int i, float4 v) {
        const int f = 4 * i;
        int r = f / a.in, c = f - r * a.in;
        const float e[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
        for (int k = 0; k < 4; k++) {
            Xs[r][c] = f2h<F16>(e[k]);
            if (++c == a.in) {
                c = 0;
                r++;
            }
        }
    };
#pragma unroll
    for (int u = 0; u < UO; u++)
        if (t + IT * u < nv4) put4(t + IT * u, ov[u]);
    for (int i = t + IT * UO; i < nv4; i += IT) put4(i, *reinterpret_cast<const float4*>(xsrc + 4 * i));
    for (int f = 4 * nv4 + t; f < xtot; f += IT) {  // the tail (or all of an unaligned span)
        const int r = f / a.in;
        Xs[r][f - r * a.in] = f2h<F16>(xsrc[f]);
    }
    {  // zeros: past `in` up to the first MFMA step boundary, and the rows past n
        const int k16 = (a.in + 15) / 16 * 16, pad = k16 - a.in;
        for (int e = t; e < rows * pad; e += IT) {
            const int r = e / pad;
            Xs[r][a.in + e - r * pad] = 0;
        }
        for (int e = t; e < (IR - rows) * k16; e += IT) {
            const int r = e / k16;
            Xs[rows + r][e - r * k16] = 0;
        }
    }
    auto putp = [&](int f, uint16_t v) {
        const PSlot p = pslot(f);
        const int q = p.idx >= p.N ? (p.idx >= 2 * p.N ? 2 : 1) : 0;
        Pv[p.l][q][p.idx - q * p.N] = v;
    };
#pragma unroll
    for (int u = 0; u < UP; u++)
        if (t + IT * u < ptot) putp(t + IT * u, pv[u]);
    for (int f = t + IT * UP; f < ptot; f += IT) putp(f, a.P[pslot(f).src]);
    if (a.mode == 1) {  // the masks (and row_sel)
#pragma unroll
        for (int u = 0; u < UM; u++)
            if (t + IT * u < nd) *reinterpret_cast<uint32_t*>(&Ms[4 * (t + IT * u)]) = mv[u];
        for (int i = t + IT * UM; i < nd; i += IT)
            *reinterpret_cast<uint32_t*>(&Ms[4 * i]) = *reinterpret_cast<const uint32_t*>(msrc + 4 * i);
        for (int f = 4 * nd + t; f < mtot; f += IT) Ms[f] = msrc[f];
        if (t < IR) Sel[t] = t < rows && selv;
    }
    for (int l = 0; l + 1 < a.nl; l++) {
        const int KS = (a.width[l] + 15) / 16, N = a.width[l + 1], JT = (N + 31) / 32;
        const int jt[2] = {min(w, JT - 1), min(w + IW, JT - 1)};
        const int nt = (w < JT) + (w + IW < JT);
        f32x16 acc[2][2];  // [row half][column tile]
        __syncthreads();
        if (l < 3) INFER_MARK(1 + 2 * l);
        linear_tiles<2, 2, F16>(Xs, a.F + a.fw[l], KS, jt, 0, nt, lane, acc);
        __syncthreads();  // every wave is done reading this layer's input
        if (l < 3) INFER_MARK(2 + 2 * l);
        const uint16_t* bias = Pv[l][0];
        const int n16 = (N + 15) / 16 * 16;
#pragma unroll
        for (int c = 0; c < 2; c++) {
            const int j = (w + IW * c) * 32 + (lane & 31);
            if (c >= nt || j >= n16) continue;
            const float bj = j < N ? h2f<F16>(bias[j]) : 0.f;
#pragma unroll
            for (int i = 0; i < 2; i++)
#pragma unroll
                for (int r = 0; r < 16; r++)
                    Xs[acc_row(i, r, lane)][j] = j < N ? f2h<F16>(acc[i][c][r] + bj) : (uint16_t)0;
        }
        const uint16_t* gg = Pv[l][1];
        const uint16_t* bb = Pv[l][2];
        __syncthreads();
        if (l < 3) INFER_MARK(8 + l);
        if (N == 512) ln_act_rows<8, true, F16>(Xs, gg, bb, N, a.slope, a.use_ln, w, lane);
        else if (N <= 64) ln_act_rows<1, false, F16>(Xs, gg, bb, N, a.slope, a.use_ln, w, lane);
        else if (N <= 128) ln_act_rows<2, false, F16>(Xs, gg, bb, N, a.slope, a.use_ln, w, lane);
        else if (N <= 256) ln_act_rows<4, false, F16>(Xs, gg, bb, N, a.slope, a.use_ln, w, lane);
        else ln_act_rows<8, false, F16>(Xs, gg, bb, N, a.slope, a.use_ln, w, lane);
    }
    // output Linear: wave w owns column tile (w & 3) of row half (w >> 2)
    const int l = a.nl - 1, KS = (a.width[l] + 15) / 16, N = a.width[l + 1], JT = (N + 31) / 32;
    const int jt[1] = {min(w & 3, JT - 1)}, ti = w >> 2;
    f32x16 acc[1][1];
    __syncthreads();
    INFER_MARK(12);
    linear_tiles<1, 1, F16>(Xs, a.F + a.fw[l], KS, jt, ti, (w & 3) < JT, lane, acc);
    INFER_MARK(13);
    const int j = (w & 3) * 32 + (lane & 31);
    const float bj = j < N ? h2f<F16>(Pv[l][0][j]) : 0.f;
    if (a.mode == 0) {  // f32 outputs: the 16-bit-rounded Linear output (gemm_bf16 + bf16_to_f32)
        if (j < N)
#pragma unroll
            for (int r = 0; r < 16; r++) {
                const int i = r0 + acc_row(ti, r, lane);
                if (i < a.n) a.out_f[(int64_t)i * N + j] = h2f<F16>(f2h<F16>(acc[0][0][r] + bj));
            }
        return;
    }
    __syncthreads();  // the logits replace the last hidden activation in Xs
    if (j < N)
#pragma unroll
        for (int r = 0; r < 16; r++) Xs[acc_row(ti, r, lane)][j] = f2h<F16>(acc[0][0][r] + bj);
    __syncthreads();
    INFER_MARK(14);
    {
        const auto rowfn = [&](int g, const uint16_t*& lg, const uint8_t*& mk, float*& pr, int& row, bool& ok) {
            const int r = w + IW * g;
            lg = Xs[r];
            mk = Ms + r * N;
            pr = reinterpret_cast<float*>(&Xs[r][kSampleProbs]);  // the row past its logits: the probs
            row = r0 + r;
            ok = Sel[r] != 0;
        };
        const auto mark = [&](int k) { INFER_MARK(k == 0 ? 7 : 11); };  // trace slots 7 / 11 are free here
        ppo::sample_rows_looped<IRW, F16>(rowfn, N, a.det, a.seed, a.step, a.row0, lane, a.act, a.logp, mark);
    }
    INFER_MARK(15);
}

}  // namespace infer

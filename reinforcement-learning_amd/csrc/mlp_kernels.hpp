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
#include <hip/hip_fp16.h>
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <cstdlib>

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
    int64_t lda, ldb, ldc;
    int I, J, K;
    int kchunk;            // K range per split (multiple of BK)
    int64_t c_split;       // element stride between split partials
    int gx, gy, gz;        // logical tile grid (J tiles, I tiles, K splits); launched as 1-D
    int64_t bplane;        // gemm_x6 with a pre-split B: element stride between the bf16 planes
    // fp16x3 arithmetic (H3): 64 shards of max |x| (float bits) of each operand tensor, and for a
    // pre-split B its per-row inverse scales [rows]
    const float* amax_a;
    const float* amax_b;
    const float* bscale;
};

DEV uint16_t f2bf(float f) {  // round-to-nearest-even (plain cast: NaN stays NaN)
    __hip_bfloat16 b = __float2bfloat16(f);
    return *reinterpret_cast<uint16_t*>(&b);
}
DEV float bf2f(uint16_t u) { return __uint_as_float((uint32_t)u << 16); }
// 16-bit inference storage: bf16 (the reference's seqHalf) or fp16 (F16, BASELINE config C5)
template <bool F16>
DEV float h2f(uint16_t u) {
    if (F16) return __half2float(__ushort_as_half(u));
    return bf2f(u);
}
template <bool F16>
DEV uint16_t f2h(float f) {
    if (F16) return __half_as_ushort(__float2half(f));
    return f2bf(f);
}

// Operand staging.  Every global load is branch-free (divergent bounds branches made the compiler
// drain vmcnt after each load and serialised the register prefetch): absent rows read a zero row,
// out-of-range elements are zeroed by a select after an in-bounds load.  VEC (compile time):
// 16-byte aligned rows whose elements past the bound up to the next multiple of 4 are readable
// and finite (they meet zeros of the other operand).
__device__ float4 g_zero_row[4];  // zero-initialised device memory

template <bool VEC>
DEV float4 load4(const float* p, int c, int lim) {
    const float* z = reinterpret_cast<const float*>(g_zero_row);
    if (VEC) {
        const float* q = (p && c < lim) ? p + c : z;
        return *reinterpret_cast<const float4*>(q);
    }
    const float* base = p ? p : z;
    float v[4];
#pragma unroll
    for (int k = 0; k < 4; k++) {
        bool ok = p && (c + k < lim);
        float t = base[ok ? c + k : 0];
        v[k] = ok ? t : 0.f;
    }
    return make_float4(v[0], v[1], v[2], v[3]);
}

// Per-thread share of one 128 x 32 tile: 4 float4.  KMAJ (global row = output index, k contiguous):
// the 4 row pointers are fixed for the whole K loop (computed once).  !KMAJ (global row = k):
// row pointers follow k.
struct RowPtrs {
    const float* p[4];
};
template <bool KMAJ>
DEV RowPtrs kmaj_rows(const float* base, int64_t ld, int o0, int on) {
    RowPtrs r;
#pragma unroll
    for (int q = 0; q < 4; q++) {
        if (!KMAJ) {
            r.p[q] = nullptr;
            continue;
        }
        int e = threadIdx.x + 256 * q;
        int go = o0 + (e >> 3);
        r.p[q] = go < on ? base + (int64_t)go * ld : nullptr;
    }
    return r;
}
template <bool KMAJ, bool VEC>
DEV void tile_load(float4 (&r)[4], const RowPtrs& rows, const float* base, int64_t ld, int o0, int on, int k0, int ke) {
#pragma unroll
    for (int q = 0; q < 4; q++) {
        int e = threadIdx.x + 256 * q;
        if (KMAJ) {
            r[q] = load4<VEC>(rows.p[q], k0 + (e & 7) * 4, ke);
        } else {
            int k = k0 + (e >> 5);
            const float* p = k < ke ? base + (int64_t)k * ld : nullptr;
            r[q] = load4<VEC>(p, o0 + (e & 31) * 4, on);
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

// XCD-aware tile order.  Workgroups are dispatched round-robin over the 8 XCDs (each with its own
// L2), so consecutive block ids land on different L2s.  Launch a 1-D grid and map block p to the
// logical tile t so that consecutive logical tiles -- the J tiles sharing one A panel, or the
// (I, J) tiles of one split-K chunk -- run on the same XCD and share its L2.
struct Tile {
    int x, y, z;
};
DEV Tile xcd_tile(int gx, int gy, int gz) {
    const int n = gx * gy * gz, p = blockIdx.x;
    const int q = n >> 3, r = n & 7, xcd = p & 7, slot = p >> 3;
    const int t = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + slot;
    Tile o;
    o.x = t % gx;
    o.y = (t / gx) % gy;
    o.z = t / (gx * gy);
    return o;
}

// fp32 GEMM on v_mfma_f32_32x32x2_f32: each MFMA j of a BK step takes k = j (lanes 0-31) and
// k = 16 + j (lanes 32-63) so that k-contiguous tiles are read as 16-byte vectors.
#ifndef RLGPU_GEMM_OCC
#define RLGPU_GEMM_OCC 3
#endif
template <int LA, int LB, bool AV, bool BV>
__global__ void __launch_bounds__(256, RLGPU_GEMM_OCC) gemm_f32(GemmArgs g) {
    constexpr bool AK = LA == A_IK, BKM = LB == B_JK;
    constexpr int ASZ = AK ? BM * (BK + KP) : BK * (BM + MP);
    constexpr int BSZ = BKM ? BN * (BK + KP) : BK * (BN + MP);
    __shared__ float As[ASZ];
    __shared__ float Bs[BSZ];
    const int t = threadIdx.x, lane = t & 63, w = t >> 6;
    const int wm = w >> 1, wn = w & 1;
    const Tile tl = xcd_tile(g.gx, g.gy, g.gz);
    const int i0 = tl.y * BM, j0 = tl.x * BN;
    const int kb = tl.z * g.kchunk;
    const int ke = min(g.K, kb + g.kchunk);
    const int h = lane >> 5, l32 = lane & 31;
    f32x16 acc[2][2];
    for (int a = 0; a < 2; a++)
        for (int b = 0; b < 2; b++)
            for (int r = 0; r < 16; r++) acc[a][b][r] = 0.f;
    float4 ra[4], rb[4];
    const RowPtrs arow = kmaj_rows<AK>(g.A, g.lda, i0, g.I);
    const RowPtrs brow = kmaj_rows<BKM>(g.B, g.ldb, j0, g.J);
    if (kb < ke) {
        tile_load<AK, AV>(ra, arow, g.A, g.lda, i0, g.I, kb, ke);
        tile_load<BKM, BV>(rb, brow, g.B, g.ldb, j0, g.J, kb, ke);
    }
    for (int k0 = kb; k0 < ke; k0 += BK) {
        tile_store<AK>(As, ra);
        tile_store<BKM>(Bs, rb);
        __syncthreads();
        if (k0 + BK < ke) {  // prefetch the next stage into registers while the MFMAs run
            tile_load<AK, AV>(ra, arow, g.A, g.lda, i0, g.I, k0 + BK, ke);
            tile_load<BKM, BV>(rb, brow, g.B, g.ldb, j0, g.J, k0 + BK, ke);
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
    float* C = g.C + (int64_t)tl.z * g.c_split;
    if (i0 + BM <= g.I && j0 + BN <= g.J) {  // interior tile: no bounds checks, one base pointer
        float* cb = C + (int64_t)(i0 + wm * 64 + 4 * h) * g.ldc + j0 + wn * 64 + l32;
#pragma unroll
        for (int ti = 0; ti < 2; ti++)
#pragma unroll
            for (int tj = 0; tj < 2; tj++) {
                const float bj = g.bias ? g.bias[j0 + wn * 64 + tj * 32 + l32] : 0.f;
                float* ct = cb + (int64_t)(ti * 32) * g.ldc + tj * 32;
#pragma unroll
                for (int r = 0; r < 16; r++) ct[(int64_t)((r & 3) + 8 * (r >> 2)) * g.ldc] = acc[ti][tj][r] + bj;
            }
        return;
    }
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

// ---- fp32 GEMM on bf16 MFMA by a three-way split (training path, default).
// gfx950 runs f32-input MFMA at 1/16 of the bf16 rate.  Every f32 operand x is split exactly into
// three bf16 terms, x = h + m + l (h = bf16(x), m = bf16(x - h), l = bf16(x - h - m); each
// subtraction is exact by Sterbenz, and 3 x 8 significant bits cover f32's 24), and
//   a.b ~= h_a h_b + [h_a m_b + m_a h_b + h_a l_b + l_a h_b + m_a m_b]
// on v_mfma_f32_32x32x16_bf16 (bf16 products are exact in f32).  The dropped terms (m l, l m, l l)
// are below 2^-24 relative, so each product carries f32-class error; the leading term and the
// bracketed correction terms accumulate in separate f32 accumulators (summed once at the end) so
// the rounding of the large running sum is the same count as an f32 FMA chain's.  Six bf16 MFMAs
// (6 x 32 cycles per K = 16) replace eight f32 ones (8 x 64 cycles).  Same tiles, layouts, split-K
// and epilogue as gemm_f32; operands are split once per LDS stage into three k-contiguous bf16
// planes, so the MFMA loop reads b128 vectors whatever the global layout.
constexpr int XPAD = 8;            // bf16 pad per LDS row
constexpr int XKMAX = 64;          // deepest stage of any variant: split-K chunks and weight-plane
                                   // padding are multiples of it
typedef unsigned u32x4_t __attribute__((ext_vector_type(4)));

DEV uint32_t pack_bf16x2(float a, float b) { return (uint32_t)f2bf(a) | ((uint32_t)f2bf(b) << 16); }

// split 8 floats (two native 4-vectors) into three bf16x8 planes
typedef float f32x4_t __attribute__((ext_vector_type(4)));
DEV void split3(const f32x4_t (&v)[2], u32x4_t& h, u32x4_t& m, u32x4_t& l) {
#pragma unroll
    for (int p = 0; p < 4; p++) {
        const float x0 = v[p >> 1][(2 * p) & 3], x1 = v[p >> 1][(2 * p + 1) & 3];
        const uint32_t hh = pack_bf16x2(x0, x1);
        const float r0 = x0 - __uint_as_float(hh << 16), r1 = x1 - __uint_as_float(hh & 0xffff0000u);
        const uint32_t mm = pack_bf16x2(r0, r1);
        const float s0 = r0 - __uint_as_float(mm << 16), s1 = r1 - __uint_as_float(mm & 0xffff0000u);
        const uint32_t ll = pack_bf16x2(s0, s1);
        h[p] = hh;
        m[p] = mm;
        l[p] = ll;
    }
}

// ---- fp32 GEMM on fp16 MFMA by a scaled two-way split (H3: RLGPU_GEMM_F16X3).
// Each operand tensor is scaled by a power of two s (exact) that puts its largest magnitude in
// [2^14, 2^15), then every element splits exactly into two fp16 terms, x s = h + l (h = fp16(x s),
// l = fp16(x s - h); the subtraction is exact).  h + l carries 22 significant bits for every
// element within 2^16 of the tensor's largest (below that, an absolute error under 2^-39 of it),
// fp16 x fp16 products are exact in f32, and
//   a.b ~= (h_a h_b + [h_a l_b + l_a h_b]) / (s_a s_b)
// on v_mfma_f32_32x32x16_f16 drops only l_a l_b (below 2^-22 relative): the 3xTF32 scheme of fp32
// emulation, with fp16's narrower exponent range covered by the scale.  Three MFMAs per K = 16
// instead of the x6 path's six, two LDS planes instead of three.  The scales come from 64 shards
// of max |x| that the operand's producer kernel fills (h3_amax_commit), so no extra pass reads the
// tensor; pre-split weights carry one scale per row.
DEV uint32_t shard_max_bits(const float* shards) {  // max over the 64 shards, every lane gets it
    uint32_t v = __float_as_uint(shards[threadIdx.x & 63]);
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
        const uint32_t u = (uint32_t)__shfl_xor((int)v, o, 64);
        v = u > v ? u : v;
    }
    return v;
}
// power-of-two p with amax * 2^p in [2^14, 2^15); 0 for a zero, subnormal, infinite or NaN max
DEV int h3_pow(uint32_t amax_bits) {
    const int e = (int)((amax_bits >> 23) & 255u);
    if (amax_bits > 0x7f7fffffu || e == 0) return 0;
    int p = 14 - (e - 127);
    return p > 126 ? 126 : p;
}
DEV float pow2f(int p) { return __uint_as_float((uint32_t)(p + 127) << 23); }  // p in [-126, 127]
DEV uint16_t f2hf(float f) { return __half_as_ushort(__float2half(f)); }
DEV float hf2f(uint16_t u) { return __half2float(__ushort_as_half(u)); }
DEV uint32_t pack_h2(uint16_t a, uint16_t b) { return (uint32_t)a | ((uint32_t)b << 16); }
// split 8 floats (two native 4-vectors), scaled by sc, into two fp16x8 planes
DEV void split2h(const f32x4_t (&v)[2], float sc, u32x4_t& h, u32x4_t& l) {
#pragma unroll
    for (int p = 0; p < 4; p++) {
        const float x0 = v[p >> 1][(2 * p) & 3] * sc, x1 = v[p >> 1][(2 * p + 1) & 3] * sc;
        const uint16_t h0 = f2hf(x0), h1 = f2hf(x1);
        h[p] = pack_h2(h0, h1);
        l[p] = pack_h2(f2hf(x0 - hf2f(h0)), f2hf(x1 - hf2f(h1)));
    }
}
// Producers: this thread's max |x| bits (vmax) -> block max -> atomicMax into shard blockIdx % 64.
// Must be reached by every thread of the 256-thread block.
DEV void h3_amax_commit(float* shards, uint32_t vmax) {
    __shared__ uint32_t red[4];
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
        const uint32_t u = (uint32_t)__shfl_xor((int)vmax, o, 64);
        vmax = u > vmax ? u : vmax;
    }
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = vmax;
    __syncthreads();
    if (threadIdx.x == 0) {
        uint32_t m = red[0];
        for (int w = 1; w < (int)(blockDim.x >> 6); w++) m = red[w] > m ? red[w] : m;
        atomicMax(reinterpret_cast<unsigned int*>(shards) + (blockIdx.x & 63), m);
    }
}
DEV uint32_t abs_bits(float x) { return __float_as_uint(x) & 0x7fffffffu; }

// Per-thread share of one 128 x XK operand stage (XK = 32 or 64 k): NQ = XK / 16 groups of 8
// consecutive k of one row, held in native 4-vectors (loop-carried prefetch registers stay where
// the loads land, so the wait for them sits at the next stage's store, after this stage's MFMAs).
//   KMAJ (k contiguous in memory): group e = t + 256 q -> row e / KG, k group e % KG (2 float4 loads)
//   !KMAJ (row index contiguous):  group e -> row e & 127, k group e >> 7 (8 scalar loads, each a
//                                  256-byte contiguous wave access)
template <bool KMAJ, int XK>
DEV int xs_row(int q) {
    constexpr int KG = XK / 8;
    const int e = threadIdx.x + 256 * q;
    return KMAJ ? e / KG : e & 127;
}
template <bool KMAJ, int XK>
DEV int xs_kg(int q) {
    constexpr int KG = XK / 8;
    const int e = threadIdx.x + 256 * q;
    return KMAJ ? e % KG : e >> 7;
}
template <bool KMAJ, int XK>
DEV RowPtrs xs_rows(const float* base, int64_t ld, int o0, int on) {
    RowPtrs r;
#pragma unroll
    for (int q = 0; q < 4; q++) {
        const int go = o0 + xs_row<KMAJ, XK>(q);
        r.p[q] = (KMAJ && q < XK / 16 && go < on) ? base + (int64_t)go * ld : nullptr;
    }
    return r;
}
template <bool VEC>
DEV f32x4_t load4v(const float* p, int c, int lim) {
    const float* z = reinterpret_cast<const float*>(g_zero_row);
    if (VEC) return *reinterpret_cast<const f32x4_t*>((p && c < lim) ? p + c : z);
    const float* base = p ? p : z;
    f32x4_t v;
#pragma unroll
    for (int k = 0; k < 4; k++) {
        const bool ok = p && (c + k < lim);
        v[k] = *(ok ? base + c + k : z);
    }
    return v;
}
template <bool KMAJ, bool VEC, int XK>
DEV void xs_load(f32x4_t (&v)[XK / 16][2], const RowPtrs& rows, const float* base, int64_t ld, int o0, int on, int k0,
                 int ke) {
    const float* z = reinterpret_cast<const float*>(g_zero_row);
#pragma unroll
    for (int q = 0; q < XK / 16; q++) {
        const int kk = k0 + xs_kg<KMAJ, XK>(q) * 8;
        if (KMAJ) {
            v[q][0] = load4v<VEC>(rows.p[q], kk, ke);
            v[q][1] = load4v<VEC>(rows.p[q], kk + 4, ke);
        } else {
            const int o = o0 + xs_row<KMAJ, XK>(q);
#pragma unroll
            for (int c = 0; c < 8; c++) {
                const bool ok = (kk + c < ke) && (o < on);
                v[q][c >> 2][c & 3] = *(ok ? base + (int64_t)(kk + c) * ld + o : z);  // absent: the zero row
            }
        }
    }
}
// Unpadded 32-deep planes (row pitch P == XK == 32 halves, 64 B) are XOR-swizzled instead of padded:
// the 16-byte chunk c of row r sits at chunk c ^ ((r >> 2) & 3).  Then both the staging stores
// (ds_write_b128: 8 lanes = 2 rows x 4 chunks, one 128-byte span) and the fragment reads
// (ds_read_b128: 16 lanes = rows {0-3, 12-15, 20-27} + 32 u, one chunk) are conflict-free; the
// padded pitch (80 B) left the stores 2-way conflicted.
template <int P, int XK>
DEV int xchunk(int row, int c) {  // physical chunk of logical chunk c
    static_assert(P != XK || XK == 32, "swizzled planes are 32 deep");
    return P == XK ? (c ^ ((row >> 2) & 3)) : c;
}
template <bool KMAJ, int XK, bool H3, int P = XK + XPAD>
DEV void xs_store(uint16_t (*lds)[BM][P], const f32x4_t (&v)[XK / 16][2], float sc) {
#pragma unroll
    for (int q = 0; q < XK / 16; q++) {
        const int row = xs_row<KMAJ, XK>(q), c = xchunk<P, XK>(row, xs_kg<KMAJ, XK>(q)) * 8;
        if (H3) {
            u32x4_t h, l;
            split2h(v[q], sc, h, l);
            *reinterpret_cast<u32x4_t*>(&lds[0][row][c]) = h;
            *reinterpret_cast<u32x4_t*>(&lds[1][row][c]) = l;
        } else {
            u32x4_t h, m, l;
            split3(v[q], h, m, l);
            *reinterpret_cast<u32x4_t*>(&lds[0][row][c]) = h;
            *reinterpret_cast<u32x4_t*>(&lds[1][row][c]) = m;
            *reinterpret_cast<u32x4_t*>(&lds[2][row][c]) = l;
        }
    }
}

// B operand given pre-split (BPRE): three bf16 planes [3][rows][ldbp] (k contiguous; rows padded to a
// multiple of 128 and ldbp a multiple of 64, zero filled), plane stride g.bplane elements.  A
// weight matrix is reused by every row tile of a minibatch, so it is split once per minibatch
// (split_weight) instead of once per tile and stage.  Per thread and stage: XK / 16 16-byte chunks
// per plane (row e / KG, chunk e % KG of 8 bf16).
template <int XK, int NP>
DEV void xp_load(u32x4_t (&v)[NP][XK / 16], const uint16_t* B, int64_t ldb, int64_t plane, int j0, int k0, int ke) {
    constexpr int KG = XK / 8;
#pragma unroll
    for (int q = 0; q < XK / 16; q++) {
        const int e = threadIdx.x + 256 * q;
        const int64_t off = (int64_t)(j0 + e / KG) * ldb + k0 + (e % KG) * 8;
        const bool ok = k0 + (e % KG) * 8 < ke;
#pragma unroll
        for (int p = 0; p < NP; p++)
            v[p][q] = *reinterpret_cast<const u32x4_t*>(ok ? B + p * plane + off : reinterpret_cast<const uint16_t*>(g_zero_row));
    }
}
template <int XK, int NP, int P = XK + XPAD>
DEV void xp_store(uint16_t (*lds)[BM][P], const u32x4_t (&v)[NP][XK / 16]) {
    constexpr int KG = XK / 8;
#pragma unroll
    for (int q = 0; q < XK / 16; q++) {
        const int e = threadIdx.x + 256 * q;
        const int c = xchunk<P, XK>(e / KG, e % KG) * 8;
#pragma unroll
        for (int p = 0; p < NP; p++) *reinterpret_cast<u32x4_t*>(&lds[p][e / KG][c]) = v[p][q];
    }
}

// W [out][in] f32 -> three bf16 planes of W (trans = 0: [out_pad][in_pad]) or W^T (trans = 1:
// [in_pad][out_pad]), zero padded; one thread per padded element.
__global__ void split_weight(const float* W, int out, int in, int trans, int rows_pad, int ld_pad, uint16_t* planes) {
    const int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const int64_t plane = (int64_t)rows_pad * ld_pad;
    if (e >= plane) return;
    const int r = (int)(e / ld_pad), c = (int)(e % ld_pad);
    const int o = trans ? c : r, i = trans ? r : c;
    const float x = (o < out && i < in) ? W[(int64_t)o * in + i] : 0.f;
    const uint16_t h = f2bf(x);
    const float r1 = x - bf2f(h);
    const uint16_t m = f2bf(r1);
    planes[e] = h;
    planes[plane + e] = m;
    planes[2 * plane + e] = f2bf(r1 - bf2f(m));
}

// H3: W [out][in] (row stride ldw) f32 -> two scaled fp16 planes of W (trans = 0: rows = out, k = in) or W^T
// (trans = 1: rows = in, k = out), zero padded, one scale per plane row: the 256-thread block of
// row r finds max |W| over the row's k, then writes x * 2^p split into (h, l) and inv[r] = 2^-p.
__global__ void __launch_bounds__(256) split_weight_h3(const float* W, int out, int in, int64_t ldw, int trans, int ld_pad,
                                                      uint16_t* planes, int64_t plane, float* inv) {
    __shared__ uint32_t red[4];
    const int r = blockIdx.x;
    const int nk = trans ? out : in, nr = trans ? in : out;
    auto at = [&](int k) -> float {  // W element (o, i) at W[o * ldw + i]
        if (r >= nr || k >= nk) return 0.f;
        return trans ? W[(int64_t)k * ldw + r] : W[(int64_t)r * ldw + k];
    };
    uint32_t m = 0;
    for (int k = threadIdx.x; k < nk; k += 256) {
        const uint32_t b = abs_bits(at(k));
        m = b > m ? b : m;
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
        const uint32_t u = (uint32_t)__shfl_xor((int)m, o, 64);
        m = u > m ? u : m;
    }
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = m;
    __syncthreads();
    m = red[0];
    for (int w = 1; w < 4; w++) m = red[w] > m ? red[w] : m;
    const int p = h3_pow(m);
    const float sc = pow2f(p);
    for (int k = threadIdx.x; k < ld_pad; k += 256) {
        const float x = at(k) * sc;
        const uint16_t h = f2hf(x);
        planes[(int64_t)r * ld_pad + k] = h;
        planes[plane + (int64_t)r * ld_pad + k] = f2hf(x - hf2f(h));
    }
    if (threadIdx.x == 0) inv[r] = pow2f(-p);
}

// max |x| over a [rows][cols] f32 matrix (row stride ld) into 64 shards: the stand-alone producer
// for callers of the H3 GEMM whose operand has no producer kernel of ours (rlgpu_gemm, tests)
__global__ void __launch_bounds__(256) amax_rows(const float* X, int64_t rows, int cols, int64_t ld, float* shards) {
    uint32_t m = 0;
    const int64_t n = rows * cols;
    for (int64_t e = (int64_t)blockIdx.x * 256 + threadIdx.x; e < n; e += (int64_t)gridDim.x * 256) {
        const uint32_t b = abs_bits(X[(e / cols) * ld + e % cols]);
        m = b > m ? b : m;
    }
    h3_amax_commit(shards, m);
}

// gemm_x6's pipeline: 32-deep stages, one LDS buffer, the next stage prefetched into registers while this
// stage's MFMAs run; two (x6) or three (H3: 146 VGPRs, 40 KB LDS) workgroups per CU.
template <int XK>
DEV void x6_mfma_stage(const uint16_t (*As)[BM][XK + XPAD], const uint16_t (*Bs)[BN][XK + XPAD], int ra, int rb, int lane,
                       f32x16 (&acc)[2][2], f32x16 (&cor)[2][2]) {
#pragma unroll
    for (int ks = 0; ks < XK / 16; ks++) {
        const int kof = ks * 16 + 8 * (lane >> 5);
        bf16x8 a[3][2], b[3][2];
#pragma unroll
        for (int p = 0; p < 3; p++)
#pragma unroll
            for (int u = 0; u < 2; u++) {
                a[p][u] = *(const bf16x8*)&As[p][ra + 32 * u][kof];
                b[p][u] = *(const bf16x8*)&Bs[p][rb + 32 * u][kof];
            }
#pragma unroll
        for (int ti = 0; ti < 2; ti++)
#pragma unroll
            for (int tj = 0; tj < 2; tj++) {
                f32x16 c = cor[ti][tj];
                c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[1][ti], b[1][tj], c, 0, 0, 0);  // m m
                c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[2][ti], b[0][tj], c, 0, 0, 0);  // l h
                c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[0][ti], b[2][tj], c, 0, 0, 0);  // h l
                c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[1][ti], b[0][tj], c, 0, 0, 0);  // m h
                c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[0][ti], b[1][tj], c, 0, 0, 0);  // h m
                cor[ti][tj] = c;
                acc[ti][tj] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[0][ti], b[0][tj], acc[ti][tj], 0, 0, 0);
            }
    }
}

typedef _Float16 h16x8 __attribute__((ext_vector_type(8)));

// ---- k-major ("T") staging of a row-index-contiguous operand (H3, 32-deep stages): A_KI (dZ^T)
// and B_KJ (activations) of the weight gradients.  Global rows are k, contiguous in the output
// index o, so each thread loads float4s along o (coalesced 512-byte rows per half wave, no scalar
// gathers) and stores each plane k-major: element (k, o) at k * TPITCH + o of the plane (the
// plane's [BM][XK + XPAD] storage, same size).  The MFMA fragments (8 consecutive k of one o per
// lane) are read back transposed with ds_read_b64_tr_b16: per 16-lane group a 4 (k) x 16 (o)
// block, lane 4q+p addressing row q, columns 4p..4p+3; two reads give k .. k+7.  TPITCH = 160
// halves puts the 4 rows of a 32-lane half at bank offsets 0 / 16 / 32 / 48: conflict-free.
constexpr int TPITCH = 160;
static_assert(32 * TPITCH == BM * (32 + XPAD), "k-major plane must fit the row-major plane storage");
typedef short v4i16 __attribute__((ext_vector_type(4)));
template <bool VEC>
DEV void xt_load(f32x4_t (&v)[2][2], const float* base, int64_t ld, int o0, int on, int k0, int ke) {
#pragma unroll
    for (int q = 0; q < 4; q++) {
        const int e = threadIdx.x + 256 * q;
        const int k = k0 + (e >> 5), o = o0 + (e & 31) * 4;
        const float* row = k < ke ? base + (int64_t)k * ld : nullptr;
        v[q >> 1][q & 1] = load4v<VEC>(row, o, on);
    }
}
DEV void xt_store(uint16_t (*lds)[BM][32 + XPAD], const f32x4_t (&v)[2][2], float sc) {
    uint16_t* ph = &lds[0][0][0];
    uint16_t* pl = &lds[1][0][0];
#pragma unroll
    for (int q = 0; q < 4; q++) {
        const int e = threadIdx.x + 256 * q;
        const int off = (e >> 5) * TPITCH + (e & 31) * 4;
        const f32x4_t x = v[q >> 1][q & 1];
        uint32_t h2[2], l2[2];
#pragma unroll
        for (int c = 0; c < 2; c++) {
            const float x0 = x[2 * c] * sc, x1 = x[2 * c + 1] * sc;
            const uint16_t h0 = f2hf(x0), h1 = f2hf(x1);
            h2[c] = pack_h2(h0, h1);
            l2[c] = pack_h2(f2hf(x0 - hf2f(h0)), f2hf(x1 - hf2f(h1)));
        }
        *reinterpret_cast<uint2*>(ph + off) = make_uint2(h2[0], h2[1]);
        *reinterpret_cast<uint2*>(pl + off) = make_uint2(l2[0], l2[1]);
    }
}
// the 32x32x16 operand fragment of output rows ob .. ob+31 at k = kof0 + 8 (lane >> 5) + 0..7
DEV h16x8 tr_frag(const uint16_t* plane, int ob, int kof0, int lane) {
    const int g = lane >> 4, i = lane & 15;
    const int o = ob + 16 * (g & 1) + 4 * (i & 3);
    const int k = kof0 + 8 * (g >> 1) + (i >> 2);
    typedef __attribute__((address_space(3))) v4i16 lds_v4i16;
    const v4i16 x = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_v4i16*)(plane + k * TPITCH + o));
    const v4i16 y = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_v4i16*)(plane + (k + 4) * TPITCH + o));
    typedef short v8i16 __attribute__((ext_vector_type(8)));
    const v8i16 r = {x[0], x[1], x[2], x[3], y[0], y[1], y[2], y[3]};
    return __builtin_bit_cast(h16x8, r);
}

template <int XK, bool TA = false, bool TB = false, int P = XK + XPAD>
DEV void h3_mfma_stage(const uint16_t (*As)[BM][P], const uint16_t (*Bs)[BN][P], int ra, int rb, int lane,
                       f32x16 (&acc)[2][2], f32x16 (&cor)[2][2]) {
#pragma unroll
    for (int ks = 0; ks < XK / 16; ks++) {
        const int kc = 2 * ks + (lane >> 5);  // logical 16-byte chunk of this lane's 8 k
        h16x8 a[2][2], b[2][2];
#pragma unroll
        for (int p = 0; p < 2; p++)
#pragma unroll
            for (int u = 0; u < 2; u++) {
                // ra / rb: this lane's row; (ra & ~31) the wave's 32-row block base
                a[p][u] = TA ? tr_frag(&As[p][0][0], (ra & ~31) + 32 * u, ks * 16, lane)
                             : *(const h16x8*)&As[p][ra + 32 * u][xchunk<P, XK>(ra + 32 * u, kc) * 8];
                b[p][u] = TB ? tr_frag(&Bs[p][0][0], (rb & ~31) + 32 * u, ks * 16, lane)
                             : *(const h16x8*)&Bs[p][rb + 32 * u][xchunk<P, XK>(rb + 32 * u, kc) * 8];
            }
        // one accumulator: the corrections, then the leading product, enter the running f32 sum (the
        // rounding count of an f32 FMA chain; a separate correction accumulator would cost 64
        // registers that the deeper stage uses instead)
#pragma unroll
        for (int ti = 0; ti < 2; ti++)
#pragma unroll
            for (int tj = 0; tj < 2; tj++) {
                f32x16 c = acc[ti][tj];
                c = __builtin_amdgcn_mfma_f32_32x32x16_f16(a[1][ti], b[0][tj], c, 0, 0, 0);  // l h
                c = __builtin_amdgcn_mfma_f32_32x32x16_f16(a[0][ti], b[1][tj], c, 0, 0, 0);  // h l
                acc[ti][tj] = __builtin_amdgcn_mfma_f32_32x32x16_f16(a[0][ti], b[0][tj], c, 0, 0, 0);  // h h
            }
    }
}

template <int LA, int LB, bool AV, bool BV, bool BPRE, bool H3 = false>
__global__ void __launch_bounds__(256, 2) gemm_x6(GemmArgs g) {
    constexpr int XK = 32, NB = 1, NQ = XK / 16, NP = H3 ? 2 : 3;
    constexpr bool AK = LA == A_IK, BKM = LB == B_JK;
    // H3 with 32-deep stages: row-index-contiguous operands staged k-major (xt_load / tr_frag)
    constexpr bool TA = H3 && !AK && XK == 32, TB = H3 && !BPRE && !BKM && XK == 32;
    // H3 with both operands k-contiguous, default variant: unpadded XOR-swizzled planes (xchunk)
    constexpr bool SWZ = H3 && !TA && !TB;
    constexpr int P = SWZ ? XK : XK + XPAD;
    __shared__ uint16_t As[NB][NP][BM][P];
    __shared__ uint16_t Bs[NB][NP][BN][P];
    const int t = threadIdx.x, lane = t & 63, w = t >> 6;
    const int wm = w >> 1, wn = w & 1;
    const Tile tl = xcd_tile(g.gx, g.gy, g.gz);
    const int i0 = tl.y * BM, j0 = tl.x * BN;
    const int kb = tl.z * g.kchunk;
    const int ke = min(g.K, kb + g.kchunk);
    f32x16 acc[2][2], cor[2][2];
#pragma unroll
    for (int a = 0; a < 2; a++)
#pragma unroll
        for (int b = 0; b < 2; b++)
#pragma unroll
            for (int r = 0; r < 16; r++) acc[a][b][r] = cor[a][b][r] = 0.f;
    f32x4_t va[NQ][2], vb[NQ][2];
    u32x4_t vp[NP][NQ];
    const uint16_t* Bp = reinterpret_cast<const uint16_t*>(g.B);
    // H3 operand scales (per tensor; a pre-split B carries per-row scales instead)
    int pa = 0, pb = 0;
    if (H3) {
        pa = h3_pow(shard_max_bits(g.amax_a));
        if (!BPRE) pb = h3_pow(shard_max_bits(g.amax_b));
    }
    const float sa = pow2f(pa), sb = pow2f(pb);
    const RowPtrs arow = xs_rows<AK, XK>(g.A, g.lda, i0, g.I);
    const RowPtrs brow = xs_rows<BKM, XK>(g.B, g.ldb, j0, g.J);
    auto load_stage = [&](int k0) {
        if constexpr (TA)
            xt_load<AV>(va, g.A, g.lda, i0, g.I, k0, ke);
        else
            xs_load<AK, AV, XK>(va, arow, g.A, g.lda, i0, g.I, k0, ke);
        if (BPRE)
            xp_load<XK, NP>(vp, Bp, g.ldb, g.bplane, j0, k0, ke);
        else if constexpr (TB)
            xt_load<BV>(vb, g.B, g.ldb, j0, g.J, k0, ke);
        else
            xs_load<BKM, BV, XK>(vb, brow, g.B, g.ldb, j0, g.J, k0, ke);
    };
    const int ra = wm * 64 + (lane & 31), rb = wn * 64 + (lane & 31);
    auto store_stage = [&](int buf) {
        if constexpr (TA)
            xt_store(As[buf], va, sa);
        else
            xs_store<AK, XK, H3, P>(As[buf], va, sa);
        if (BPRE)
            xp_store<XK, NP, P>(Bs[buf], vp);
        else if constexpr (TB)
            xt_store(Bs[buf], vb, sb);
        else
            xs_store<BKM, XK, H3, P>(Bs[buf], vb, sb);
    };
    auto mfma_stage = [&](int buf) {
        if constexpr (H3)
            h3_mfma_stage<XK, TA, TB, P>(As[buf], Bs[buf], ra, rb, lane, acc, cor);
        else
            x6_mfma_stage<XK>(As[buf], Bs[buf], ra, rb, lane, acc, cor);
    };
    load_stage(kb);
    for (int k0 = kb; k0 < ke; k0 += XK) {
        store_stage(0);
        __syncthreads();
        // prefetch the next stage into registers while the MFMAs run; unconditional (past ke it
        // reads the zero row) so the loop-carried registers are the load destinations
        load_stage(k0 + XK);
        __builtin_amdgcn_sched_barrier(0);  // keep the split of the prefetched stage after the MFMAs
        mfma_stage(0);
        __syncthreads();
    }
    float* C = g.C + (int64_t)tl.z * g.c_split;
    const int h = lane >> 5, l32 = lane & 31;
    // H3: undo the operand scales (powers of two: exact); the pre-split B's per-row inverse scale
    // is read for the tile's columns (rows past J carry 1)
    const int pab = pa + pb;
    float csc[2];
#pragma unroll
    for (int tj = 0; tj < 2; tj++) csc[tj] = (H3 && BPRE) ? g.bscale[j0 + wn * 64 + tj * 32 + l32] : 1.f;
    if (i0 + BM <= g.I && j0 + BN <= g.J) {  // interior tile: no bounds checks, one base pointer
        float* cb = C + (int64_t)(i0 + wm * 64 + 4 * h) * g.ldc + j0 + wn * 64 + l32;
#pragma unroll
        for (int ti = 0; ti < 2; ti++)
#pragma unroll
            for (int tj = 0; tj < 2; tj++) {
                const float bj = g.bias ? g.bias[j0 + wn * 64 + tj * 32 + l32] : 0.f;
                float* ct = cb + (int64_t)(ti * 32) * g.ldc + tj * 32;
#pragma unroll
                for (int r = 0; r < 16; r++) {
                    const float v = acc[ti][tj][r] + cor[ti][tj][r];
                    ct[(int64_t)((r & 3) + 8 * (r >> 2)) * g.ldc] = (H3 ? ldexpf(v * csc[tj], -pab) : v) + bj;
                }
            }
        return;
    }
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
                const float v = acc[ti][tj][r] + cor[ti][tj][r];
                if (i < g.I) C[(int64_t)i * g.ldc + j] = (H3 ? ldexpf(v * csc[tj], -pab) : v) + bj;
            }
        }
}

// weight planes are padded to whole 256-row blocks (the 256 x 256 tiles of gemm_h3q / gemm_h3qt)
constexpr int BNW = 2 * BN;
// tr_frag over a k-major plane of row pitch P halves (P = COLS + 32: conflict-free, see TPITCH)
template <int P>
DEV h16x8 trp_frag(const uint16_t* plane, int ob, int kof0, int lane) {
    const int g = lane >> 4, i = lane & 15;
    const int o = ob + 16 * (g & 1) + 4 * (i & 3);
    const int k = kof0 + 8 * (g >> 1) + (i >> 2);
    typedef __attribute__((address_space(3))) v4i16 lds_v4i16;
    const v4i16 x = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_v4i16*)(plane + k * P + o));
    const v4i16 y = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_v4i16*)(plane + (k + 4) * P + o));
    typedef short v8i16 __attribute__((ext_vector_type(8)));
    const v8i16 r = {x[0], x[1], x[2], x[3], y[0], y[1], y[2], y[3]};
    return __builtin_bit_cast(h16x8, r);
}

// ---- H3 GEMM with 256 x 256 tiles (gemm_h3q): the forward and input-gradient GEMMs (A_IK fp32 x the
// pre-split fp16 B planes, J a multiple of 256).  The 128 x 128 tile reads 32 KB from L2 per 128 x 128 x 32
// stage; at ~70 GB/s of L2 per CU (MI355X_MICROARCH.md, "Indexed rows") three such workgroups per CU need
// more feed cycles than their MFMAs take, so the stage skeleton, not the matrix pipe, sets gemm_x6's time.
// A 256 x 256 tile halves the L2 bytes per product.  8 waves (512 threads, one workgroup per CU, two waves
// per SIMD), each 64 x 128 (2 x 4 MFMA blocks); double-buffered LDS (2 x 64 KB) with one barrier per stage:
// this stage's MFMAs run on one buffer while the next stage (in registers since the previous iteration)
// is split into the other and the stage after is loaded.  Per 16-deep k step and block the products enter
// the one accumulator as l.h, h.l, h.h -- gemm_x6's H3 order -- so the results are bit-identical to it.
constexpr int BQ = 256;
template <bool AV>
__global__ void __launch_bounds__(512, 1) gemm_h3q(GemmArgs g) {
    constexpr int XK = 32, KG = XK / 8;
    __shared__ uint16_t As[2][2][BQ][XK];  // [buffer][plane][row][k], 16-byte chunks XOR-swizzled (xchunk)
    __shared__ uint16_t Bs[2][2][BQ][XK];
    const int t = threadIdx.x, lane = t & 63, w = t >> 6;
    const int wm = w >> 1, wn = w & 1;
    const Tile tl = xcd_tile(g.gx, g.gy, 1);
    const int i0 = tl.y * BQ, j0 = tl.x * BQ;
    const int ke = g.K;
    f32x16 acc[2][4];
#pragma unroll
    for (int a = 0; a < 2; a++)
#pragma unroll
        for (int b = 0; b < 4; b++)
#pragma unroll
            for (int r = 0; r < 16; r++) acc[a][b][r] = 0.f;
    // this thread's share of a stage: A groups e = t + 512 q (row e / KG, k group e % KG), 8 floats each;
    // B chunks of the same (row, k group) in both planes
    const float* arow[2];
#pragma unroll
    for (int q = 0; q < 2; q++) {
        const int gi = i0 + (t + 512 * q) / KG;
        arow[q] = gi < g.I ? g.A + (int64_t)gi * g.lda : nullptr;
    }
    const int kg = t % KG;
    f32x4_t va[2][2];
    u32x4_t vp[2][2];
    const uint16_t* Bp = reinterpret_cast<const uint16_t*>(g.B);
    const int pa = h3_pow(shard_max_bits(g.amax_a));
    const float sa = pow2f(pa);
    auto load_stage = [&](int k0) {
        const int kk = k0 + kg * 8;
        const bool ok = kk < ke;
#pragma unroll
        for (int q = 0; q < 2; q++) {
            va[q][0] = load4v<AV>(arow[q], kk, ke);
            va[q][1] = load4v<AV>(arow[q], kk + 4, ke);
            const int64_t off = (int64_t)(j0 + (t + 512 * q) / KG) * g.ldb + kk;
#pragma unroll
            for (int p = 0; p < 2; p++)
                vp[p][q] = *reinterpret_cast<const u32x4_t*>(ok ? Bp + p * g.bplane + off
                                                               : reinterpret_cast<const uint16_t*>(g_zero_row));
        }
    };
    auto store_stage = [&](int buf) {
#pragma unroll
        for (int q = 0; q < 2; q++) {
            const int row = (t + 512 * q) / KG, c = xchunk<XK, XK>(row, kg) * 8;
            u32x4_t h, l;
            split2h(va[q], sa, h, l);
            *reinterpret_cast<u32x4_t*>(&As[buf][0][row][c]) = h;
            *reinterpret_cast<u32x4_t*>(&As[buf][1][row][c]) = l;
#pragma unroll
            for (int p = 0; p < 2; p++) *reinterpret_cast<u32x4_t*>(&Bs[buf][p][row][c]) = vp[p][q];
        }
    };
    const int ra = wm * 64 + (lane & 31), rb = wn * 128 + (lane & 31);
    auto mfma_stage = [&](int buf) {
#pragma unroll
        for (int ks = 0; ks < XK / 16; ks++) {
            const int kc = 2 * ks + (lane >> 5);
            h16x8 a[2][2], b[2][4];
#pragma unroll
            for (int p = 0; p < 2; p++) {
#pragma unroll
                for (int u = 0; u < 2; u++)
                    a[p][u] = *(const h16x8*)&As[buf][p][ra + 32 * u][xchunk<XK, XK>(ra + 32 * u, kc) * 8];
#pragma unroll
                for (int u = 0; u < 4; u++)
                    b[p][u] = *(const h16x8*)&Bs[buf][p][rb + 32 * u][xchunk<XK, XK>(rb + 32 * u, kc) * 8];
            }
#pragma unroll
            for (int ti = 0; ti < 2; ti++)
#pragma unroll
                for (int tj = 0; tj < 4; tj++) {
                    f32x16 c = acc[ti][tj];
                    c = __builtin_amdgcn_mfma_f32_32x32x16_f16(a[1][ti], b[0][tj], c, 0, 0, 0);  // l h
                    c = __builtin_amdgcn_mfma_f32_32x32x16_f16(a[0][ti], b[1][tj], c, 0, 0, 0);  // h l
                    acc[ti][tj] = __builtin_amdgcn_mfma_f32_32x32x16_f16(a[0][ti], b[0][tj], c, 0, 0, 0);  // h h
                }
        }
    };
    load_stage(0);
    store_stage(0);
    __syncthreads();
    load_stage(XK);  // unconditional: past K it reads the zero row
    int buf = 0;
    for (int k0 = 0; k0 < ke; k0 += XK) {
        mfma_stage(buf);
        store_stage(buf ^ 1);
        load_stage(k0 + 2 * XK);
        __syncthreads();
        buf ^= 1;
    }
    const int h = lane >> 5, l32 = lane & 31;
#pragma unroll
    for (int tj = 0; tj < 4; tj++) {
        const int j = j0 + wn * 128 + tj * 32 + l32;
        const float bsc = g.bscale[j];
        const float bj = g.bias ? g.bias[j] : 0.f;
#pragma unroll
        for (int ti = 0; ti < 2; ti++)
#pragma unroll
            for (int r = 0; r < 16; r++) {
                const int i = i0 + wm * 64 + ti * 32 + (r & 3) + 8 * (r >> 2) + 4 * h;
                if (i < g.I) g.C[(int64_t)i * g.ldc + j] = ldexpf(acc[ti][tj][r] * bsc, -pa) + bj;
            }
    }
}

// ---- gemm_h3q's weight-gradient form (gemm_h3qt): A_KI (dZ^T) x B_KJ (activations), both row-index
// contiguous, staged k-major (float4 loads along the output index, planes [k][256 + 32],
// fragments read back with ds_read_b64_tr_b16); split-K over grid z like the other kernels.  Same products in
// the same order per split as gemm_x6: bit-identical partials.
template <bool VEC>
DEV void q_kload(f32x4_t (&v)[4], const float* base, int64_t ld, int o0, int on, int k0, int ke) {
#pragma unroll
    for (int q = 0; q < 4; q++) {  // element group e = t + 512 q: k row e / 64, float4 e % 64 of the 256 columns
        const int e = (int)threadIdx.x + 512 * q;
        const int k = k0 + e / 64, o = o0 + (e % 64) * 4;
        const float* row = k < ke ? base + (int64_t)k * ld : nullptr;
        v[q] = load4v<VEC>(row, o, on);
    }
}
DEV void q_kstore(uint16_t* ph, uint16_t* pl, const f32x4_t (&v)[4], float sc) {
    constexpr int P = BQ + 32;
#pragma unroll
    for (int q = 0; q < 4; q++) {
        const int e = (int)threadIdx.x + 512 * q;
        const int off = (e / 64) * P + (e % 64) * 4;
        uint32_t h2[2], l2[2];
#pragma unroll
        for (int c = 0; c < 2; c++) {
            const float x0 = v[q][2 * c] * sc, x1 = v[q][2 * c + 1] * sc;
            const uint16_t h0 = f2hf(x0), h1 = f2hf(x1);
            h2[c] = pack_h2(h0, h1);
            l2[c] = pack_h2(f2hf(x0 - hf2f(h0)), f2hf(x1 - hf2f(h1)));
        }
        *reinterpret_cast<uint2*>(ph + off) = make_uint2(h2[0], h2[1]);
        *reinterpret_cast<uint2*>(pl + off) = make_uint2(l2[0], l2[1]);
    }
}
template <bool AV, bool BV>
__global__ void __launch_bounds__(512, 1) gemm_h3qt(GemmArgs g) {
    constexpr int XK = 32, P = BQ + 32;
    __shared__ uint16_t As[2][2][XK * P];  // [buffer][plane][k][o]
    __shared__ uint16_t Bs[2][2][XK * P];
    const int t = threadIdx.x, lane = t & 63, w = t >> 6;
    const int wm = w >> 1, wn = w & 1;
    const Tile tl = xcd_tile(g.gx, g.gy, g.gz);
    const int i0 = tl.y * BQ, j0 = tl.x * BQ;
    const int kb = tl.z * g.kchunk;
    const int ke = min(g.K, kb + g.kchunk);
    f32x16 acc[2][4];
#pragma unroll
    for (int a = 0; a < 2; a++)
#pragma unroll
        for (int b = 0; b < 4; b++)
#pragma unroll
            for (int r = 0; r < 16; r++) acc[a][b][r] = 0.f;
    f32x4_t va[4], vb[4];
    const int pa = h3_pow(shard_max_bits(g.amax_a)), pb = h3_pow(shard_max_bits(g.amax_b));
    const float sa = pow2f(pa), sb = pow2f(pb);
    auto load_stage = [&](int k0) {
        q_kload<AV>(va, g.A, g.lda, i0, g.I, k0, ke);
        q_kload<BV>(vb, g.B, g.ldb, j0, g.J, k0, ke);
    };
    auto store_stage = [&](int buf) {
        q_kstore(&As[buf][0][0], &As[buf][1][0], va, sa);
        q_kstore(&Bs[buf][0][0], &Bs[buf][1][0], vb, sb);
    };
    auto mfma_stage = [&](int buf) {
#pragma unroll
        for (int ks = 0; ks < XK / 16; ks++) {
            h16x8 a[2][2], b[2][4];
#pragma unroll
            for (int p = 0; p < 2; p++) {
#pragma unroll
                for (int u = 0; u < 2; u++) a[p][u] = trp_frag<P>(&As[buf][p][0], wm * 64 + 32 * u, ks * 16, lane);
#pragma unroll
                for (int u = 0; u < 4; u++) b[p][u] = trp_frag<P>(&Bs[buf][p][0], wn * 128 + 32 * u, ks * 16, lane);
            }
#pragma unroll
            for (int ti = 0; ti < 2; ti++)
#pragma unroll
                for (int tj = 0; tj < 4; tj++) {
                    f32x16 c = acc[ti][tj];
                    c = __builtin_amdgcn_mfma_f32_32x32x16_f16(a[1][ti], b[0][tj], c, 0, 0, 0);  // l h
                    c = __builtin_amdgcn_mfma_f32_32x32x16_f16(a[0][ti], b[1][tj], c, 0, 0, 0);  // h l
                    acc[ti][tj] = __builtin_amdgcn_mfma_f32_32x32x16_f16(a[0][ti], b[0][tj], c, 0, 0, 0);  // h h
                }
        }
    };
    load_stage(kb);
    store_stage(0);
    __syncthreads();
    load_stage(kb + XK);  // unconditional: past ke it reads the zero row
    int buf = 0;
    for (int k0 = kb; k0 < ke; k0 += XK) {
        mfma_stage(buf);
        store_stage(buf ^ 1);
        load_stage(k0 + 2 * XK);
        __syncthreads();
        buf ^= 1;
    }
    float* C = g.C + (int64_t)tl.z * g.c_split;
    const int h = lane >> 5, l32 = lane & 31;
    const int pab = pa + pb;
#pragma unroll
    for (int tj = 0; tj < 4; tj++) {
        const int j = j0 + wn * 128 + tj * 32 + l32;
        if (j >= g.J) continue;
        const float bj = g.bias ? g.bias[j] : 0.f;
#pragma unroll
        for (int ti = 0; ti < 2; ti++)
#pragma unroll
            for (int r = 0; r < 16; r++) {
                const int i = i0 + wm * 64 + ti * 32 + (r & 3) + 8 * (r >> 2) + 4 * h;
                if (i < g.I) C[(int64_t)i * g.ldc + j] = ldexpf(acc[ti][tj][r] * 1.f, -pab) + bj;
            }
    }
}

// ---- bf16 inference GEMM: C[i,j] = bf16( sum_k A[i,k] W[j,k] + bias[j] ) on
// v_mfma_f32_32x32x16_bf16 (fp32 accumulate).  A [I][lda] and W [J][ldb] bf16, k contiguous,
// 16-byte aligned rows, K a multiple of 8 with zero padding (the padded inference copy of the
// weights and the converted obs), so every staging load is one uint4 of 8 bf16 per thread.
constexpr int HBK = 64, HPAD = 8;             // K per LDS stage: 16 MFMAs per wave between barriers
constexpr int HCH = HBK / 8;                   // 16-byte chunks per tile row
constexpr int HQ = BM * HCH / 256;             // uint4 per thread per operand tile

struct HGemmArgs {
    const uint16_t* A;      // [I][lda] bf16
    const uint16_t* B;      // [J][ldb] bf16
    const uint16_t* bias;   // [J] bf16 or null
    uint16_t* C;            // [I][ldc] bf16
    int64_t lda, ldb, ldc;
    int I, J, K;            // K multiple of 8
    int gx, gy;             // logical tile grid; launched as 1-D (xcd_tile)
};

__device__ uint4 g_zero_u4[4];

// HQ 16-byte vectors per thread: row (t + 256q) / HCH, 8-element column chunk ((t + 256q) % HCH) * 8
typedef unsigned u32x4 __attribute__((ext_vector_type(4)));  // native vector: stays in VGPRs
DEV void htile_load(u32x4 (&r)[HQ], const uint16_t* const (&rows)[HQ], int k0, int K) {
#pragma unroll
    for (int q = 0; q < HQ; q++) {
        int c = k0 + ((threadIdx.x + 256 * q) % HCH) * 8;
        const uint16_t* p = (rows[q] && c < K) ? rows[q] + c : reinterpret_cast<const uint16_t*>(g_zero_u4);
        r[q] = *reinterpret_cast<const u32x4*>(p);
    }
}
DEV void htile_store(uint16_t (*lds)[HBK + HPAD], const u32x4 (&r)[HQ]) {
#pragma unroll
    for (int q = 0; q < HQ; q++) {
        int e = threadIdx.x + 256 * q;
        *reinterpret_cast<u32x4*>(&lds[e / HCH][(e % HCH) * 8]) = r[q];
    }
}

typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));
template <bool F16>
DEV f32x16 mfma16(bf16x8 a, bf16x8 b, f32x16 c) {
    if constexpr (F16)
        return __builtin_amdgcn_mfma_f32_32x32x16_f16(__builtin_bit_cast(f16x8, a), __builtin_bit_cast(f16x8, b), c, 0, 0, 0);
    else
        return __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c, 0, 0, 0);
}
template <bool F16>
__global__ void __launch_bounds__(256, 2) gemm_bf16(HGemmArgs g) {
    __shared__ uint16_t As[BM][HBK + HPAD];
    __shared__ uint16_t Bs[BN][HBK + HPAD];
    const int t = threadIdx.x, lane = t & 63, w = t >> 6;
    const int wm = w >> 1, wn = w & 1;
    const Tile tl = xcd_tile(g.gx, g.gy, 1);
    const int i0 = tl.y * BM, j0 = tl.x * BN;
    const uint16_t* arow[HQ];
    const uint16_t* brow[HQ];
#pragma unroll
    for (int q = 0; q < HQ; q++) {
        int rr = (t + 256 * q) / HCH;
        arow[q] = i0 + rr < g.I ? g.A + (int64_t)(i0 + rr) * g.lda : nullptr;
        brow[q] = j0 + rr < g.J ? g.B + (int64_t)(j0 + rr) * g.ldb : nullptr;
    }
    f32x16 acc[2][2];
    for (int a = 0; a < 2; a++)
        for (int b = 0; b < 2; b++)
            for (int r = 0; r < 16; r++) acc[a][b][r] = 0.f;
    u32x4 ra[HQ], rb[HQ];
    htile_load(ra, arow, 0, g.K);
    htile_load(rb, brow, 0, g.K);
    for (int k0 = 0; k0 < g.K; k0 += HBK) {
        htile_store(As, ra);
        htile_store(Bs, rb);
        __syncthreads();
        if (k0 + HBK < g.K) {
            htile_load(ra, arow, k0 + HBK, g.K);
            htile_load(rb, brow, k0 + HBK, g.K);
        }
#pragma unroll
        for (int ks = 0; ks < HBK / 16; ks++) {
            int kof = ks * 16 + 8 * (lane >> 5);
            bf16x8 a0 = *(const bf16x8*)&As[wm * 64 + (lane & 31)][kof];
            bf16x8 a1 = *(const bf16x8*)&As[wm * 64 + 32 + (lane & 31)][kof];
            bf16x8 b0 = *(const bf16x8*)&Bs[wn * 64 + (lane & 31)][kof];
            bf16x8 b1 = *(const bf16x8*)&Bs[wn * 64 + 32 + (lane & 31)][kof];
            acc[0][0] = mfma16<F16>(a0, b0, acc[0][0]);
            acc[0][1] = mfma16<F16>(a0, b1, acc[0][1]);
            acc[1][0] = mfma16<F16>(a1, b0, acc[1][0]);
            acc[1][1] = mfma16<F16>(a1, b1, acc[1][1]);
        }
        __syncthreads();
    }
#pragma unroll
    for (int ti = 0; ti < 2; ti++)
#pragma unroll
        for (int tj = 0; tj < 2; tj++) {
            int j = j0 + wn * 64 + tj * 32 + (lane & 31);
            if (j >= g.J) continue;
            float bj = g.bias ? h2f<F16>(g.bias[j]) : 0.f;
#pragma unroll
            for (int r = 0; r < 16; r++) {
                int i = i0 + wm * 64 + ti * 32 + (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5);
                if (i < g.I) g.C[(int64_t)i * g.ldc + j] = f2h<F16>(acc[ti][tj][r] + bj);
            }
        }
}

// f32 rows [n][C] -> bf16 rows [n][ldx] (zero padded): the inference input of the first layer
template <bool F16>
__global__ void rows_to_bf16(const float* src, int C, int n, uint16_t* X, int ldx) {
    int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (e >= (int64_t)n * ldx) return;
    int r = (int)(e / ldx), c = (int)(e % ldx);
    X[e] = c < C ? f2h<F16>(src[(int64_t)r * C + c]) : (uint16_t)0;
}

// fp32 Linear.weight [out][in] -> padded bf16 [out][ldp] (zeros past in)
template <bool F16>
__global__ void weight_to_bf16(const float* w, int out, int in, uint16_t* h, int ldp) {
    int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (e >= (int64_t)out * ldp) return;
    int o = (int)(e / ldp), k = (int)(e % ldp);
    h[e] = k < in ? f2h<F16>(w[(int64_t)o * in + k]) : (uint16_t)0;
}

// out[e] (+)= sum_s part[s*stride + e], fixed order (deterministic split-K reduction)
// Minibatch gather (ExperienceBuffer::_GetSamples index_select, ExperienceBuffer.cpp:140-163):
// X[r, 0..C) = src[idx[start + r], 0..C), rows padded to ldx (16-byte aligned) with zeros.
// amax (optional): 64 shards of max |X| for the H3 training GEMMs (h3_amax_commit).
// Grid-stride (launch at most GATHER_BLOCKS blocks) so that the per-block max commits stay few.
constexpr int GATHER_BLOCKS = 2048;
__global__ void __launch_bounds__(256) gather_rows(const float* src, int C, const int32_t* idx, int64_t start, int n, float* X,
                                                  int ldx, float* amax) {
    uint32_t m = 0;
    const int64_t total = (int64_t)n * ldx;
    for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < total; e += (int64_t)gridDim.x * blockDim.x) {
        int r = (int)(e / ldx), c = (int)(e % ldx);
        int64_t s = idx ? (int64_t)idx[start + r] : start + r;
        const float v = c < C ? src[s * C + c] : 0.f;
        X[e] = v;
        const uint32_t b = abs_bits(v);
        m = b > m ? b : m;
    }
    if (amax) h3_amax_commit(amax, m);
}

__global__ void reduce_splits(const float* part, int splits, int64_t stride, int64_t n, float* out, int accumulate) {
    int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (e >= n) return;
    float s = 0.f;
    for (int k = 0; k < splits; k++) s += part[k * stride + e];
    out[e] = accumulate ? out[e] + s : s;
}
// the same sums, 4 columns per thread (n, stride multiples of 4, 16-byte aligned pointers); the
// split loop is unrolled so several partial loads are in flight
__global__ void reduce_splits4(const float* part, int splits, int64_t stride, int64_t n, float* out, int accumulate) {
    int64_t e = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) * 4;
    if (e >= n) return;
    float4 s = make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll 4
    for (int k = 0; k < splits; k++) {
        float4 v = *reinterpret_cast<const float4*>(part + k * stride + e);
        s.x += v.x;
        s.y += v.y;
        s.z += v.z;
        s.w += v.w;
    }
    float4* o = reinterpret_cast<float4*>(out + e);
    if (accumulate) {
        float4 v = *o;
        s = make_float4(v.x + s.x, v.y + s.y, v.z + s.z, v.w + s.w);
    }
    *o = s;
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
// The same butterflies without the LDS crossbar: the xor-32 / xor-16 exchanges by
// v_permlane32_swap / v_permlane16_swap (both halves of the swap are summed, own + partner in either
// order), xor 8 / 4 / 2 / 1 by DPP row_ror 8 / 4 / 2 / 1 -- after the wider steps a lane's value
// depends only on its index modulo twice the distance, where the rotation reaches the xor partner.
// Every lane combines the same two partial values as in wave_sum / wave_max, so the results are
// bit-identical.
DEV float xchg32_sum(float v, bool mx) {
    auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(v), __float_as_uint(v), false, false);
    const float a = __uint_as_float(r[0]), b = __uint_as_float(r[1]);
    return mx ? fmaxf(a, b) : a + b;
}
DEV float xchg16_sum(float v, bool mx) {
    auto r = __builtin_amdgcn_permlane16_swap(__float_as_uint(v), __float_as_uint(v), false, false);
    const float a = __uint_as_float(r[0]), b = __uint_as_float(r[1]);
    return mx ? fmaxf(a, b) : a + b;
}
template <int CTRL>
DEV float dpp_f(float v) { return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), CTRL, 0xF, 0xF, false)); }
DEV float wave_sum_x(float v) {
    v = xchg32_sum(v, false);
    v = xchg16_sum(v, false);
    v += dpp_f<0x128>(v);
    v += dpp_f<0x124>(v);
    v += dpp_f<0x122>(v);
    v += dpp_f<0x121>(v);
    return v;
}
DEV float wave_max_x(float v) {
    v = xchg32_sum(v, true);
    v = xchg16_sum(v, true);
    v = fmaxf(v, dpp_f<0x128>(v));
    v = fmaxf(v, dpp_f<0x124>(v));
    v = fmaxf(v, dpp_f<0x122>(v));
    v = fmaxf(v, dpp_f<0x121>(v));
    return v;
}


// Column ownership of the wave-per-row kernels: with MAXH >= 4 columns per lane, lane l owns the
// 4-column groups starting at 4 l + 256 q (q < MAXH / 4), so every 16-byte load / store instruction
// of a wave covers one contiguous 1 KB span of the row (full 128-byte lines, no half-line writes);
// MAXH < 4 (H <= 128): the contiguous columns [MAXH l, MAXH l + MAXH).
template <int MAXH>
DEV int lcol(int lane, int q) {
    return MAXH >= 4 ? 4 * lane + 256 * (q >> 2) + (q & 3) : MAXH * lane + q;
}

// LayerNorm (eps 1e-5, biased variance) + LeakyReLU, training: one wave per row.
// Keeps act [R,H] and the row statistics stats [R] = (mean, rstd) for the backward, which
// recomputes xhat = (z - mean) * rstd from the untouched pre-norm input z with the same operations
// (bit-identical to a stored xhat, one [R,H] write less per layer).
// Columns per lane: lcol (float4 loads / stores when H is a multiple of 4); gamma / beta stay in
// registers.  Each wave walks LNF_ROWS/4 rows, lnf_rf<MAXH>() of them at a time: their loads are
// issued together before the first reduction and their wave reductions interleave, so a wave keeps
// that many rows of HBM traffic in flight (the per-row arithmetic and its order are unchanged).
// The rank-1 head (critic value) of one row already in registers, lcol layout: the arithmetic of
// head1_fwd (same per-lane order, same reduction), so fusing it into the LayerNorm forward that
// produces the row changes no bit; lane 0 writes *out.
template <int MAXH>
DEV void head1_row(const float (&x)[MAXH], const float* w, const float* b, int H, bool vec, int lane, float* out) {
    float s = 0.f;
    if (vec) {
#pragma unroll
        for (int q = 0; q < MAXH; q += 4) {
            const int c = lcol<MAXH>(lane, q);
            if (c < H) s += x[q] * w[c] + x[q + 1] * w[c + 1] + x[q + 2] * w[c + 2] + x[q + 3] * w[c + 3];
        }
    } else {
#pragma unroll
        for (int q = 0; q < MAXH; q++) {
            const int c = lcol<MAXH>(lane, q);
            if (c < H) s += x[q] * w[c];
        }
    }
    s = wave_sum(s);
    if (lane == 0) *out = s + b[0];
}

constexpr int LNF_ROWS = 16;
template <int MAXH>
constexpr int lnf_rf() {
    return MAXH <= 8 ? 4 : (MAXH <= 16 ? 2 : 1);
}
template <int MAXH, int ROWS = LNF_ROWS, int RFX = lnf_rf<MAXH>()>
__global__ void __launch_bounds__(256) ln_act_fwd_f32(const float* Z, const float* gamma, const float* beta, int R, int H,
                                                     float slope, int use_ln, float* act, float2* stats, float* amax,
                                                     const float* head_w = nullptr, const float* head_b = nullptr,
                                                     float* head_out = nullptr) {
    uint32_t vmax = 0;  // max |act| of this thread's outputs (H3 operand scale, when amax is given)
    const int wv = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const bool vec = (H % 4 == 0) && (MAXH % 4 == 0);
    float g[MAXH], b[MAXH];
#pragma unroll
    for (int q = 0; q < MAXH; q++) {
        const int c = lcol<MAXH>(lane, q);
        g[q] = (use_ln && c < H) ? gamma[c] : 1.f;
        b[q] = (use_ln && c < H) ? beta[c] : 0.f;
    }
    constexpr int RF = RFX;
    for (int i0 = 0; i0 < ROWS / 4; i0 += RF) {
        int row[RF];
        float v[RF][MAXH];
#pragma unroll
        for (int r = 0; r < RF; r++) {  // all RF rows' loads first (a row past R reloads row R-1)
            row[r] = blockIdx.x * ROWS + (i0 + r) * 4 + wv;
            const float* z = Z + (int64_t)min(row[r], R - 1) * H;
            if (vec) {
#pragma unroll
                for (int q = 0; q < MAXH; q += 4) {
                    const int c = lcol<MAXH>(lane, q);
                    float4 t = c < H ? *reinterpret_cast<const float4*>(z + c) : make_float4(0.f, 0.f, 0.f, 0.f);
                    v[r][q] = t.x; v[r][q + 1] = t.y; v[r][q + 2] = t.z; v[r][q + 3] = t.w;
                }
            } else {
#pragma unroll
                for (int q = 0; q < MAXH; q++) {
                    const int c = lcol<MAXH>(lane, q);
                    v[r][q] = c < H ? z[c] : 0.f;
                }
            }
        }
        float mean[RF], rs[RF];
#pragma unroll
        for (int r = 0; r < RF; r++) {
            mean[r] = 0.f;
            rs[r] = 1.f;
        }
        if (use_ln) {
#pragma unroll
            for (int r = 0; r < RF; r++) {
                float s = 0.f;
#pragma unroll
                for (int q = 0; q < MAXH; q++) s += v[r][q];
                mean[r] = wave_sum_x(s) / (float)H;
            }
#pragma unroll
            for (int r = 0; r < RF; r++) {
                float s2 = 0.f;
#pragma unroll
                for (int q = 0; q < MAXH; q++) {
                    float d = lcol<MAXH>(lane, q) < H ? v[r][q] - mean[r] : 0.f;
                    s2 += d * d;
                }
                rs[r] = 1.f / sqrtf(wave_sum_x(s2) / (float)H + 1e-5f);
            }
        }
#pragma unroll
        for (int r = 0; r < RF; r++) {
            if (row[r] >= R) continue;
            float a[MAXH];
#pragma unroll
            for (int q = 0; q < MAXH; q++) {
                const float xh = use_ln ? (v[r][q] - mean[r]) * rs[r] : v[r][q];
                const float hv = use_ln ? xh * g[q] + b[q] : xh;
                a[q] = hv > 0.f ? hv : hv * slope;
            }
            float* ao = act + (int64_t)row[r] * H;
            if (vec) {
#pragma unroll
                for (int q = 0; q < MAXH; q += 4) {
                    const int c = lcol<MAXH>(lane, q);
                    if (c < H) *reinterpret_cast<float4*>(ao + c) = make_float4(a[q], a[q + 1], a[q + 2], a[q + 3]);
                }
            } else {
#pragma unroll
                for (int q = 0; q < MAXH; q++) {
                    const int c = lcol<MAXH>(lane, q);
                    if (c < H) ao[c] = a[q];
                }
            }
            if (lane == 0) stats[row[r]] = make_float2(mean[r], rs[r]);
#pragma unroll
            for (int q = 0; q < MAXH; q++) {
                const uint32_t b = lcol<MAXH>(lane, q) < H ? abs_bits(a[q]) : 0u;
                vmax = b > vmax ? b : vmax;
            }
            if (head_w) head1_row<MAXH>(a, head_w, head_b, H, vec, lane, head_out + row[r]);
        }
    }
    if (amax) h3_amax_commit(amax, vmax);
}

// bf16 inference variant: Z bf16 in, bf16(LeakyReLU(bf16(LN(Z)))) out (torch bf16 module chain).
// With MAXH >= 8 columns per lane, lane l owns the 8-column groups at 8 l + 512 q (each 16-byte
// load / store instruction of a wave covers one contiguous 1 KB span); gamma / beta in registers;
// each wave walks LNF_ROWS/4 rows.
template <int MAXH>
DEV int hcol(int lane, int q) {
    return MAXH >= 8 ? 8 * lane + 512 * (q >> 3) + (q & 7) : MAXH * lane + q;
}
template <int MAXH, bool F16>
__global__ void __launch_bounds__(256) ln_act_fwd_bf16(const uint16_t* Z, const uint16_t* gamma, const uint16_t* beta, int R,
                                                      int H, float slope, int use_ln, uint16_t* out) {
    const int wv = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const bool vec = (H % 8 == 0) && (MAXH % 8 == 0);
    float g[MAXH], b[MAXH];
#pragma unroll
    for (int q = 0; q < MAXH; q++) {
        const int c = hcol<MAXH>(lane, q);
        g[q] = (use_ln && c < H) ? h2f<F16>(gamma[c]) : 1.f;
        b[q] = (use_ln && c < H) ? h2f<F16>(beta[c]) : 0.f;
    }
    for (int i = 0; i < LNF_ROWS / 4; i++) {
        const int row = blockIdx.x * LNF_ROWS + i * 4 + wv;
        if (row >= R) break;
        const uint16_t* z = Z + (int64_t)row * H;
        float v[MAXH];
        if (vec) {
#pragma unroll
            for (int q = 0; q < MAXH; q += 8) {
                const int c = hcol<MAXH>(lane, q);
                u32x4 t = {0u, 0u, 0u, 0u};
                if (c < H) t = *reinterpret_cast<const u32x4*>(z + c);
#pragma unroll
                for (int k = 0; k < 4; k++) {
                    v[q + 2 * k] = h2f<F16>((uint16_t)(t[k] & 0xffffu));
                    v[q + 2 * k + 1] = h2f<F16>((uint16_t)(t[k] >> 16));
                }
            }
        } else {
#pragma unroll
            for (int q = 0; q < MAXH; q++) {
                const int c = hcol<MAXH>(lane, q);
                v[q] = c < H ? h2f<F16>(z[c]) : 0.f;
            }
        }
        float mean = 0.f, rs = 1.f;
        if (use_ln) {
            float s = 0.f;
#pragma unroll
            for (int q = 0; q < MAXH; q++) s += v[q];
            mean = wave_sum(s) / (float)H;
            float s2 = 0.f;
#pragma unroll
            for (int q = 0; q < MAXH; q++) {
                float d = hcol<MAXH>(lane, q) < H ? v[q] - mean : 0.f;
                s2 += d * d;
            }
            rs = 1.f / sqrtf(wave_sum(s2) / (float)H + 1e-5f);
        }
        uint16_t o[MAXH];
#pragma unroll
        for (int q = 0; q < MAXH; q++) {
            float hv = use_ln ? h2f<F16>(f2h<F16>((v[q] - mean) * rs * g[q] + b[q])) : v[q];
            o[q] = f2h<F16>(hv > 0.f ? hv : hv * slope);
        }
        uint16_t* op = out + (int64_t)row * H;
        if (vec) {
#pragma unroll
            for (int q = 0; q < MAXH; q += 8) {
                const int c = hcol<MAXH>(lane, q);
                u32x4 t;
#pragma unroll
                for (int k = 0; k < 4; k++) t[k] = (uint32_t)o[q + 2 * k] | ((uint32_t)o[q + 2 * k + 1] << 16);
                if (c < H) *reinterpret_cast<u32x4*>(op + c) = t;
            }
        } else {
#pragma unroll
            for (int q = 0; q < MAXH; q++) {
                const int c = hcol<MAXH>(lane, q);
                if (c < H) op[c] = o[q];
            }
        }
    }
}

// Backward of LeakyReLU(LN(Z)): dZ from dA; per-block column partials of
// dbias = sum dZ, dgamma = sum dH*xhat, dbeta = sum dH -> part[blk][3][H] (the flat parameter
// order Linear.bias, LayerNorm.weight, LayerNorm.bias, so one reduction serves all three).
// Columns per lane: lcol (float4 loads / stores); gamma / beta stay in registers; each of the 4
// waves walks LNB_ROWS/4 rows.
constexpr int LNB_ROWS = 32;
constexpr int LNB_ROWS_MIN = 16;  // fewest rows per block of any variant (partial buffers are sized for it)
// ROWS rows per block, PR rows per wave and pass (loads issued before the reductions); every wave
// adds its rows to its partials in ascending order whatever PR is, so PR changes no bit
template <int MAXH, bool HEAD = false, int ROWS = LNB_ROWS, int PR = 2>
__global__ void __launch_bounds__(256) ln_act_bwd(const float* dA, const float* Z, const float2* stats, const float* gamma,
                                                 const float* beta, int R, int H, float slope, int use_ln, float* dZ,
                                                 float* part, float* amax, const float* head_dv = nullptr,
                                                 const float* head_w = nullptr, float* head_part = nullptr) {
    __shared__ float red[4][3][64 * MAXH];
    __shared__ float hred[HEAD ? 4 : 1][HEAD ? 64 * MAXH + 1 : 1];  // rank-1 head partials (head_part)
    uint32_t vmax = 0;  // max |dZ| of this thread's outputs (H3 operand scale, when amax is given)
    const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const bool vec = (H % 4 == 0) && (MAXH % 4 == 0);
    float g[MAXH], b[MAXH], pg[MAXH], pb[MAXH], pz[MAXH], hw[MAXH], ph[MAXH];
    float phb = 0.f;
#pragma unroll
    for (int q = 0; q < MAXH; q++) {
        int c = lcol<MAXH>(lane, q);
        g[q] = (use_ln && c < H) ? gamma[c] : 1.f;
        b[q] = (use_ln && c < H) ? beta[c] : 0.f;
        hw[q] = (!dA && c < H) ? head_w[c] : 0.f;
        pg[q] = pb[q] = pz[q] = ph[q] = 0.f;
    }
    const int r0 = blockIdx.x * ROWS;
    // PR rows per wave and pass: all their loads are issued before any row's reductions
    for (int rr = w; rr < ROWS; rr += 4 * PR) {
        float xs[PR][MAXH], as[PR][MAXH];
        float2 sts[PR];
        float dvs[PR];
#pragma unroll
        for (int j = 0; j < PR; j++) {
            dvs[j] = 0.f;
            const int row = r0 + rr + 4 * j;
            const bool ok = row < R;
            const int rw = ok ? row : R - 1;  // a valid row (its values are not used)
            const float* da = dA + (int64_t)rw * H;
            const float* xh = Z + (int64_t)rw * H;  // pre-norm z; xhat recomputed below
            sts[j] = stats[rw];
            if (vec) {
#pragma unroll
                for (int q = 0; q < MAXH; q += 4) {
                    const int c = lcol<MAXH>(lane, q);
                    const float4 zero = make_float4(0.f, 0.f, 0.f, 0.f);
                    float4 t = c < H ? *reinterpret_cast<const float4*>(xh + c) : zero;
                    xs[j][q] = t.x; xs[j][q + 1] = t.y; xs[j][q + 2] = t.z; xs[j][q + 3] = t.w;
                    if (dA) {
                        float4 u = c < H ? *reinterpret_cast<const float4*>(da + c) : zero;
                        as[j][q] = u.x; as[j][q + 1] = u.y; as[j][q + 2] = u.z; as[j][q + 3] = u.w;
                    }
                }
            } else {
#pragma unroll
                for (int q = 0; q < MAXH; q++) {
                    const int c = lcol<MAXH>(lane, q);
                    bool in = c < H;
                    xs[j][q] = in ? xh[c] : 0.f;
                    if (dA) as[j][q] = in ? da[c] : 0.f;
                }
            }
            if (!dA) {  // rank-1 head: dA[row, c] = dv[row] * w[c], the product head1_bwd would have stored
                const float dv = head_dv[rw];
                dvs[j] = dv;
#pragma unroll
                for (int q = 0; q < MAXH; q++) as[j][q] = dv * hw[q];
            }
        }
#pragma unroll
        for (int j = 0; j < PR; j++) {
        const int row = r0 + rr + 4 * j;
        if (row >= R) break;
        const float2 st = sts[j];
        float* x = xs[j];
        const float* av = as[j];
        float dh[MAXH];
        if (use_ln) {
#pragma unroll
            for (int q = 0; q < MAXH; q++) x[q] = (x[q] - st.x) * st.y;  // the forward's xhat, same ops
        }
        float s1 = 0.f, s2 = 0.f;
#pragma unroll
        for (int q = 0; q < MAXH; q++) {
            float h = x[q] * g[q] + b[q];
            dh[q] = h > 0.f ? av[q] : av[q] * slope;
            float gg = dh[q] * g[q];
            s1 += gg;
            s2 += gg * x[q];
            // the rank-1 head's weight gradient dv * act, act recomputed as the forward made it
            // (head1_bwd's per-lane sums in its row order: the same bits)
            if (HEAD && lcol<MAXH>(lane, q) < H) ph[q] += dvs[j] * (h > 0.f ? h : h * slope);
        }
        if (HEAD) phb += dvs[j];
        float* dz = dZ + (int64_t)row * H;
        float d[MAXH];
        if (use_ln) {
            float m1 = wave_sum_x(s1) / (float)H, m2 = wave_sum_x(s2) / (float)H;  // == wave_sum
            float rs = st.y;
#pragma unroll
            for (int q = 0; q < MAXH; q++) d[q] = rs * (dh[q] * g[q] - m1 - x[q] * m2);
        } else {
#pragma unroll
            for (int q = 0; q < MAXH; q++) d[q] = dh[q];
        }
        if (vec) {
#pragma unroll
            for (int q = 0; q < MAXH; q += 4) {
                const int c = lcol<MAXH>(lane, q);
                if (c < H) *reinterpret_cast<float4*>(dz + c) = make_float4(d[q], d[q + 1], d[q + 2], d[q + 3]);
            }
        } else {
#pragma unroll
            for (int q = 0; q < MAXH; q++) {
                const int c = lcol<MAXH>(lane, q);
                if (c < H) dz[c] = d[q];
            }
        }
#pragma unroll
        for (int q = 0; q < MAXH; q++) {
            bool in = lcol<MAXH>(lane, q) < H;
            pz[q] += in ? d[q] : 0.f;
            pg[q] += in ? dh[q] * x[q] : 0.f;
            pb[q] += in ? dh[q] : 0.f;
            const uint32_t bb = in ? abs_bits(d[q]) : 0u;
            vmax = bb > vmax ? bb : vmax;
        }
        }
    }
#pragma unroll
    for (int q = 0; q < MAXH; q++) {
        const int c = lcol<MAXH>(lane, q);
        red[w][0][c] = pz[q];
        red[w][1][c] = pg[q];
        red[w][2][c] = pb[q];
    }
    __syncthreads();
    if (HEAD) {
#pragma unroll
        for (int q = 0; q < MAXH; q++) hred[w][lcol<MAXH>(lane, q)] = ph[q];
        if (lane == 0) hred[w][64 * MAXH] = phb;
    }
    __syncthreads();
    float* out = part + (int64_t)blockIdx.x * 3 * H;
    for (int k = 0; k < 3; k++)
        for (int c = threadIdx.x; c < H; c += 256)
            out[k * H + c] = red[0][k][c] + red[1][k][c] + red[2][k][c] + red[3][k][c];
    if (HEAD) {  // [blk][w | b], head1_bwd's layout and order
        float* ho = head_part + (int64_t)blockIdx.x * (H + 1);
        for (int c = threadIdx.x; c < H; c += 256) ho[c] = hred[0][c] + hred[1][c] + hred[2][c] + hred[3][c];
        if (threadIdx.x == 0)
            ho[H] = hred[0][64 * MAXH] + hred[1][64 * MAXH] + hred[2][64 * MAXH] + hred[3][64 * MAXH];
    }
    if (amax) h3_amax_commit(amax, vmax);
}

// Wide rows (H > 512, H % 4 == 0; C5's 2048): the wave-per-row kernels above hold a whole row per lane set
// (32 columns per lane at H = 2048: spills, 1 workgroup per CU).  Here a workgroup walks LNW_ROWS rows,
// LNW_RB at a time, each thread owning the float4 column groups 4 t + 1024 k (every load / store of a wave
// is one contiguous 1 KB), the row sums reduced over the 4 waves through LDS in a fixed order.  Same
// arguments as the wave-per-row kernels (the rank-1 head options are not taken: those layers keep them).
constexpr int LNW_ROWS = 32;
DEV int wcol(int k) { return 4 * (int)threadIdx.x + 1024 * k; }
DEV float4 ld4(const float* p, int c, int H) { return c < H ? *reinterpret_cast<const float4*>(p + c) : make_float4(0.f, 0.f, 0.f, 0.f); }

template <int NV, int LNW_RB = 4>
__global__ void __launch_bounds__(256) ln_act_fwd_wide(const float* Z, const float* gamma, const float* beta, int R, int H,
                                                      float slope, int use_ln, float* act, float2* stats, float* amax,
                                                      const float*, const float*, float*) {
    __shared__ float red[2][LNW_RB][4];
    const int w = threadIdx.x >> 6;
    uint32_t vmax = 0;
    float4 g[NV], b[NV];
#pragma unroll
    for (int k = 0; k < NV; k++) {
        g[k] = use_ln ? ld4(gamma, wcol(k), H) : make_float4(1.f, 1.f, 1.f, 1.f);
        b[k] = use_ln ? ld4(beta, wcol(k), H) : make_float4(0.f, 0.f, 0.f, 0.f);
    }
    const int r_end = min(R, (int)(blockIdx.x + 1) * LNW_ROWS);
    for (int r0 = blockIdx.x * LNW_ROWS; r0 < r_end; r0 += LNW_RB) {
        float4 v[LNW_RB][NV];
#pragma unroll
        for (int j = 0; j < LNW_RB; j++) {
            const float* z = Z + (int64_t)min(r0 + j, R - 1) * H;
#pragma unroll
            for (int k = 0; k < NV; k++) v[j][k] = ld4(z, wcol(k), H);
        }
        float mean[LNW_RB], rs[LNW_RB];
#pragma unroll
        for (int j = 0; j < LNW_RB; j++) {
            mean[j] = 0.f;
            rs[j] = 1.f;
        }
        if (use_ln) {
#pragma unroll
            for (int j = 0; j < LNW_RB; j++) {
                float s = 0.f;
#pragma unroll
                for (int k = 0; k < NV; k++) s += ((v[j][k].x + v[j][k].y) + v[j][k].z) + v[j][k].w;
                s = wave_sum_x(s);
                if ((threadIdx.x & 63) == 0) red[0][j][w] = s;
            }
            __syncthreads();
#pragma unroll
            for (int j = 0; j < LNW_RB; j++) {
                mean[j] = (((red[0][j][0] + red[0][j][1]) + red[0][j][2]) + red[0][j][3]) / (float)H;
                float s2 = 0.f;
#pragma unroll
                for (int k = 0; k < NV; k++) {
                    const bool in = wcol(k) < H;
                    const float dx = v[j][k].x - mean[j], dy = v[j][k].y - mean[j], dz = v[j][k].z - mean[j],
                                dw = v[j][k].w - mean[j];
                    s2 += in ? ((dx * dx + dy * dy) + dz * dz) + dw * dw : 0.f;
                }
                s2 = wave_sum_x(s2);
                if ((threadIdx.x & 63) == 0) red[1][j][w] = s2;
            }
            __syncthreads();
#pragma unroll
            for (int j = 0; j < LNW_RB; j++)
                rs[j] = 1.f / sqrtf((((red[1][j][0] + red[1][j][1]) + red[1][j][2]) + red[1][j][3]) / (float)H + 1e-5f);
        }
#pragma unroll
        for (int j = 0; j < LNW_RB; j++) {
            const int row = r0 + j;
            if (row >= R) break;
            float* ao = act + (int64_t)row * H;
#pragma unroll
            for (int k = 0; k < NV; k++) {
                const int c = wcol(k);
                if (c >= H) continue;
                float a[4];
                const float vv[4] = {v[j][k].x, v[j][k].y, v[j][k].z, v[j][k].w};
                const float gg[4] = {g[k].x, g[k].y, g[k].z, g[k].w}, bb[4] = {b[k].x, b[k].y, b[k].z, b[k].w};
#pragma unroll
                for (int e = 0; e < 4; e++) {
                    const float xh = use_ln ? (vv[e] - mean[j]) * rs[j] : vv[e];
                    const float hv = use_ln ? xh * gg[e] + bb[e] : xh;
                    a[e] = hv > 0.f ? hv : hv * slope;
                    const uint32_t bits = abs_bits(a[e]);
                    vmax = bits > vmax ? bits : vmax;
                }
                *reinterpret_cast<float4*>(ao + c) = make_float4(a[0], a[1], a[2], a[3]);
            }
            if (threadIdx.x == 0) stats[row] = make_float2(mean[j], rs[j]);
        }
    }
    if (amax) h3_amax_commit(amax, vmax);
}

template <int NV, int LNW_RB = 4>
__global__ void __launch_bounds__(256) ln_act_bwd_wide(const float* dA, const float* Z, const float2* stats, const float* gamma,
                                                      const float* beta, int R, int H, float slope, int use_ln, float* dZ,
                                                      float* part, float* amax, const float*, const float*, float*) {
    __shared__ float red[2][2][LNW_RB][4];  // [pass parity][s1 | s2][row][wave]
    const int w = threadIdx.x >> 6;
    uint32_t vmax = 0;
    float4 g[NV], b[NV], pz[NV], pg[NV], pb[NV];
#pragma unroll
    for (int k = 0; k < NV; k++) {
        g[k] = use_ln ? ld4(gamma, wcol(k), H) : make_float4(1.f, 1.f, 1.f, 1.f);
        b[k] = use_ln ? ld4(beta, wcol(k), H) : make_float4(0.f, 0.f, 0.f, 0.f);
        pz[k] = pg[k] = pb[k] = make_float4(0.f, 0.f, 0.f, 0.f);
    }
    const int r_end = min(R, (int)(blockIdx.x + 1) * LNW_ROWS);
    int par = 0;
    for (int r0 = blockIdx.x * LNW_ROWS; r0 < r_end; r0 += LNW_RB, par ^= 1) {
        float x[LNW_RB][NV][4], dh[LNW_RB][NV][4];
        float2 st[LNW_RB];
#pragma unroll
        for (int j = 0; j < LNW_RB; j++) {
            const int rw = min(r0 + j, R - 1);
            st[j] = stats[rw];
#pragma unroll
            for (int k = 0; k < NV; k++) {
                const float4 z = ld4(Z + (int64_t)rw * H, wcol(k), H);
                const float4 a = ld4(dA + (int64_t)rw * H, wcol(k), H);
                x[j][k][0] = z.x, x[j][k][1] = z.y, x[j][k][2] = z.z, x[j][k][3] = z.w;
                dh[j][k][0] = a.x, dh[j][k][1] = a.y, dh[j][k][2] = a.z, dh[j][k][3] = a.w;
            }
        }
        float m1[LNW_RB], m2[LNW_RB];
#pragma unroll
        for (int j = 0; j < LNW_RB; j++) {
            float s1 = 0.f, s2 = 0.f;
#pragma unroll
            for (int k = 0; k < NV; k++) {
                const float gg[4] = {g[k].x, g[k].y, g[k].z, g[k].w}, bb[4] = {b[k].x, b[k].y, b[k].z, b[k].w};
#pragma unroll
                for (int e = 0; e < 4; e++) {
                    if (use_ln) x[j][k][e] = (x[j][k][e] - st[j].x) * st[j].y;  // the forward's xhat, same ops
                    const float h = x[j][k][e] * gg[e] + bb[e];
                    dh[j][k][e] = h > 0.f ? dh[j][k][e] : dh[j][k][e] * slope;
                    const float t = dh[j][k][e] * gg[e];
                    s1 += t;
                    s2 += t * x[j][k][e];
                }
            }
            m1[j] = m2[j] = 0.f;
            if (use_ln) {
                s1 = wave_sum_x(s1);
                s2 = wave_sum_x(s2);
                if ((threadIdx.x & 63) == 0) {
                    red[par][0][j][w] = s1;
                    red[par][1][j][w] = s2;
                }
            }
        }
        if (use_ln) {
            __syncthreads();  // parity buffers: the next pass writes the other half, so one barrier per pass
#pragma unroll
            for (int j = 0; j < LNW_RB; j++) {
                m1[j] = (((red[par][0][j][0] + red[par][0][j][1]) + red[par][0][j][2]) + red[par][0][j][3]) / (float)H;
                m2[j] = (((red[par][1][j][0] + red[par][1][j][1]) + red[par][1][j][2]) + red[par][1][j][3]) / (float)H;
            }
        }
#pragma unroll
        for (int j = 0; j < LNW_RB; j++) {
            const int row = r0 + j;
            if (row >= R) break;
            float* dz = dZ + (int64_t)row * H;
#pragma unroll
            for (int k = 0; k < NV; k++) {
                const int c = wcol(k);
                if (c >= H) continue;
                const float gg[4] = {g[k].x, g[k].y, g[k].z, g[k].w};
                float d[4];
#pragma unroll
                for (int e = 0; e < 4; e++) {
                    d[e] = use_ln ? st[j].y * (dh[j][k][e] * gg[e] - m1[j] - x[j][k][e] * m2[j]) : dh[j][k][e];
                    const uint32_t bits = abs_bits(d[e]);
                    vmax = bits > vmax ? bits : vmax;
                }
                *reinterpret_cast<float4*>(dz + c) = make_float4(d[0], d[1], d[2], d[3]);
                pz[k].x += d[0], pz[k].y += d[1], pz[k].z += d[2], pz[k].w += d[3];
                pg[k].x += dh[j][k][0] * x[j][k][0], pg[k].y += dh[j][k][1] * x[j][k][1];
                pg[k].z += dh[j][k][2] * x[j][k][2], pg[k].w += dh[j][k][3] * x[j][k][3];
                pb[k].x += dh[j][k][0], pb[k].y += dh[j][k][1], pb[k].z += dh[j][k][2], pb[k].w += dh[j][k][3];
            }
        }
    }
    // this thread's columns' partials over the workgroup's rows, in row order: part[blk][dbias | dgamma | dbeta]
    float* out = part + (int64_t)blockIdx.x * 3 * H;
#pragma unroll
    for (int k = 0; k < NV; k++) {
        const int c = wcol(k);
        if (c >= H) continue;
        *reinterpret_cast<float4*>(out + c) = pz[k];
        *reinterpret_cast<float4*>(out + H + c) = pg[k];
        *reinterpret_cast<float4*>(out + 2 * H + c) = pb[k];
    }
    if (amax) h3_amax_commit(amax, vmax);
}

// the wide kernels for H in (512, 4096] with H % 4 == 0 (null: not applicable)
inline decltype(&ln_act_fwd_wide<2>) ln_act_fwd_wide_any(int H) {
    if (H <= 512 || H % 4 != 0 || H > 4096) return nullptr;
    if (H <= 1024) return &ln_act_fwd_wide<1>;
    if (H <= 2048) return &ln_act_fwd_wide<2>;
    return &ln_act_fwd_wide<4>;
}
inline decltype(&ln_act_bwd_wide<2>) ln_act_bwd_wide_any(int H) {
    if (H <= 512 || H % 4 != 0 || H > 4096) return nullptr;
    if (H <= 1024) return &ln_act_bwd_wide<1>;
    if (H <= 2048) return &ln_act_bwd_wide<2>;
    return &ln_act_bwd_wide<4>;
}

// NPER (columns per lane) dispatch: H <= 64 * NPER
#define RLGPU_NPER_DISPATCH(NAME)                                  \
    inline decltype(&NAME<16>) NAME##_any(int H) {                 \
        if (H <= 64) return &NAME<1>;                              \
        if (H <= 128) return &NAME<2>;                             \
        if (H <= 256) return &NAME<4>;                             \
        if (H <= 512) return &NAME<8>;                             \
        if (H <= 1024) return &NAME<16>;                           \
        return &NAME<32>;                                          \
    }
RLGPU_NPER_DISPATCH(ln_act_fwd_f32)
template <bool F16>
inline decltype(&ln_act_fwd_bf16<16, F16>) ln_act_fwd_bf16_any(int H) {
    if (H <= 64) return &ln_act_fwd_bf16<1, F16>;
    if (H <= 128) return &ln_act_fwd_bf16<2, F16>;
    if (H <= 256) return &ln_act_fwd_bf16<4, F16>;
    if (H <= 512) return &ln_act_fwd_bf16<8, F16>;
    if (H <= 1024) return &ln_act_fwd_bf16<16, F16>;
    return &ln_act_fwd_bf16<32, F16>;
}
RLGPU_NPER_DISPATCH(ln_act_bwd)
// the variant that also emits a following rank-1 head's dw / db partials (head_part)
inline decltype(&ln_act_bwd<16, true>) ln_act_bwd_head_any(int H) {
    if (H <= 64) return &ln_act_bwd<1, true>;
    if (H <= 128) return &ln_act_bwd<2, true>;
    if (H <= 256) return &ln_act_bwd<4, true>;
    if (H <= 512) return &ln_act_bwd<8, true>;
    if (H <= 1024) return &ln_act_bwd<16, true>;
    return &ln_act_bwd<32, true>;
}

// The LayerNorm kernels by width: the wide workgroup-per-row-group kernels above 512 columns (not for the
// rank-1 head's fused backward), the wave-per-row kernels below.
inline decltype(&ln_act_fwd_f32<8>) ln_act_fwd_f32_pick(int H, int* rows, bool head = false) {
    *rows = LNF_ROWS;
    if (!head)
        if (auto f = ln_act_fwd_wide_any(H)) {
            *rows = LNW_ROWS;
            return f;
        }
    return ln_act_fwd_f32_any(H);
}
inline decltype(&ln_act_bwd<8>) ln_act_bwd_pick(int H, bool head, int* rows) {
    *rows = LNB_ROWS;
    if (!head)
        if (auto f = ln_act_bwd_wide_any(H)) {
            *rows = LNW_ROWS;
            return f;
        }
    return head ? ln_act_bwd_head_any(H) : ln_act_bwd_any(H);
}

// Rank-1 output layer (the critic's Linear(H, 1)): GEMM tiles would be 1/128 occupied, so the
// head runs as wave-per-row dot products.  Columns per lane: lcol (float4 loads when H is a
// multiple of 4); w stays in registers and each wave walks H1_ROWS/4 rows.
constexpr int H1_ROWS = 16;
template <int MAXH>
__global__ void __launch_bounds__(256) head1_fwd(const float* X, const float* w, const float* b, int R, int H, float* out) {
    const int wv = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const bool vec = (H % 4 == 0) && (MAXH % 4 == 0);
    float wr[MAXH];
#pragma unroll
    for (int q = 0; q < MAXH; q++) {
        const int c = lcol<MAXH>(lane, q);
        wr[q] = c < H ? w[c] : 0.f;
    }
    const float bias = b[0];
    for (int i = 0; i < H1_ROWS / 4; i++) {
        const int row = blockIdx.x * H1_ROWS + i * 4 + wv;
        if (row >= R) break;
        const float* x = X + (int64_t)row * H;
        float s = 0.f;
        if (vec) {
#pragma unroll
            for (int q = 0; q < MAXH; q += 4) {
                const int c = lcol<MAXH>(lane, q);
                if (c < H) {
                    float4 t = *reinterpret_cast<const float4*>(x + c);
                    s += t.x * wr[q] + t.y * wr[q + 1] + t.z * wr[q + 2] + t.w * wr[q + 3];
                }
            }
        } else {
#pragma unroll
            for (int q = 0; q < MAXH; q++) {
                const int c = lcol<MAXH>(lane, q);
                if (c < H) s += x[c] * wr[q];
            }
        }
        s = wave_sum(s);
        if (lane == 0) out[row] = s + bias;
    }
}

// Backward of the rank-1 head: dA[i, :] = dv[i] * w; partials part[blk][0..H) = sum dv*X[i, :],
// part[blk][H] = sum dv (bias) over the block's rows.  Same lane layout as head1_fwd.
template <int MAXH>
__global__ void __launch_bounds__(256) head1_bwd(const float* X, const float* w, const float* dv, int R, int H, float* dA,
                                                float* part) {
    __shared__ float red[4][64 * MAXH + 1];
    const int wv = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const bool vec = (H % 4 == 0) && (MAXH % 4 == 0);
    float wr[MAXH], acc[MAXH];
    float accb = 0.f;
#pragma unroll
    for (int q = 0; q < MAXH; q++) {
        const int c = lcol<MAXH>(lane, q);
        wr[q] = c < H ? w[c] : 0.f;
        acc[q] = 0.f;
    }
    const int r0 = blockIdx.x * LNB_ROWS;
    for (int rr = wv; rr < LNB_ROWS; rr += 4) {
        const int row = r0 + rr;
        if (row >= R) break;
        const float d = dv[row];
        const float* x = X + (int64_t)row * H;
        float* da = dA ? dA + (int64_t)row * H : nullptr;  // null: the LayerNorm backward recomputes dA
        if (vec) {
#pragma unroll
            for (int q = 0; q < MAXH; q += 4) {
                const int c = lcol<MAXH>(lane, q);
                if (c < H) {
                    float4 t = *reinterpret_cast<const float4*>(x + c);
                    if (dA) *reinterpret_cast<float4*>(da + c) = make_float4(d * wr[q], d * wr[q + 1], d * wr[q + 2], d * wr[q + 3]);
                    acc[q] += d * t.x;
                    acc[q + 1] += d * t.y;
                    acc[q + 2] += d * t.z;
                    acc[q + 3] += d * t.w;
                }
            }
        } else {
#pragma unroll
            for (int q = 0; q < MAXH; q++) {
                const int c = lcol<MAXH>(lane, q);
                if (c < H) {
                    if (dA) da[c] = d * wr[q];
                    acc[q] += d * x[c];
                }
            }
        }
        accb += d;
    }
#pragma unroll
    for (int q = 0; q < MAXH; q++) red[wv][lcol<MAXH>(lane, q)] = acc[q];
    if (lane == 0) red[wv][64 * MAXH] = accb;
    __syncthreads();
    float* out = part + (int64_t)blockIdx.x * (H + 1);
    for (int c = threadIdx.x; c < H; c += 256) out[c] = red[0][c] + red[1][c] + red[2][c] + red[3][c];
    if (threadIdx.x == 0) out[H] = red[0][64 * MAXH] + red[1][64 * MAXH] + red[2][64 * MAXH] + red[3][64 * MAXH];
}
RLGPU_NPER_DISPATCH(head1_fwd)
RLGPU_NPER_DISPATCH(head1_bwd)

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

// The column sums of one tile of reduce_cols (block (x, y) of a G-group grid): the same loads in the same
// order, so reduce_batch's column jobs give reduce_cols's bits.
DEV void reduce_cols_tile(const float* part, int nblk, int64_t stride, int n, int x, int y, int G, float* out,
                          int64_t out_stride, int accumulate, float (*red)[64]) {
    const int cl = threadIdx.x & 63, gi = threadIdx.x >> 6;
    const int c = x * 64 + cl;
    float s = 0.f;
    if (c < n) {
        const int step = 16 * G;
        for (int b = y + G * gi; b < nblk; b += 8 * step) {
            float v[8];
#pragma unroll
            for (int k = 0; k < 8; k++) {
                const int bk = b + k * step;
                v[k] = part[(int64_t)(bk < nblk ? bk : b) * stride + c];
            }
#pragma unroll
            for (int k = 0; k < 8; k++)
                if (b + k * step < nblk) s += v[k];
        }
    }
    red[gi][cl] = s;
    __syncthreads();
    if (gi == 0 && c < n) {
        float tot = 0.f;
        for (int k = 0; k < 16; k++) tot += red[k][cl];
        float* o = out + (int64_t)y * out_stride + c;
        *o = accumulate ? *o + tot : tot;
    }
}

// Every reduction of one backward pass in one launch per level (instead of one or two launches per
// reduction).  Job k: dst[c] += sum over nblk partial rows (stride floats apart) of column c < n.
//   vec = 1: split-K weight-gradient partials (few rows, many columns): 4 columns per thread, rows in
//            order -- reduce_splits4's sums; vec = 2: one column per thread -- reduce_splits's.
//   vec = 0: per-block column partials: reduce_cols's scheme, level 1 over G row groups into mid[y][c]
//            (or straight into dst when G = 1), level 2 over mid's G rows into dst.
// Blocks of 1024 threads; b.tile0[k] = first block of job k at this level (a job with no tiles at a
// level is skipped).  Same bits as the separate launches.
constexpr int kRedJobs = 16;
struct RedJob {
    const float* part;
    float* dst;
    float* mid;
    int64_t stride;
    int nblk, n, G, vec;
};
struct RedBatch {
    RedJob j[kRedJobs];
    int tile0[kRedJobs + 1];
    int njobs, level;
};
__global__ void __launch_bounds__(1024) reduce_batch(RedBatch b) {
    __shared__ float red[16][64];
    const int t = blockIdx.x;
    int k = 0;
    while (k + 1 < b.njobs && b.tile0[k + 1] <= t) k++;
    const RedJob& J = b.j[k];
    const int r = t - b.tile0[k];
    if (J.vec == 1) {
        const int64_t e = ((int64_t)r * 1024 + threadIdx.x) * 4;
        if (e >= J.n) return;
        float4 s = make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll 4
        for (int q = 0; q < J.nblk; q++) {
            const float4 v = *reinterpret_cast<const float4*>(J.part + q * J.stride + e);
            s.x += v.x;
            s.y += v.y;
            s.z += v.z;
            s.w += v.w;
        }
        float4* o = reinterpret_cast<float4*>(J.dst + e);
        const float4 v = *o;
        *o = make_float4(v.x + s.x, v.y + s.y, v.z + s.z, v.w + s.w);
        return;
    }
    if (J.vec == 2) {
        const int64_t e = (int64_t)r * 1024 + threadIdx.x;
        if (e >= J.n) return;
        float s = 0.f;
        for (int q = 0; q < J.nblk; q++) s += J.part[q * J.stride + e];
        J.dst[e] = J.dst[e] + s;
        return;
    }
    const int cx = (J.n + 63) / 64;
    if (b.level == 1)
        reduce_cols_tile(J.part, J.nblk, J.stride, J.n, r % cx, r / cx, J.G, J.G > 1 ? J.mid : J.dst, J.n, J.G > 1 ? 0 : 1,
                         red);
    else
        reduce_cols_tile(J.mid, J.G, J.n, J.n, r, 0, 1, J.dst, 0, 1, red);
}

// Column reduction of per-block partials, deterministic, two levels:
//   stage 1 (grid ceil(n/64) x G): block (x, y) sums partial rows b = y, y+G, ... of 64 columns
//            (16 row groups of 64 threads, combined in LDS in a fixed order) -> out2[y][c]
//   stage 2 (the same kernel with G = 1 on out2, accumulate = 1): grad[c] += sum_y out2[y][c]
__global__ void __launch_bounds__(1024) reduce_cols(const float* part, int nblk, int64_t stride, int64_t off, int n,
                                                   float* out, int64_t out_stride, int accumulate) {
    __shared__ float red[16][64];
    const int cl = threadIdx.x & 63, gi = threadIdx.x >> 6;
    const int c = blockIdx.x * 64 + cl;
    const int G = gridDim.y, y = blockIdx.y;
    float s = 0.f;
    if (c < n) {
        // eight partial rows loaded before they are added (in the same order as a plain loop: the
        // same bits), so a thread has eight loads in flight instead of one
        const int step = 16 * G;
        for (int b = y + G * gi; b < nblk; b += 8 * step) {
            float v[8];
#pragma unroll
            for (int k = 0; k < 8; k++) {
                const int bk = b + k * step;
                v[k] = part[(int64_t)(bk < nblk ? bk : b) * stride + off + c];
            }
#pragma unroll
            for (int k = 0; k < 8; k++)
                if (b + k * step < nblk) s += v[k];
        }
    }
    red[gi][cl] = s;
    __syncthreads();
    if (gi == 0 && c < n) {
        float tot = 0.f;
        for (int k = 0; k < 16; k++) tot += red[k][cl];
        float* o = out + (int64_t)y * out_stride + c;
        *o = accumulate ? *o + tot : tot;
    }
}

}  // namespace mlp

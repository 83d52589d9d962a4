// ppo.hip -- C ABI of include/rlgpu_ppo.h: actor/critic MLPs, action sampling, PPO minibatch
// loss + backward, clip_grad_norm_ + AdamW, on hand-written MFMA / wave kernels.
#include <hipcub/hipcub.hpp>

#include <cmath>
#include <cstring>
#include <vector>

#include "../../include/rlgpu_ppo.h"
#include "common.hpp"
#include "mlp_kernels.hpp"
#include "ppo_kernels.hpp"
#include "infer_kernels.hpp"

namespace {

using rlgpu::ceil_div;

// launch a kernel template instantiated on the 16-bit inference format (bf16 / fp16)
#define RLGPU_H16_LAUNCH(F16, KERN, ...)                                                     \
    do {                                                                                     \
        if (F16) hipLaunchKernelGGL(KERN<true>, __VA_ARGS__);                                \
        else hipLaunchKernelGGL(KERN<false>, __VA_ARGS__);                                   \
    } while (0)

struct Layer {
    int in, out;
    int64_t w, b, g, be;      // offsets into the flat fp32 buffers (g/be = -1 without LayerNorm)
    int in_pad;               // bf16 copy: weight rows padded to a multiple of 8 (16 bytes)
    int64_t hw, hb, hg, hbe;  // offsets into the padded bf16 inference copy
    int64_t fw = -1;          // offset into the fragment-major inference copy (infer::weight_to_frag)
    // three-way bf16 split of the weight for the x6 training GEMMs (offsets into Model::wsplit):
    // forward B = W [out_pad128][in_pad32], backward dA B = W^T [in_pad128][out_pad32]; -1 = none
    int64_t sf = -1, sb = -1;
    int sf_rows = 0, sf_ld = 0, sb_rows = 0, sb_ld = 0;
    int64_t sfs = -1, sbs = -1;  // H3: per-row inverse scales of the planes (offsets into Model::wscale)
};

struct Model {
    std::vector<Layer> L;  // hidden layers then the output layer (last; none for the shared head)
    bool head_only = false;  // the shared head: every layer is [Linear -> LayerNorm -> LeakyReLU]
    int in, out;
    int64_t off, count;
    float lr;
    int mode = 0;  // training GEMM arithmetic (rlgpu_ppo_config.train_gemm)
    // fp32 training workspace (per model, so the two models' passes can overlap on two streams)
    std::vector<float*> xhat, act, rstd;
    float *y = nullptr, *dy = nullptr, *dA = nullptr, *dZ = nullptr, *wpart = nullptr, *cpart = nullptr, *mid = nullptr;  // y: model output
    float* hpart = nullptr;  // rank-1 head dw / db partials, written by the last LayerNorm backward
    // per-layer partial buffers of the deferred reductions (so a backward pass reduces them all at its end):
    // split-K weight-gradient partials of layer l, LayerNorm-backward column partials of hidden layer l, and
    // the loss kernel's output-bias partials
    std::vector<float*> wpart_l, cpart_l;
    float* lpart = nullptr;
    int64_t midn = 0;  // floats per row of a reduction's level-1 sums (m.mid holds kRedJobs x 16 rows)
    uint16_t* wsplit = nullptr;  // split weight planes (x6 / H3 modes)
    int64_t nsplit = 0;
    float* wscale = nullptr;     // H3: per-row inverse scales of the weight planes
    int64_t nscale = 0;
    // H3: 64-shard max |x| slots of the GEMM operand tensors (kAmaxSlots x 64 floats):
    // act[l] at slot l, dZ of layer l at kAmaxDZ + l, the loss gradient dout at kAmaxOut
    float* amax = nullptr;
    float* dX = nullptr;  // gradient w.r.t. the model input (policy / critic behind a shared head)
};
// hidden [Linear -> LayerNorm -> LeakyReLU] layers of a model (all of the shared head's)
inline int nhid(const Model& m) { return (int)m.L.size() - (m.head_only ? 0 : 1); }
constexpr int kAmaxDZ = RLGPU_MAX_LAYERS, kAmaxOut = 2 * RLGPU_MAX_LAYERS, kAmaxSlots = 2 * RLGPU_MAX_LAYERS + 1;
inline bool split_mode(int mode) { return mode == RLGPU_GEMM_F32X6 || mode == RLGPU_GEMM_F16X3; }

constexpr int kMaxSplits = 256;
// concurrent gemm_f32 workgroups on the device (CUs x RLGPU_GEMM_OCC), set at create: the split-K
// weight gradients are sized to fill whole rounds of workgroups
int g_cus = 256;  // compute units of the device, set at create
// Forward / input-gradient H3 GEMMs with output widths that are multiples of 256 on the 256 x 256 tile kernel
// mlp::gemm_h3q, and weight gradients on mlp::gemm_h3qt (same bits as gemm_x6): by default for 1024 or
// more output columns (the C5 leg's 2048-wide layers: 31.6 -> 27.6 ms per 50k minibatch against 128 x 256 tiles,
// profiles/r05ad_h3_quad_ab.txt); at 512 columns
// (K = 512, 16 stages per tile) its one workgroup per CU cannot hide the tile's prologue and epilogue and the
// C2 minibatch takes 1.59 -> 1.70 ms.  RLGPU_H3_QUAD=0: never, 1: for every width that is a multiple of 256.
inline bool h3_quad(int J) {
    static const int mode = [] {
        const char* e = getenv("RLGPU_H3_QUAD");
        return e ? atoi(e) : -1;
    }();
    if (J % mlp::BQ != 0) return false;
    return mode == 1 ? true : (mode == 0 ? false : J >= 1024);
}
inline bool split_mode_(int mode) { return mode == RLGPU_GEMM_F32X6 || mode == RLGPU_GEMM_F16X3; }
inline int gemm_slots(int mode) {
    // H3: 146 / 156 VGPRs (forward / weight-gradient instances), 40 KB LDS -> three workgroups per CU
    // (-Rpass-analysis=kernel-resource-usage: occupancy 3 waves / SIMD); x6: two
    if (mode == RLGPU_GEMM_F16X3) return g_cus * 3;
    return g_cus * (split_mode_(mode) ? 2 : RLGPU_GEMM_OCC);
}
// K granularity of a split-K chunk: a whole number of stages of either kernel
inline int kgran(int mode) { return split_mode_(mode) ? mlp::XKMAX : mlp::BK; }

}  // namespace

struct rlgpu_ppo {
    rlgpu_ppo_config cfg;
    Model M[3];       // policy, critic, shared head (M[2], present when nm == 3)
    int nm = 2;
    bool shared() const { return nm == 3; }
    float* dshared = nullptr;  // the shared head's output gradient: policy dX + critic dX
    int64_t nparams = 0, nhalf = 0;
    float *params = nullptr, *grads = nullptr, *exp_avg = nullptr, *exp_avg_sq = nullptr;
    uint16_t* half = nullptr;
    uint16_t* half_ver = nullptr;  // bf16 policy copy of an old version (self-play), same layout as half
    uint16_t *frag = nullptr, *frag_ver = nullptr;  // the weights of half / half_ver in MFMA fragment order
    int64_t nfrag = 0;
    bool has_ver = false;
    // the training GEMMs' split weight planes are stale (parameters changed since the last split):
    // set by init / refresh_half / the optimizer step, cleared when forward_train re-splits.  With
    // the whole iteration as one batch the planes are rebuilt once per optimizer step, not per
    // minibatch.
    bool split_dirty[3] = {true, true, true};
    int64_t step = 0;
    int hmax = 0;
    float *scratch = nullptr;  // clip partials + coefficients
    hipStream_t aux = nullptr;  // second stream: the critic's minibatch pass overlaps the policy's
    hipEvent_t ev_fork = nullptr, ev_join = nullptr;
    float* x0 = nullptr;       // gathered minibatch obs, rows padded to x_ld floats
    int x_ld = 0;
    float* x_amax = nullptr;   // H3: 64-shard max |x0| (with both models' slots: one memset per pass)
    float* amax_all = nullptr;
    int64_t amax_count = 0;
    uint16_t* xh = nullptr;    // bf16 obs for inference, rows padded to xh_ld
    int xh_ld = 0;
    uint16_t *zh = nullptr, *ah[2] = {nullptr, nullptr}, *logits_h = nullptr;
    float* logits_f = nullptr;  // fp32 inference (RLGPU_INFER_F32): the policy's logits [max_rows][A]
    std::vector<void*> allocs;

    template <class T>
    T* alloc(size_t count) {
        void* p = nullptr;
        RLGPU_CHECK_HIP(hipMalloc(&p, count * sizeof(T) + 16));
        allocs.push_back(p);
        return (T*)p;
    }
};

// inference precision (rlgpu_ppo_config.infer_fp16): the 16-bit copy's type, and whether the policy / critic
// inference runs the fp32 training forward instead (useHalfPrecision = false, Models.cpp:36-68)
inline bool f16(const rlgpu_ppo* h) { return h->cfg.infer_fp16 == RLGPU_INFER_F16; }
inline bool infer_f32(const rlgpu_ppo* h) { return h->cfg.infer_fp16 == RLGPU_INFER_F32; }

namespace {

// ---- learn-phase kernel timing (rlgpu_kernel_timing / rlgpu_kernel_timing_read): HIP events
// around the training GEMM and LayerNorm launches, recorded on the stream each launch goes to (the
// policy's and the critic's passes run on two streams).  Off unless enabled; bench.py reports the
// learn phase's roofline from it.  Work per launch: flops (GEMMs) or algorithmic bytes (row kernels).
namespace ktime {
enum { FWD_GEMM = 0, WGRAD_GEMM = 1, LN_FWD = 2, LN_BWD = 3, NSLOT = 4 };
struct Rec {
    hipEvent_t a, b;
    int slot;
    double work;
};
struct State {
    bool on = false;
    std::vector<Rec> recs;
    std::vector<hipEvent_t> pool;  // events of cleared records, reused
};
State g;
hipEvent_t event() {
    hipEvent_t e;
    if (!g.pool.empty()) {
        e = g.pool.back();
        g.pool.pop_back();
    } else {
        RLGPU_CHECK_HIP(hipEventCreate(&e));
    }
    return e;
}
void clear() {
    for (auto& r : g.recs) {
        g.pool.push_back(r.a);
        g.pool.push_back(r.b);
    }
    g.recs.clear();
}
// brackets one launch on stream s
struct Span {
    int idx = -1;
    hipStream_t s;
    Span(int slot, double work, hipStream_t s_) : s(s_) {
        if (!g.on) return;
        Rec r{event(), event(), slot, work};
        RLGPU_CHECK_HIP(hipEventRecord(r.a, s));
        g.recs.push_back(r);
        idx = (int)g.recs.size() - 1;
    }
    ~Span() {
        if (idx >= 0) (void)hipEventRecord(g.recs[idx].b, s);
    }
};
}  // namespace ktime

// C[I,J] (+ bias) = A . B with the layouts of mlp::gemm_f32.  *_tail_ok: the operand's rows are
// zero-padded up to a multiple of 4 past the bound (so float4 loads may straddle it).
template <int LA, int LB, bool AV, bool BV, bool PRE, bool H3>
void x6_launch_v(dim3 grid, dim3 blk, hipStream_t s, const mlp::GemmArgs& g) {
    hipLaunchKernelGGL((mlp::gemm_x6<LA, LB, AV, BV, PRE, H3>), grid, blk, 0, s, g);
}
template <int LA, int LB, bool H3>
void x6_launch(bool av, bool bv, dim3 grid, dim3 blk, hipStream_t s, const mlp::GemmArgs& g) {
    if (av && bv) x6_launch_v<LA, LB, true, true, false, H3>(grid, blk, s, g);
    else if (av) x6_launch_v<LA, LB, true, false, false, H3>(grid, blk, s, g);
    else if (bv) x6_launch_v<LA, LB, false, true, false, H3>(grid, blk, s, g);
    else x6_launch_v<LA, LB, false, false, false, H3>(grid, blk, s, g);
}

// amax_a / amax_b: the operands' 64-shard max |x| (RLGPU_GEMM_F16X3 only)
void gemm_f32(int mode, int la, int lb, const float* A, int64_t lda, const float* B, int64_t ldb, float* C, int64_t ldc,
              const float* bias, int I, int J, int K, int splits, hipStream_t s, bool a_tail_ok = false,
              bool b_tail_ok = false, const float* amax_a = nullptr, const float* amax_b = nullptr) {
    mlp::GemmArgs g{};
    g.amax_a = amax_a;
    g.amax_b = amax_b;
    if (mode == RLGPU_GEMM_F16X3 && !(amax_a && amax_b)) throw rlgpu::Error(RLGPU_ERR_STATE, "H3 GEMM without operand scales");
    g.A = A;
    g.B = B;
    g.C = C;
    g.bias = bias;
    g.lda = lda;
    g.ldb = ldb;
    g.ldc = ldc;
    g.I = I;
    g.J = J;
    g.K = K;
    int chunk = (int)ceil_div(K, splits);
    g.kchunk = (int)ceil_div(chunk, kgran(mode)) * kgran(mode);
    int z = (int)ceil_div(K, g.kchunk);
    g.c_split = (int64_t)I * ldc;
    // float4 path: 16-byte aligned rows and a bound (K for k-contiguous, I / J otherwise) that is a
    // multiple of 4 or zero-padded past it (split-K chunk ends are multiples of BK)
    const int a_lim = la == mlp::A_IK ? K : I, b_lim = lb == mlp::B_JK ? K : J;
    const bool av = (lda % 4 == 0) && ((uintptr_t)A % 16 == 0) && (a_lim % 4 == 0 || a_tail_ok);
    const bool bv = (ldb % 4 == 0) && ((uintptr_t)B % 16 == 0) && (b_lim % 4 == 0 || b_tail_ok);
    g.gx = (int)ceil_div(J, mlp::BN);
    g.gy = (int)ceil_div(I, mlp::BM);
    g.gz = z;
    if (mode == RLGPU_GEMM_F16X3 && la == mlp::A_KI && lb == mlp::B_KJ && I % mlp::BQ == 0 && h3_quad(J)) {
        // 256 x 256 tiles, the same split-K chunks (same bits as gemm_x6)
        g.gx = J / mlp::BQ;
        g.gy = I / mlp::BQ;
        dim3 gridq(g.gx * g.gy * g.gz), blkq(512);
        if (av && bv) hipLaunchKernelGGL((mlp::gemm_h3qt<true, true>), gridq, blkq, 0, s, g);
        else if (av) hipLaunchKernelGGL((mlp::gemm_h3qt<true, false>), gridq, blkq, 0, s, g);
        else if (bv) hipLaunchKernelGGL((mlp::gemm_h3qt<false, true>), gridq, blkq, 0, s, g);
        else hipLaunchKernelGGL((mlp::gemm_h3qt<false, false>), gridq, blkq, 0, s, g);
        RLGPU_CHECK_HIP(hipGetLastError());
        return;
    }
    dim3 grid(g.gx * g.gy * g.gz), blk(256);
#define RLGPU_GEMM_CASE(LA, LB)                                                                                  \
    if (la == LA && lb == LB) {                                                                                  \
        if (mode == RLGPU_GEMM_F32X6) {                                                                          \
            x6_launch<LA, LB, false>(av, bv, grid, blk, s, g);                                                   \
        } else if (mode == RLGPU_GEMM_F16X3) {                                                                   \
            x6_launch<LA, LB, true>(av, bv, grid, blk, s, g);                                                    \
        } else {                                                                                                 \
            if (av && bv) hipLaunchKernelGGL((mlp::gemm_f32<LA, LB, true, true>), grid, blk, 0, s, g);           \
            else if (av) hipLaunchKernelGGL((mlp::gemm_f32<LA, LB, true, false>), grid, blk, 0, s, g);          \
            else if (bv) hipLaunchKernelGGL((mlp::gemm_f32<LA, LB, false, true>), grid, blk, 0, s, g);          \
            else hipLaunchKernelGGL((mlp::gemm_f32<LA, LB, false, false>), grid, blk, 0, s, g);                 \
        }                                                                                                        \
        RLGPU_CHECK_HIP(hipGetLastError());                                                                      \
        return;                                                                                                  \
    }
    RLGPU_GEMM_CASE(mlp::A_IK, mlp::B_JK)
    RLGPU_GEMM_CASE(mlp::A_IK, mlp::B_KJ)
    RLGPU_GEMM_CASE(mlp::A_KI, mlp::B_KJ)
#undef RLGPU_GEMM_CASE
    throw rlgpu::Error(RLGPU_ERR_UNSUPPORTED, "gemm layout");
}

// C[I,J] (+ bias) = A . B on the x6 GEMM with B given as pre-split planes (Layer::sf / sb layout)
// H3 (bscale given): fp16 planes with per-row inverse scales bscale, A scaled by amax_a's shards
void gemm_x6_pre(const float* A, int64_t lda, const uint16_t* Bp, int ldbp, int64_t bplane, float* C, int64_t ldc,
                 const float* bias, int I, int J, int K, hipStream_t s, bool a_tail_ok = false,
                 const float* amax_a = nullptr, const float* bscale = nullptr) {
    ktime::Span span(ktime::FWD_GEMM, 2.0 * I * J * K, s);
    mlp::GemmArgs g{};
    g.amax_a = amax_a;
    g.bscale = bscale;
    const bool h3 = bscale != nullptr;
    if (h3 && !amax_a) throw rlgpu::Error(RLGPU_ERR_STATE, "H3 GEMM without operand scales");
    g.A = A;
    g.B = reinterpret_cast<const float*>(Bp);
    g.C = C;
    g.bias = bias;
    g.lda = lda;
    g.ldb = ldbp;
    g.ldc = ldc;
    g.I = I;
    g.J = J;
    g.K = K;
    g.kchunk = (int)ceil_div(K, mlp::XKMAX) * mlp::XKMAX;
    g.c_split = 0;
    g.bplane = bplane;
    g.gx = (int)ceil_div(J, mlp::BN);
    g.gy = (int)ceil_div(I, mlp::BM);
    g.gz = 1;
    const bool av = (lda % 4 == 0) && ((uintptr_t)A % 16 == 0) && (K % 4 == 0 || a_tail_ok);
    if (h3 && av && h3_quad(J)) {  // 256 x 256 tiles (bit-identical to gemm_x6's H3 path)
        g.gx = J / mlp::BQ;
        g.gy = (int)ceil_div(I, mlp::BQ);
        hipLaunchKernelGGL((mlp::gemm_h3q<true>), dim3(g.gx * g.gy), dim3(512), 0, s, g);
        RLGPU_CHECK_HIP(hipGetLastError());
        return;
    }
    dim3 grid(g.gx * g.gy), blk(256);
    if (h3) {
        if (av)
            x6_launch_v<mlp::A_IK, mlp::B_JK, true, true, true, true>(grid, blk, s, g);
        else
            x6_launch_v<mlp::A_IK, mlp::B_JK, false, true, true, true>(grid, blk, s, g);
    } else {
        if (av)
            x6_launch_v<mlp::A_IK, mlp::B_JK, true, true, true, false>(grid, blk, s, g);
        else
            x6_launch_v<mlp::A_IK, mlp::B_JK, false, true, true, false>(grid, blk, s, g);
    }
    RLGPU_CHECK_HIP(hipGetLastError());
}

// refresh the split weight planes of model m from the current parameters (once per minibatch /
// training forward: the weights change only at the optimizer step, but may be written directly)
void split_weights(const float* P, Model& m, hipStream_t s) {
    if (!split_mode(m.mode)) return;
    if (m.mode == RLGPU_GEMM_F16X3) {
        for (auto& L : m.L) {
            if (L.sf >= 0)
                hipLaunchKernelGGL(mlp::split_weight_h3, dim3(L.sf_rows), dim3(256), 0, s, P + L.w, L.out, L.in, (int64_t)L.in, 0, L.sf_ld,
                                   m.wsplit + L.sf, (int64_t)L.sf_rows * L.sf_ld, m.wscale + L.sfs);
            if (L.sb >= 0)
                hipLaunchKernelGGL(mlp::split_weight_h3, dim3(L.sb_rows), dim3(256), 0, s, P + L.w, L.out, L.in, (int64_t)L.in, 1, L.sb_ld,
                                   m.wsplit + L.sb, (int64_t)L.sb_rows * L.sb_ld, m.wscale + L.sbs);
        }
        RLGPU_CHECK_HIP(hipGetLastError());
        return;
    }
    for (auto& L : m.L) {
        if (L.sf >= 0) {
            int64_t e = (int64_t)L.sf_rows * L.sf_ld;
            hipLaunchKernelGGL(mlp::split_weight, dim3(ceil_div(e, 256)), dim3(256), 0, s, P + L.w, L.out, L.in, 0, L.sf_rows,
                               L.sf_ld, m.wsplit + L.sf);
        }
        if (L.sb >= 0) {
            int64_t e = (int64_t)L.sb_rows * L.sb_ld;
            hipLaunchKernelGGL(mlp::split_weight, dim3(ceil_div(e, 256)), dim3(256), 0, s, P + L.w, L.out, L.in, 1, L.sb_rows,
                               L.sb_ld, m.wsplit + L.sb);
        }
    }
    RLGPU_CHECK_HIP(hipGetLastError());
}

// split-K count of a weight gradient [out, in] over `rows`: one full round of workgroups
// (tiles x splits ~ gemm_slots), each split at least 4 K steps
int splits_for(int mode, int rows, int out, int in) {
    // H3 weight gradients of 1024 or more columns: counted in 128 x 256 blocks (the chunking gemm_h3qt's
    // 256 x 256 tiles were tuned with, profiles/r05ad_h3_quad_ab.txt)
    const int bn = (mode == RLGPU_GEMM_F16X3 && in >= 1024) ? mlp::BNW : mlp::BN;
    const int tiles = (int)(ceil_div(out, mlp::BM) * ceil_div(in, bn));
    int s = gemm_slots(mode) / tiles;
    const int maxs = rows / (4 * mlp::BK);
    if (s > maxs) s = maxs;
    if (s > kMaxSplits) s = kMaxSplits;
    return s < 1 ? 1 : s;
}

// The reductions of one backward pass, launched together at its end: one mlp::reduce_batch launch per level
// for all of them instead of one or two launches each (the partial buffers are per layer, so nothing is
// overwritten before the flush).  Same summation orders, same bits as the separate launches.
struct Reducer {
    mlp::RedBatch b{};
    Model* m = nullptr;
    void add(const float* part, int nblk, int64_t stride, int n, float* dst, bool splits, hipStream_t s) {
        if (b.njobs == mlp::kRedJobs) flush(s);
        mlp::RedJob& J = b.j[b.njobs];
        J.part = part;
        J.dst = dst;
        J.stride = stride;
        J.nblk = nblk;
        J.n = n;
        J.mid = m->mid + (int64_t)b.njobs * 16 * m->midn;
        if (splits) {
            J.G = 1;
            J.vec = (n % 4 == 0 && stride % 4 == 0 && ((uintptr_t)part & 15) == 0 && ((uintptr_t)dst & 15) == 0) ? 1 : 2;
        } else {
            J.G = nblk >= 256 ? 16 : 1;
            J.vec = 0;
            if ((int64_t)n > m->midn) throw rlgpu::Error(RLGPU_ERR_STATE, "reduction wider than its level-1 buffer");
        }
        b.njobs++;
    }
    void flush(hipStream_t s) {
        if (!b.njobs) return;
        bool two = false;
        int t = 0;
        for (int k = 0; k < b.njobs; k++) {
            const mlp::RedJob& J = b.j[k];
            b.tile0[k] = t;
            t += J.vec == 1 ? (int)ceil_div(J.n, 4096) : J.vec == 2 ? (int)ceil_div(J.n, 1024) : (int)ceil_div(J.n, 64) * J.G;
            two |= J.vec == 0 && J.G > 1;
        }
        b.tile0[b.njobs] = t;
        b.level = 1;
        hipLaunchKernelGGL(mlp::reduce_batch, dim3(t), dim3(1024), 0, s, b);
        RLGPU_CHECK_HIP(hipGetLastError());
        if (two) {
            t = 0;
            for (int k = 0; k < b.njobs; k++) {
                const mlp::RedJob& J = b.j[k];
                b.tile0[k] = t;
                t += (J.vec == 0 && J.G > 1) ? (int)ceil_div(J.n, 64) : 0;
            }
            b.tile0[b.njobs] = t;
            b.level = 2;
            hipLaunchKernelGGL(mlp::reduce_batch, dim3(t), dim3(1024), 0, s, b);
            RLGPU_CHECK_HIP(hipGetLastError());
        }
        b.njobs = 0;
    }
};

// dW (+)= dZ^T . X  over n rows (split-K over rows into `wpart`, fixed-order reduction into grad: now, or
// through R at the end of the pass)
void weight_grad(Model& m, const float* dZ, int out, const float* X, int64_t ldx, int in, int n, float* gW, hipStream_t s,
                 bool x_tail_ok = false, const float* amax_dz = nullptr, const float* amax_x = nullptr, int64_t ldz = 0,
                 Reducer* R = nullptr, float* wpart = nullptr) {
    if (!wpart) wpart = m.wpart;
    int splits = splits_for(m.mode, n, out, in);
    int chunk = (int)ceil_div(ceil_div(n, splits), kgran(m.mode)) * kgran(m.mode);
    int z = (int)ceil_div(n, chunk);
    // ldz > out: dZ rows zero-padded to ldz floats (16-byte loads across the row end)
    {
    ktime::Span span(ktime::WGRAD_GEMM, 2.0 * out * in * (double)n, s);
    gemm_f32(m.mode, mlp::A_KI, mlp::B_KJ, dZ, ldz ? ldz : out, X, ldx, wpart, in, nullptr, out, in, n, splits, s,
             ldz > out, x_tail_ok, amax_dz, amax_x);
    }
    int64_t e = (int64_t)out * in;
    if (R) {
        R->add(wpart, z, e, (int)e, gW, true, s);
        return;
    }
    if (e % 4 == 0 && ((uintptr_t)gW & 15) == 0 && ((uintptr_t)wpart & 15) == 0)
        hipLaunchKernelGGL(mlp::reduce_splits4, dim3(ceil_div(e / 4, 256)), dim3(256), 0, s, wpart, z, e, e, gW, 1);
    else
        hipLaunchKernelGGL(mlp::reduce_splits, dim3(ceil_div(e, 256)), dim3(256), 0, s, wpart, z, e, e, gW, 1);
    RLGPU_CHECK_HIP(hipGetLastError());
}

// grad[0..n) += column sums of nblk partial rows (stride apart) -- two fixed-order levels
void reduce_partials(Model& m, const float* part, int nblk, int64_t stride, int n, float* grad, hipStream_t s) {
    const int G = nblk >= 256 ? 16 : 1;
    float* mid = m.mid;  // [16][<= 3 * max(H, 1024)]
    if (G > 1) {
        hipLaunchKernelGGL(mlp::reduce_cols, dim3(ceil_div(n, 64), G), dim3(1024), 0, s, part, nblk, stride, (int64_t)0, n,
                           mid, (int64_t)n, 0);
        hipLaunchKernelGGL(mlp::reduce_cols, dim3(ceil_div(n, 64), 1), dim3(1024), 0, s, mid, G, (int64_t)n, (int64_t)0, n,
                           grad, (int64_t)0, 1);
    } else {
        hipLaunchKernelGGL(mlp::reduce_cols, dim3(ceil_div(n, 64), 1), dim3(1024), 0, s, part, nblk, stride, (int64_t)0, n,
                           grad, (int64_t)0, 1);
    }
    RLGPU_CHECK_HIP(hipGetLastError());
}

void colsum_into(Model& m, const float* X, int n, int C, float* g, hipStream_t s) {
    int nb = (int)ceil_div(n, mlp::CS_ROWS);
    hipLaunchKernelGGL(mlp::colsum_partial, dim3(nb), dim3(256), 0, s, X, n, C, m.cpart);
    RLGPU_CHECK_HIP(hipGetLastError());
    reduce_partials(m, m.cpart, nb, C, C, g, s);
}

// row stride of a multi-column loss gradient dout [n, out]: a multiple of 4 floats (the policy loss
// writes the padding columns as zeros)
inline int dout_ld(int out) { return out > 1 ? (out + 3) / 4 * 4 : out; }

// H3 operand scale slots (null in the other modes): slot k of model m, and the gathered obs
inline float* amax_slot(Model& m, int k) { return m.mode == RLGPU_GEMM_F16X3 ? m.amax + (int64_t)k * 64 : nullptr; }
inline const float* wscale_at(const Model& m, int64_t off) {
    return m.mode == RLGPU_GEMM_F16X3 ? m.wscale + off : nullptr;
}

// A training model's input: rows of ld floats, their H3 scale shards (null outside H3), and whether
// the rows are zero-padded past the model input to a multiple of 4 (16-byte loads across the row end).
struct Input {
    const float* X;
    int64_t ld;
    const float* amax;
    bool tail_ok;
};
// the gathered minibatch obs (rows of x_ld floats, zero-padded)
inline Input obs_input(rlgpu_ppo* h) { return {h->x0, h->x_ld, h->x_amax, true}; }
// what model mi reads: the obs, or the shared head's last activation (PPOLearner.cpp:403,474)
inline Input model_input(rlgpu_ppo* h, int mi) {
    if (mi == 2 || !h->shared()) return obs_input(h);
    Model& sm = h->M[2];
    const int l = nhid(sm) - 1;
    return {sm.act[l], sm.L[l].out, amax_slot(sm, l), false};
}

// fp32 training forward of model mi on x; keeps activations; writes the output layer to `out` (the
// shared head has none: its last activation stays in m.act).
void forward_train(rlgpu_ppo* h, int mi, const Input& x, int n, float* out, hipStream_t s) {
    Model& m = h->M[mi];
    const float* P = h->params;
    if (h->split_dirty[mi]) {
        split_weights(P, m, s);
        h->split_dirty[mi] = false;
    }
    const int nh = nhid(m);
    const float* in = x.X;
    const float* in_amax = x.amax;
    int64_t ld = x.ld;
    bool tail_ok = x.tail_ok;
    const Layer* O = m.head_only ? nullptr : &m.L[nh];
    const bool head1 = O && O->out == 1 && nh > 0;  // rank-1 head fused into the last LayerNorm forward
    for (int l = 0; l < nh; l++) {
        const Layer& L = m.L[l];
        const float* gg = L.g >= 0 ? P + L.g : nullptr;
        const float* bb = L.be >= 0 ? P + L.be : nullptr;
        const bool fuse = head1 && l == nh - 1;
        if (L.sf >= 0)
            gemm_x6_pre(in, ld, m.wsplit + L.sf, L.sf_ld, (int64_t)L.sf_rows * L.sf_ld, m.xhat[l], L.out, P + L.b, n, L.out,
                        L.in, s, tail_ok, in_amax, wscale_at(m, L.sfs));
        else
            gemm_f32(m.mode, mlp::A_IK, mlp::B_JK, in, ld, P + L.w, L.in, m.xhat[l], L.out, P + L.b, n, L.out, L.in, 1, s,
                     tail_ok, false, in_amax);
        // bytes: z read, act written, (mean, rstd) written
        ktime::Span span(ktime::LN_FWD, (double)n * (8.0 * L.out + 8.0), s);
        int lnf_rows = 0;
        const auto lnf = mlp::ln_act_fwd_f32_pick(L.out, &lnf_rows, fuse);
        hipLaunchKernelGGL(lnf, dim3(ceil_div(n, lnf_rows)), dim3(256), 0, s, m.xhat[l], gg, bb, n, L.out,
                           h->cfg.leaky_slope, h->cfg.layer_norm, m.act[l], reinterpret_cast<float2*>(m.rstd[l]),
                           amax_slot(m, l), fuse ? P + O->w : nullptr, fuse ? P + O->b : nullptr, fuse ? out : nullptr);
        RLGPU_CHECK_HIP(hipGetLastError());
        in = m.act[l];
        in_amax = amax_slot(m, l);
        ld = L.out;
        tail_ok = false;
    }
    if (!O || head1) return;
    if (O->out == 1) {  // rank-1 head (critic value) of a model without hidden layers: wave-per-row dot products
        if (ld != O->in)
            throw rlgpu::Error(RLGPU_ERR_UNSUPPORTED, "a rank-1 model without hidden layers needs obs_size % 4 == 0");
        hipLaunchKernelGGL(mlp::head1_fwd_any(O->in), dim3(ceil_div(n, mlp::H1_ROWS)), dim3(256), 0, s, in, P + O->w, P + O->b, n,
                           O->in, out);
        RLGPU_CHECK_HIP(hipGetLastError());
        return;
    }
    if (O->sf >= 0)
        gemm_x6_pre(in, ld, m.wsplit + O->sf, O->sf_ld, (int64_t)O->sf_rows * O->sf_ld, out, O->out, P + O->b, n, O->out, O->in, s,
                    tail_ok, in_amax, wscale_at(m, O->sfs));
    else
        gemm_f32(m.mode, mlp::A_IK, mlp::B_JK, in, ld, P + O->w, O->in, out, O->out, P + O->b, n, O->out, O->in, 1, s, tail_ok,
                 false, in_amax);
}

// backward of model mi (input x) from dout into the grad buffer (accumulating).  dout: the loss
// gradient [n, out] of the output layer, or -- the shared head -- the gradient of its last
// activation [n, H].  dout_part: optional per-block column partials of dout (dout_nblk rows of `out`
// floats, written by the loss kernel) for the output bias, instead of a separate column-sum pass.
// H3: dout's max |x| is in slot kAmaxOut.  When m.dX is set (a model behind the shared head) the
// gradient w.r.t. the model input is written there too.
void backward(rlgpu_ppo* h, int mi, const Input& x, int n, const float* dout, hipStream_t s,
              const float* dout_part = nullptr, int dout_nblk = 0) {
    Model& m = h->M[mi];
    const float* P = h->params;
    float* G = h->grads;
    const int nh = nhid(m);
    const float* dA_top = m.dA;  // gradient of the last hidden layer's activation
    bool rank1 = false;          // rank-1 output layer folded into the last LayerNorm backward
    // the pass's bias / LayerNorm / weight-gradient reductions, launched together at its end
    Reducer red;
    red.m = &m;
    Reducer* R = &red;
    const Layer* O = m.head_only ? nullptr : &m.L[nh];
    if (!O) {
        dA_top = dout;
    } else if (O->out == 1 && nh == 0) {  // rank-1 head on the input: dA = dv w^T, dw / db partials in one pass
        if (x.ld != O->in)
            throw rlgpu::Error(RLGPU_ERR_UNSUPPORTED, "a rank-1 model without hidden layers needs obs_size % 4 == 0");
        int nb = (int)ceil_div(n, mlp::LNB_ROWS);
        hipLaunchKernelGGL(mlp::head1_bwd_any(O->in), dim3(nb), dim3(256), 0, s, x.X, P + O->w, dout, n, O->in,
                           m.dX ? m.dX : m.dA, m.cpart);
        RLGPU_CHECK_HIP(hipGetLastError());
        reduce_partials(m, m.cpart, nb, O->in + 1, O->in + 1, G + O->w, s);  // [w | b] contiguous in the flat buffer
        return;
    } else if (O->out == 1) {
        // rank-1 head after a LayerNorm: its backward recomputes dA = dv w^T and the activation, and
        // emits the head's dw / db partials (m.hpart) beside its own -- no separate head pass
        rank1 = true;
    } else {
        if (m.mode == RLGPU_GEMM_F16X3 && !dout_part)
            throw rlgpu::Error(RLGPU_ERR_STATE, "H3 backward: the loss kernel must provide dout's scale");
        // dout rows of dld floats (the policy loss pads them with zeros to a multiple of 4)
        const int dld = dout_ld(O->out);
        const Input a = nh > 0 ? Input{m.act[nh - 1], O->in, amax_slot(m, nh - 1), false} : x;
        weight_grad(m, dout, O->out, a.X, a.ld, O->in, n, G + O->w, s, a.tail_ok, amax_slot(m, kAmaxOut), a.amax, dld, R,
                    m.wpart_l[nh]);
        if (dout_part)
            R->add(dout_part, dout_nblk, O->out, O->out, G + O->b, false, s);
        else if (dld == O->out)
            colsum_into(m, dout, n, O->out, G + O->b, s);
        else
            throw rlgpu::Error(RLGPU_ERR_STATE, "backward: padded dout needs the loss kernel's bias partials");
        // dA = dout . W_out (into the input gradient when the output layer reads the model input)
        float* dA = nh > 0 ? m.dA : m.dX;
        if (dA) {
            if (O->sb >= 0)
                gemm_x6_pre(dout, dld, m.wsplit + O->sb, O->sb_ld, (int64_t)O->sb_rows * O->sb_ld, dA, O->in, nullptr, n, O->in,
                            O->out, s, dld > O->out, amax_slot(m, kAmaxOut), wscale_at(m, O->sbs));
            else
                gemm_f32(m.mode, mlp::A_IK, mlp::B_KJ, dout, dld, P + O->w, O->in, dA, O->in, nullptr, n, O->in, O->out, 1, s,
                         dld > O->out, false, amax_slot(m, kAmaxOut), nullptr);
        }
    }
    for (int l = nh - 1; l >= 0; l--) {
        const Layer& L = m.L[l];
        const float* gg = L.g >= 0 ? P + L.g : nullptr;
        const float* bb = L.be >= 0 ? P + L.be : nullptr;
        const bool r1 = rank1 && l == nh - 1;  // dA of the rank-1 head, recomputed in the kernel
        int lnb_rows = 0;
        const auto lnb = mlp::ln_act_bwd_pick(L.out, r1, &lnb_rows);
        const float* dA_in = l == nh - 1 ? dA_top : m.dA;
        float* dz = m.dZ;  // this layer's dZ
        const int nb = (int)ceil_div(n, lnb_rows);
        {
            // bytes: dA (recomputed for the rank-1 head: its dv instead), z, stats read; dZ written
            ktime::Span span(ktime::LN_BWD, (double)n * ((r1 ? 4.0 : 4.0 * L.out) + 8.0 * L.out + 8.0), s);
            hipLaunchKernelGGL(lnb, dim3(nb), dim3(256), 0, s, r1 ? nullptr : dA_in, m.xhat[l],
                               reinterpret_cast<const float2*>(m.rstd[l]), gg, bb, n, L.out, h->cfg.leaky_slope,
                               h->cfg.layer_norm, m.dZ, m.cpart_l[l], amax_slot(m, kAmaxDZ + l), r1 ? dout : nullptr,
                               r1 ? P + O->w : nullptr, r1 ? m.hpart : nullptr);
            RLGPU_CHECK_HIP(hipGetLastError());
        }
        // partials [blk][dbias | dgamma | dbeta] -> flat grads [b][g][be] (contiguous after L.b); the rank-1
        // head's [w | b] are contiguous too
        int ncol = h->cfg.layer_norm ? 3 * L.out : L.out;
        if (r1) R->add(m.hpart, nb, O->in + 1, O->in + 1, G + O->w, false, s);
        R->add(m.cpart_l[l], nb, 3 * (int64_t)L.out, ncol, G + L.b, false, s);
        const Input a = l > 0 ? Input{m.act[l - 1], L.in, amax_slot(m, l - 1), false} : x;
        weight_grad(m, dz, L.out, a.X, a.ld, L.in, n, G + L.w, s, a.tail_ok, amax_slot(m, kAmaxDZ + l), a.amax, 0, R,
                    m.wpart_l[l]);
        float* dA = l > 0 ? m.dA : m.dX;  // the first layer's only when the input gradient is wanted
        if (!dA) continue;
        if (L.sb >= 0)
            gemm_x6_pre(dz, L.out, m.wsplit + L.sb, L.sb_ld, (int64_t)L.sb_rows * L.sb_ld, dA, L.in, nullptr, n, L.in,
                        L.out, s, false, amax_slot(m, kAmaxDZ + l), wscale_at(m, L.sbs));
        else
            gemm_f32(m.mode, mlp::A_IK, mlp::B_KJ, dz, L.out, P + L.w, L.in, dA, L.in, nullptr, n, L.in, L.out, 1, s, false,
                     false, amax_slot(m, kAmaxDZ + l), nullptr);
    }
    red.flush(s);
}

void gather_obs(rlgpu_ppo* h, const float* obs, const int32_t* idx, int64_t start, int n, hipStream_t s) {
    int64_t e = (int64_t)n * h->x_ld;
    // H3: clear every operand-scale slot of this pass, then the gather fills the obs slot
    if (h->amax_all) RLGPU_CHECK_HIP(hipMemsetAsync(h->amax_all, 0, h->amax_count * sizeof(float), s));
    hipLaunchKernelGGL(mlp::gather_rows, dim3(std::min<int64_t>(ceil_div(e, 256), mlp::GATHER_BLOCKS)), dim3(256), 0, s, obs,
                       h->cfg.obs_size, idx, start, n, h->x0, h->x_ld, h->x_amax);
    RLGPU_CHECK_HIP(hipGetLastError());
}

// The Linear layers a 16-bit forward of model mi runs through: the shared head's first (for the
// policy / critic), then the model's -- Model::Forward chained as InferPolicyProbsFromModels /
// InferCritic do (PPOLearner.cpp:90-91,188-191).  The shared head's f32 output re-enters the policy
// as bf16 (Models.cpp:64), which is exact, so the chain is one 16-bit network.
struct Link {
    const Layer* L;
    bool hidden;  // [Linear -> LayerNorm -> LeakyReLU]; false: the output Linear
};
std::vector<Link> chain(const rlgpu_ppo* h, int mi) {
    std::vector<Link> c;
    if (mi != 2 && h->shared())
        for (auto& L : h->M[2].L) c.push_back({&L, true});
    const Model& m = h->M[mi];
    for (size_t l = 0; l < m.L.size(); l++) c.push_back({&m.L[l], m.head_only || l + 1 < m.L.size()});
    return c;
}

// bf16 inference forward of n rows through chain(mi); returns the 16-bit result [n, out] (h->logits_h
// after an output Linear, else the last activation buffer).  Model::Forward with halfPrec
// (Models.cpp:42-68): every module runs on the bf16 copy, activations rounded to bf16.
const uint16_t* forward_half(rlgpu_ppo* h, int mi, const float* X, int n, hipStream_t s, const uint16_t* weights = nullptr) {
    const uint16_t* P = weights ? weights : h->half;
    const auto c = chain(h, mi);
    {
        int64_t e = (int64_t)n * h->xh_ld;
        RLGPU_H16_LAUNCH(f16(h), mlp::rows_to_bf16, dim3(ceil_div(e, 256)), dim3(256), 0, s, X, h->cfg.obs_size, n, h->xh,
                         h->xh_ld);
        RLGPU_CHECK_HIP(hipGetLastError());
    }
    const uint16_t* in = h->xh;
    int64_t ld = h->xh_ld;
    int cur = 0;
    for (const Link& k : c) {
        const Layer& L = *k.L;
        mlp::HGemmArgs g;
        g.A = in;
        g.B = P + L.hw;
        g.bias = P + L.hb;
        g.C = k.hidden ? h->zh : h->logits_h;
        g.lda = ld;
        g.ldb = L.in_pad;
        g.ldc = L.out;
        g.I = n;
        g.J = L.out;
        g.K = L.in_pad;
        g.gx = (int)ceil_div(L.out, mlp::BN);
        g.gy = (int)ceil_div(n, mlp::BM);
        RLGPU_H16_LAUNCH(f16(h), mlp::gemm_bf16, dim3(g.gx * g.gy), dim3(256), 0, s, g);
        RLGPU_CHECK_HIP(hipGetLastError());
        if (!k.hidden) return h->logits_h;
        const uint16_t* gg = L.hg >= 0 ? P + L.hg : nullptr;
        const uint16_t* bb = L.hbe >= 0 ? P + L.hbe : nullptr;
        hipLaunchKernelGGL(f16(h) ? mlp::ln_act_fwd_bf16_any<true>(L.out) : mlp::ln_act_fwd_bf16_any<false>(L.out), dim3(ceil_div(n, mlp::LNF_ROWS)), dim3(256), 0, s, h->zh, gg, bb, n, L.out,
                           h->cfg.leaky_slope, h->cfg.layer_norm, h->ah[cur]);
        RLGPU_CHECK_HIP(hipGetLastError());
        in = h->ah[cur];
        ld = L.out;
        cur ^= 1;
    }
    return in;
}

// Fused inference (infer::mlp_infer): one launch per forward when every layer fits the kernel's
// LDS tile (inputs / hidden widths <= 512, outputs <= 128); RLGPU_FUSED_INFER=0 selects the
// layer-by-layer path (forward_half), which computes the same bits.
unsigned long long* g_infer_trace = nullptr;  // rlgpu_debug_infer_trace
int64_t g_infer_trace_cap = 0;             // its capacity (uint64 entries)
bool fused_ok(const rlgpu_ppo* h, int mi) {
    if (infer_f32(h)) return false;  // fp32 inference runs the training forward (forward_f32)
    const char* e = getenv("RLGPU_FUSED_INFER");
    if (e && atoi(e) == 0) return false;
    const auto c = chain(h, mi);
    if ((int)c.size() > infer::kMaxLinear || c.back().hidden) return false;  // the kernel ends on an output Linear
    for (size_t l = 0; l < c.size(); l++) {
        if (c[l].L->in > infer::IMAX) return false;
        if (c[l].L->out > (l + 1 < c.size() ? infer::IMAX : infer::IOUT)) return false;
    }
    return true;
}

// one fused forward over n rows of X with the 16-bit copy P: mode 0 writes f32 outputs to out_f,
// mode 1 samples actions (masks, act, logp; row_sel / sel as ppo::sample_actions)
void infer_fused(rlgpu_ppo* h, int mi, bool ver, const float* X, int n, int mode, float* out_f,
                 const uint8_t* masks, int det, uint64_t step, int32_t* act, float* logp, const uint8_t* row_sel, int sel,
                 hipStream_t s, int64_t row0 = 0) {
    const auto c = chain(h, mi);
    infer::InferArgs a{};
    a.X = X;
    a.n = n;
    a.in = h->cfg.obs_size;
    a.P = ver ? h->half_ver : h->half;
    a.F = ver ? h->frag_ver : h->frag;
    a.nl = (int)c.size();
    a.width[0] = a.in;
    for (int l = 0; l < a.nl; l++) {
        const Layer& L = *c[l].L;
        a.width[l + 1] = L.out;
        a.fw[l] = L.fw;
        a.hb[l] = L.hb;
        a.hg[l] = L.hg;
        a.hbe[l] = L.hbe;
    }
    a.slope = h->cfg.leaky_slope;
    a.use_ln = h->cfg.layer_norm;
    a.mode = mode;
    a.out_f = out_f;
    a.masks = masks;
    a.det = det;
    a.seed = h->cfg.seed;
    a.step = step;
    a.row0 = row0;
    a.act = act;
    a.logp = logp;
    a.row_sel = row_sel;
    a.sel = sel;
    a.trace = g_infer_trace;
    if (a.trace && ceil_div(n, infer::IR) * 16 > g_infer_trace_cap)
        throw rlgpu::Error(RLGPU_ERR_INVALID_ARG, "rlgpu_debug_infer_trace: buffer of " + std::to_string(g_infer_trace_cap) +
                                                      " entries, this launch needs " + std::to_string(ceil_div(n, infer::IR) * 16));
    RLGPU_H16_LAUNCH(f16(h), infer::mlp_infer, dim3(ceil_div(n, infer::IR)), dim3(infer::IT), 0, s, a);
    RLGPU_CHECK_HIP(hipGetLastError());
}

// Model layout in the flat buffers.  out = 0: the shared head (hidden layers only, PPOLearner.cpp:56-64);
// input_grad: the model reads the shared head's output, so its first layer also gets the transposed
// weight planes for the input gradient.
void build_model(rlgpu_ppo* h, Model& m, int in, const int32_t* layers, int nl, int out, float lr, bool input_grad = false) {
    m.head_only = out == 0;
    if (m.head_only) nl--;  // the last hidden layer takes the output layer's slot in the loop below
    m.in = in;
    m.out = m.head_only ? layers[nl] : out;
    m.lr = lr;
    m.mode = h->cfg.train_gemm;
    m.off = h->nparams;
    int prev = in;
    for (int l = 0; l <= nl; l++) {
        Layer L;
        L.in = prev;
        const bool hidden = l < nl || m.head_only;
        L.out = l < nl ? layers[l] : m.out;
        L.w = h->nparams;
        h->nparams += (int64_t)L.in * L.out;
        L.b = h->nparams;
        h->nparams += L.out;
        L.g = L.be = -1;
        if (hidden && h->cfg.layer_norm) {
            L.g = h->nparams;
            h->nparams += L.out;
            L.be = h->nparams;
            h->nparams += L.out;
        }
        L.in_pad = (L.in + 7) / 8 * 8;
        h->nhalf = (h->nhalf + 7) / 8 * 8;
        L.hw = h->nhalf;
        h->nhalf += (int64_t)L.out * L.in_pad;
        L.hb = h->nhalf;
        h->nhalf += L.out;
        L.hg = L.hbe = -1;
        L.fw = h->nfrag;
        h->nfrag += infer::frag_size(L.out, L.in);
        if (L.g >= 0) {
            L.hg = h->nhalf;
            h->nhalf += L.out;
            L.hbe = h->nhalf;
            h->nhalf += L.out;
        }
        if (L.out > h->hmax) h->hmax = L.out;
        if (L.in > h->hmax && l > 0) h->hmax = L.in;
        if (split_mode(m.mode) && L.out > 1) {  // the rank-1 critic head has no GEMM
            const int np = m.mode == RLGPU_GEMM_F16X3 ? 2 : 3;  // planes per split weight
            const int rpad = m.mode == RLGPU_GEMM_F16X3 ? mlp::BNW : mlp::BN;  // rows: whole B tiles
            L.sf_rows = (int)ceil_div(L.out, rpad) * rpad;
            L.sf_ld = (int)ceil_div(L.in, mlp::XKMAX) * mlp::XKMAX;
            L.sf = m.nsplit;
            m.nsplit += np * (int64_t)L.sf_rows * L.sf_ld;
            L.sfs = m.nscale;
            m.nscale += L.sf_rows;
            if (l > 0 || input_grad) {  // dA of the first layer only behind the shared head
                L.sb_rows = (int)ceil_div(L.in, rpad) * rpad;
                L.sb_ld = (int)ceil_div(L.out, mlp::XKMAX) * mlp::XKMAX;
                L.sb = m.nsplit;
                m.nsplit += np * (int64_t)L.sb_rows * L.sb_ld;
                L.sbs = m.nscale;
                m.nscale += L.sb_rows;
            }
        }
        m.L.push_back(L);
        prev = L.out;
    }
    m.count = h->nparams - m.off;
}

void sumsq_coef(rlgpu_ppo* h, const float* x, int64_t n, float max_norm, float* coef, float* norm_out, hipStream_t s) {
    const int nb = 512;
    hipLaunchKernelGGL(ppo::sumsq_partial, dim3(nb), dim3(256), 0, s, x, n, h->scratch);
    hipLaunchKernelGGL(ppo::clip_coef, dim3(1), dim3(64), 0, s, h->scratch, nb, max_norm, coef, norm_out);
    RLGPU_CHECK_HIP(hipGetLastError());
}

// bf16 inference copy of model mi from `src` (the model's flat fp32 parameters, torch order) into
// the padded layout at `dst` (h->half or h->half_ver)
void half_from(rlgpu_ppo* h, int mi, const float* src, uint16_t* dst, uint16_t* fdst, hipStream_t s) {
    const Model& m = h->M[mi];
    for (auto& L : m.L) {
        const int64_t nf = infer::frag_size(L.out, L.in);
        RLGPU_H16_LAUNCH(f16(h), infer::weight_to_frag, dim3(ceil_div(nf, 256)), dim3(256), 0, s, src + (L.w - m.off),
                         L.out, L.in, fdst + L.fw);
        int64_t e = (int64_t)L.out * L.in_pad;
        RLGPU_H16_LAUNCH(f16(h), mlp::weight_to_bf16, dim3(ceil_div(e, 256)), dim3(256), 0, s, src + (L.w - m.off), L.out, L.in,
                           dst + L.hw, L.in_pad);
        int nv = L.g >= 0 ? 3 * L.out : L.out;  // bias | LN weight | LN bias, contiguous in both layouts
        RLGPU_H16_LAUNCH(f16(h), ppo::to_half, dim3(ceil_div(nv, 256)), dim3(256), 0, s, src + (L.b - m.off), dst + L.hb,
                           (int64_t)nv);
    }
    RLGPU_CHECK_HIP(hipGetLastError());
}

void refresh_half(rlgpu_ppo* h, hipStream_t s) {
    for (int mi = 0; mi < h->nm; mi++) {
        half_from(h, mi, h->params + h->M[mi].off, h->half, h->frag, s);
        h->split_dirty[mi] = true;
    }
}

}  // namespace

extern "C" int rlgpu_ppo_create(const rlgpu_ppo_config* cfg, rlgpu_ppo** out) {
    return rlgpu::guarded([&] {
        RLGPU_REQUIRE(cfg && out, "rlgpu_ppo_create: null argument");
        RLGPU_REQUIRE(cfg->obs_size > 0 && cfg->num_actions > 0 && cfg->num_actions <= ppo::kMaxA,
                      "num_actions must be in [1, 128]");
        RLGPU_REQUIRE(cfg->n_policy_layers >= 1 && cfg->n_policy_layers <= RLGPU_MAX_LAYERS && cfg->n_critic_layers >= 1 &&
                          cfg->n_critic_layers <= RLGPU_MAX_LAYERS,
                      "1..8 hidden layers per model");
        RLGPU_REQUIRE(cfg->max_rows > 0, "max_rows must be > 0");
        for (int i = 0; i < cfg->n_policy_layers; i++)
            RLGPU_REQUIRE(cfg->policy_layers[i] > 0 && cfg->policy_layers[i] <= 2048, "hidden sizes must be in [1, 2048]");
        for (int i = 0; i < cfg->n_critic_layers; i++)
            RLGPU_REQUIRE(cfg->critic_layers[i] > 0 && cfg->critic_layers[i] <= 2048, "hidden sizes must be in [1, 2048]");
        RLGPU_REQUIRE(cfg->n_shared_layers >= 0 && cfg->n_shared_layers <= RLGPU_MAX_LAYERS, "0..8 shared-head layers");
        for (int i = 0; i < cfg->n_shared_layers; i++)
            RLGPU_REQUIRE(cfg->shared_layers[i] > 0 && cfg->shared_layers[i] <= 2048, "hidden sizes must be in [1, 2048]");
        auto* h = new rlgpu_ppo();
        try {
            h->cfg = *cfg;
            const bool sh = cfg->n_shared_layers > 0;
            h->nm = sh ? 3 : 2;
            // PPOLearner::MakeModels (PPOLearner.cpp:42-74): behind a shared head the policy / critic
            // take its last width as input
            const int min = sh ? cfg->shared_layers[cfg->n_shared_layers - 1] : cfg->obs_size;
            build_model(h, h->M[0], min, cfg->policy_layers, cfg->n_policy_layers, cfg->num_actions, cfg->policy_lr, sh);
            h->nparams = (h->nparams + 63) / 64 * 64;  // 256-byte aligned model start: float4 weight rows
            build_model(h, h->M[1], min, cfg->critic_layers, cfg->n_critic_layers, 1, cfg->critic_lr, sh);
            if (sh) {  // shared head LR = min(policy, critic) (PPOLearner::SetLearningRates, :652-663)
                h->nparams = (h->nparams + 63) / 64 * 64;
                build_model(h, h->M[2], cfg->obs_size, cfg->shared_layers, cfg->n_shared_layers, 0,
                            std::min(cfg->policy_lr, cfg->critic_lr));
            }
            int64_t P = h->nparams, R = cfg->max_rows;
            h->params = h->alloc<float>(P);
            h->grads = h->alloc<float>(P);
            h->exp_avg = h->alloc<float>(P);
            h->exp_avg_sq = h->alloc<float>(P);
            h->half = h->alloc<uint16_t>(h->nhalf + 8);
            h->half_ver = h->alloc<uint16_t>(h->nhalf + 8);
            h->frag = h->alloc<uint16_t>(h->nfrag);
            h->frag_ver = h->alloc<uint16_t>(h->nfrag);
            RLGPU_CHECK_HIP(hipMemset(h->params, 0, P * 4));
            RLGPU_CHECK_HIP(hipMemset(h->grads, 0, P * 4));
            RLGPU_CHECK_HIP(hipMemset(h->exp_avg, 0, P * 4));
            RLGPU_CHECK_HIP(hipMemset(h->exp_avg_sq, 0, P * 4));
            for (int mi = 0; mi < h->nm; mi++) {
                Model& m = h->M[mi];
                const int nh = nhid(m);
                for (int l = 0; l < nh; l++) {
                    m.xhat.push_back(h->alloc<float>(R * m.L[l].out));
                    m.act.push_back(h->alloc<float>(R * m.L[l].out));
                    m.rstd.push_back(h->alloc<float>(2 * R));  // (mean, rstd) per row
                }
            }
            int H = h->hmax;
            int omax = cfg->num_actions > 1 ? cfg->num_actions : 1;
            int64_t wmax = 0, wpart_max = 0;
            {
                int dev = 0, cus = 256;
                if (hipGetDevice(&dev) == hipSuccess) {
                    hipDeviceProp_t prop;
                    if (hipGetDeviceProperties(&prop, dev) == hipSuccess && prop.multiProcessorCount > 0)
                        cus = prop.multiProcessorCount;
                }
                g_cus = cus;
            }
            for (int mi = 0; mi < h->nm; mi++)
                for (auto& L : h->M[mi].L) {
                    const Model& m = h->M[mi];
                    wmax = std::max<int64_t>(wmax, (int64_t)L.in * L.out);
                    // splits_for is non-decreasing in the row count, and z = ceil(n / chunk) <= splits
                    wpart_max = std::max<int64_t>(wpart_max, (int64_t)splits_for(m.mode, (int)R, L.out, L.in) * L.in * L.out);
                }
            int64_t nb = ceil_div(R, std::min(std::min(mlp::LNB_ROWS_MIN, mlp::CS_ROWS), ppo::PL_ROWS));
            for (int mi = 0; mi < h->nm; mi++) {
                Model& m = h->M[mi];
                if (!m.head_only) {
                    m.y = h->alloc<float>(R * omax);
                    m.dy = h->alloc<float>(R * ((omax + 3) / 4 * 4));
                }
                if (sh && mi < 2) m.dX = h->alloc<float>(R * (int64_t)m.in);  // input gradient behind the shared head
                m.dA = h->alloc<float>(R * H);
                m.dZ = h->alloc<float>(R * H);
                m.wpart = h->alloc<float>(wpart_max);
                m.cpart = h->alloc<float>(nb * 3 * std::max(H, omax) + nb);
                m.hpart = h->alloc<float>(nb * ((int64_t)H + 1));
                // the deferred reductions' per-layer partials and level-1 rows (Reducer)
                for (auto& L : m.L) {
                    m.wpart_l.push_back(h->alloc<float>((int64_t)splits_for(m.mode, (int)R, L.out, L.in) * L.in * L.out));
                    m.cpart_l.push_back(h->alloc<float>(nb * 3 * (int64_t)L.out));
                }
                m.lpart = h->alloc<float>(nb * (int64_t)omax);
                m.midn = 3 * (int64_t)std::max(std::max(H, omax) + 1, 1024);
                m.mid = h->alloc<float>((int64_t)mlp::kRedJobs * 16 * m.midn);
                if (m.nsplit) m.wsplit = h->alloc<uint16_t>(m.nsplit);
                if (m.mode == RLGPU_GEMM_F16X3 && m.nscale) m.wscale = h->alloc<float>(m.nscale);
            }
            if (sh) h->dshared = h->alloc<float>(R * (int64_t)h->M[2].out);
            if (cfg->train_gemm == RLGPU_GEMM_F16X3) {  // operand-scale shards: every model's slots + the obs
                h->amax_count = (3 * (int64_t)kAmaxSlots + 1) * 64;
                h->amax_all = h->alloc<float>(h->amax_count);
                RLGPU_CHECK_HIP(hipMemset(h->amax_all, 0, h->amax_count * sizeof(float)));
                for (int mi = 0; mi < 3; mi++) h->M[mi].amax = h->amax_all + (int64_t)mi * kAmaxSlots * 64;
                h->x_amax = h->amax_all + 3 * (int64_t)kAmaxSlots * 64;
            }
            RLGPU_CHECK_HIP(hipStreamCreateWithFlags(&h->aux, hipStreamNonBlocking));
            RLGPU_CHECK_HIP(hipEventCreateWithFlags(&h->ev_fork, hipEventDisableTiming));
            RLGPU_CHECK_HIP(hipEventCreateWithFlags(&h->ev_join, hipEventDisableTiming));
            h->scratch = h->alloc<float>(2048 + 16 * 3 * 1024);
            h->x_ld = (cfg->obs_size + 3) / 4 * 4;
            h->x0 = h->alloc<float>(R * h->x_ld);
            h->xh_ld = (cfg->obs_size + 7) / 8 * 8;
            h->xh = h->alloc<uint16_t>(R * h->xh_ld);
            h->zh = h->alloc<uint16_t>(R * H);
            h->ah[0] = h->alloc<uint16_t>(R * H);
            h->ah[1] = h->alloc<uint16_t>(R * H);
            h->logits_h = h->alloc<uint16_t>(R * omax);
            if (cfg->infer_fp16 == RLGPU_INFER_F32) h->logits_f = h->alloc<float>(R * omax);
            *out = h;
        } catch (...) {
            for (void* p : h->allocs) (void)hipFree(p);
            delete h;
            throw;
        }
    });
}

extern "C" int rlgpu_ppo_destroy(rlgpu_ppo* h) {
    return rlgpu::guarded([&] {
        if (!h) return;
        if (h->aux) (void)hipStreamSynchronize(h->aux);
        if (h->ev_fork) (void)hipEventDestroy(h->ev_fork);
        if (h->ev_join) (void)hipEventDestroy(h->ev_join);
        if (h->aux) (void)hipStreamDestroy(h->aux);
        for (void* p : h->allocs) (void)hipFree(p);
        delete h;
    });
}

extern "C" int rlgpu_ppo_buffers(rlgpu_ppo* h, float** d_params, float** d_grads, int64_t* num_params) {
    return rlgpu::guarded([&] {
        RLGPU_REQUIRE(h, "null handle");
        if (d_params) *d_params = h->params;
        if (d_grads) *d_grads = h->grads;
        if (num_params) *num_params = h->nparams;
    });
}

extern "C" int rlgpu_ppo_model_range(rlgpu_ppo* h, int32_t model, int64_t* offset, int64_t* count) {
    return rlgpu::guarded([&] {
        RLGPU_REQUIRE(h && model >= 0 && model <= 2, "model must be 0 (policy), 1 (critic) or 2 (shared head)");
        const bool present = model < h->nm;
        if (offset) *offset = present ? h->M[model].off : h->nparams;
        if (count) *count = present ? h->M[model].count : 0;
    });
}

extern "C" int rlgpu_ppo_init_params(rlgpu_ppo* h, uint64_t seed, void* stream) {
    return rlgpu::guarded([&] {
        RLGPU_REQUIRE(h, "null handle");
        hipStream_t s = rlgpu::as_stream(stream);
        uint32_t sid = 0;  // Philox stream per tensor, in model order (policy, critic, shared head)
        for (int mi = 0; mi < h->nm; mi++)
            for (auto& L : h->M[mi].L) {
                float bound = 1.f / std::sqrt((float)L.in);
                int64_t nw = (int64_t)L.in * L.out;
                hipLaunchKernelGGL(ppo::init_uniform, dim3(ceil_div(nw, 256)), dim3(256), 0, s, h->params + L.w, nw, bound, seed,
                                   sid++);
                hipLaunchKernelGGL(ppo::init_uniform, dim3(ceil_div(L.out, 256)), dim3(256), 0, s, h->params + L.b,
                                   (int64_t)L.out, bound, seed, sid++);
                if (L.g >= 0) {
                    hipLaunchKernelGGL(ppo::fill, dim3(ceil_div(L.out, 256)), dim3(256), 0, s, h->params + L.g, (int64_t)L.out,
                                       1.f);
                    hipLaunchKernelGGL(ppo::fill, dim3(ceil_div(L.out, 256)), dim3(256), 0, s, h->params + L.be, (int64_t)L.out,
                                       0.f);
                }
            }
        RLGPU_CHECK_HIP(hipGetLastError());
        refresh_half(h, s);
    });
}

extern "C" int rlgpu_ppo_refresh_half(rlgpu_ppo* h, void* stream) {
    return rlgpu::guarded([&] {
        RLGPU_REQUIRE(h, "null handle");
        refresh_half(h, rlgpu::as_stream(stream));
    });
}

// fp32 forward of model 0 or 1 (through the shared head, if any) on n <= max_rows rows of X into out:
// the training forward's arithmetic (rlgpu_ppo_forward precision 0, and the fp32 inference)
void forward_f32(rlgpu_ppo* h, int model, const float* X, int n, float* out, hipStream_t s) {
    gather_obs(h, X, nullptr, 0, n, s);
    if (h->shared()) forward_train(h, 2, obs_input(h), n, nullptr, s);
    forward_train(h, model, model_input(h, model), n, out, s);
}

extern "C" int rlgpu_ppo_forward(rlgpu_ppo* h, int32_t model, int32_t precision, const float* d_in, int32_t n, float* d_out,
                                 void* stream) {
    return rlgpu::guarded([&] {
        RLGPU_REQUIRE(h && d_in && d_out, "null argument");
        RLGPU_REQUIRE(model >= 0 && model < h->nm, "model must be 0, 1 or (with a shared head) 2");
        RLGPU_REQUIRE(n >= 0 && n <= h->cfg.max_rows, "n must be in [0, max_rows]");
        if (n == 0) return;
        hipStream_t s = rlgpu::as_stream(stream);
        const int64_t e = (int64_t)n * h->M[model].out;
        if (precision == 0) {
            if (model == 2) {  // the shared head's last activation
                gather_obs(h, d_in, nullptr, 0, n, s);
                forward_train(h, 2, obs_input(h), n, nullptr, s);
                RLGPU_CHECK_HIP(hipMemcpyAsync(d_out, model_input(h, 0).X, e * sizeof(float), hipMemcpyDeviceToDevice, s));
            } else {
                forward_f32(h, model, d_in, n, d_out, s);
            }
        } else if (fused_ok(h, model)) {
            infer_fused(h, model, false, d_in, n, 0, d_out, nullptr, 0, 0, nullptr, nullptr, nullptr, 0, s);
        } else {
            const uint16_t* y = forward_half(h, model, d_in, n, s);
            RLGPU_H16_LAUNCH(f16(h), ppo::bf16_to_f32, dim3(ceil_div(e, 256)), dim3(256), 0, s, y, d_out, e);
            RLGPU_CHECK_HIP(hipGetLastError());
        }
    });
}

extern "C" int rlgpu_ppo_infer_actions(rlgpu_ppo* h, const float* d_obs, const uint8_t* d_masks, int32_t n,
                                       int32_t deterministic, uint64_t rng_step, int32_t* d_actions, float* d_logp,
                                       void* stream) {
    return rlgpu::guarded([&] {
        RLGPU_REQUIRE(h && d_obs && d_masks && d_actions, "null argument");
        RLGPU_REQUIRE(n >= 0, "n must be >= 0");
        hipStream_t s = rlgpu::as_stream(stream);
        int R = h->cfg.max_rows;
        for (int64_t b = 0; b < n; b += R) {
            int m = (int)std::min<int64_t>(R, n - b);
            if (infer_f32(h)) {  // useHalfPrecision = false: fp32 logits, the same sampler
                forward_f32(h, 0, d_obs + b * h->cfg.obs_size, m, h->logits_f, s);
                hipLaunchKernelGGL((ppo::sample_actions<false, float>), dim3(ceil_div(m, 4)), dim3(256), 0, s, h->logits_f,
                                   d_masks + b * h->cfg.num_actions, m, h->cfg.num_actions, deterministic, h->cfg.seed,
                                   rng_step, b + h->cfg.sample_row_offset, d_actions + b, d_logp ? d_logp + b : nullptr,
                                   nullptr, 0);
                RLGPU_CHECK_HIP(hipGetLastError());
                continue;
            }
            if (fused_ok(h, 0)) {
                infer_fused(h, 0, false, d_obs + b * h->cfg.obs_size, m, 1, nullptr, d_masks + b * h->cfg.num_actions,
                            deterministic, rng_step, d_actions + b, d_logp ? d_logp + b : nullptr, nullptr, 0, s,
                            b + h->cfg.sample_row_offset);
                continue;
            }
            forward_half(h, 0, d_obs + b * h->cfg.obs_size, m, s);
            RLGPU_H16_LAUNCH(f16(h), ppo::sample_actions, dim3(ceil_div(m, 4)), dim3(256), 0, s, h->logits_h,
                               d_masks + b * h->cfg.num_actions, m, h->cfg.num_actions, deterministic, h->cfg.seed,
                               rng_step, b + h->cfg.sample_row_offset, d_actions + b, d_logp ? d_logp + b : nullptr);
            RLGPU_CHECK_HIP(hipGetLastError());
        }
    });
}

extern "C" int rlgpu_debug_infer_trace(void* d_buf, int64_t capacity) {
    return rlgpu::guarded([&] {
        RLGPU_REQUIRE(!d_buf || capacity >= 16, "rlgpu_debug_infer_trace: capacity below one workgroup's 16 marks");
        g_infer_trace = (unsigned long long*)d_buf;
        g_infer_trace_cap = d_buf ? capacity : 0;
    });
}

extern "C" int rlgpu_ppo_set_version(rlgpu_ppo* h, const float* d_policy_params, void* stream) {
    return rlgpu::guarded([&] {
        RLGPU_REQUIRE(h && d_policy_params, "rlgpu_ppo_set_version: null argument");
        hipStream_t s = rlgpu::as_stream(stream);
        half_from(h, 0, d_policy_params, h->half_ver, h->frag_ver, s);
        // the version's shared head follows its policy (GetPolicyModels, PPOLearner.cpp:665-674)
        if (h->shared()) half_from(h, 2, d_policy_params + h->M[0].count, h->half_ver, h->frag_ver, s);
        h->has_ver = true;
    });
}

extern "C" int rlgpu_ppo_infer_actions_mixed(rlgpu_ppo* h, const float* d_obs, const uint8_t* d_masks, int32_t n,
                                             int32_t deterministic, uint64_t rng_step, const uint8_t* d_old_rows,
                                             int32_t* d_actions, float* d_logp, void* stream) {
    return rlgpu::guarded([&] {
        RLGPU_REQUIRE(h && d_obs && d_masks && d_actions && d_old_rows, "null argument");
        RLGPU_REQUIRE(h->has_ver, "rlgpu_ppo_infer_actions_mixed: no version set (rlgpu_ppo_set_version)");
        if (infer_f32(h))
            throw rlgpu::Error(RLGPU_ERR_UNSUPPORTED, "rlgpu_ppo_infer_actions_mixed: fp32 inference (RLGPU_INFER_F32) "
                                                      "keeps no old-version copy (self-play needs 16-bit inference)");
        RLGPU_REQUIRE(n >= 0, "n must be >= 0");
        hipStream_t s = rlgpu::as_stream(stream);
        int R = h->cfg.max_rows;
        for (int64_t b = 0; b < n; b += R) {
            int m = (int)std::min<int64_t>(R, n - b);
            for (int old = 0; old < 2; old++) {  // current policy rows, then the old version's rows
                if (fused_ok(h, 0)) {
                    infer_fused(h, 0, old != 0, d_obs + b * h->cfg.obs_size, m, 1, nullptr,
                                d_masks + b * h->cfg.num_actions, deterministic, rng_step, d_actions + b,
                                (d_logp && !old) ? d_logp + b : nullptr, d_old_rows + b, old, s,
                                b + h->cfg.sample_row_offset);
                    continue;
                }
                forward_half(h, 0, d_obs + b * h->cfg.obs_size, m, s, old ? h->half_ver : h->half);
                RLGPU_H16_LAUNCH(f16(h), ppo::sample_actions, dim3(ceil_div(m, 4)), dim3(256), 0, s, h->logits_h,
                                   d_masks + b * h->cfg.num_actions, m, h->cfg.num_actions, deterministic, h->cfg.seed,
                                   rng_step, b + h->cfg.sample_row_offset, d_actions + b,
                                   (d_logp && !old) ? d_logp + b : nullptr, d_old_rows + b, old);
                RLGPU_CHECK_HIP(hipGetLastError());
            }
        }
    });
}

extern "C" int rlgpu_ppo_infer_actions_rows(rlgpu_ppo* h, const float* d_obs, const uint8_t* d_masks, int32_t n, int64_t row0,
                                            int32_t deterministic, uint64_t rng_step, const uint8_t* d_old_rows,
                                            int32_t* d_actions, float* d_logp, void* stream) {
    return rlgpu::guarded([&] {
        RLGPU_REQUIRE(h && d_obs && d_masks && d_actions, "null argument");
        RLGPU_REQUIRE(n >= 0 && row0 >= 0, "n and row0 must be >= 0");
        RLGPU_REQUIRE(!d_old_rows || h->has_ver, "rlgpu_ppo_infer_actions_rows: old rows without a version set");
        if (!fused_ok(h, 0))
            throw rlgpu::Error(RLGPU_ERR_UNSUPPORTED, "rlgpu_ppo_infer_actions_rows: the policy is not on the fused kernel "
                                                      "(widths, RLGPU_FUSED_INFER = 0 or fp32 inference)");
        hipStream_t s = rlgpu::as_stream(stream);
        // the fused kernel keeps no per-row buffers: one launch per pass over all n rows (no max_rows chunks)
        const int64_t r0 = row0 + h->cfg.sample_row_offset;
        if (!d_old_rows) {
            infer_fused(h, 0, false, d_obs, n, 1, nullptr, d_masks, deterministic, rng_step, d_actions, d_logp, nullptr, 0, s,
                        r0);
            return;
        }
        for (int old = 0; old < 2; old++)  // current policy rows, then the old version's rows
            infer_fused(h, 0, old != 0, d_obs, n, 1, nullptr, d_masks, deterministic, rng_step, d_actions,
                        (d_logp && !old) ? d_logp : nullptr, d_old_rows, old, s, r0);
    });
}

extern "C" int rlgpu_ppo_fused_infer(rlgpu_ppo* h, int32_t model) { return h && fused_ok(h, model) ? 1 : 0; }

extern "C" int rlgpu_ppo_infer_critic(rlgpu_ppo* h, const float* d_obs, int64_t n, float* d_values, void* stream) {
    return rlgpu::guarded([&] {
        RLGPU_REQUIRE(h && d_obs && d_values, "null argument");
        hipStream_t s = rlgpu::as_stream(stream);
        // the fused kernel keeps no per-row buffers: one launch over up to 2^30 rows (no max_rows chunks)
        const int64_t R = fused_ok(h, 1) ? (int64_t)1 << 30 : h->cfg.max_rows;
        for (int64_t b = 0; b < n; b += R) {
            int m = (int)std::min<int64_t>(R, n - b);
            if (infer_f32(h)) {  // useHalfPrecision = false
                forward_f32(h, 1, d_obs + b * h->cfg.obs_size, m, d_values + b, s);
                continue;
            }
            if (fused_ok(h, 1)) {
                infer_fused(h, 1, false, d_obs + b * h->cfg.obs_size, m, 0, d_values + b, nullptr, 0, 0, nullptr, nullptr,
                            nullptr, 0, s);
                continue;
            }
            forward_half(h, 1, d_obs + b * h->cfg.obs_size, m, s);
            RLGPU_H16_LAUNCH(f16(h), ppo::bf16_to_f32, dim3(ceil_div(m, 256)), dim3(256), 0, s, h->logits_h, d_values + b,
                               (int64_t)m);
            RLGPU_CHECK_HIP(hipGetLastError());
        }
    });
}

extern "C" int rlgpu_mean_std(const float* d_x, int64_t n, float* d_out, void* stream) {
    return rlgpu::guarded([&] {
        RLGPU_REQUIRE(d_x && d_out && n > 0, "rlgpu_mean_std: bad argument");
        hipStream_t s = rlgpu::as_stream(stream);
        const int nb = 256;
        double* part = nullptr;
        RLGPU_CHECK_HIP(hipMallocAsync((void**)&part, nb * 2 * sizeof(double), s));
        hipLaunchKernelGGL(ppo::moments_partial, dim3(nb), dim3(256), 0, s, d_x, n, part);
        hipLaunchKernelGGL(ppo::moments_final, dim3(1), dim3(64), 0, s, part, nb, n, d_out);
        RLGPU_CHECK_HIP(hipGetLastError());
        RLGPU_CHECK_HIP(hipFreeAsync(part, s));
    });
}

extern "C" int rlgpu_ppo_minibatch(rlgpu_ppo* h, const float* d_obs, const uint8_t* d_masks, const int32_t* d_actions,
                                   const float* d_old_logp, const float* d_adv, const float* d_target, const int32_t* d_index,
                                   int64_t start, int32_t n, int64_t batch_size, const float* d_adv_stats, float* d_metrics,
                                   void* stream) {
    return rlgpu::guarded([&] {
        RLGPU_REQUIRE(h && d_obs && d_masks && d_actions && d_old_logp && d_adv && d_target && d_adv_stats,
                      "rlgpu_ppo_minibatch: null argument");
        RLGPU_REQUIRE(n > 0 && n <= h->cfg.max_rows, "minibatch rows must be in [1, max_rows]");
        RLGPU_REQUIRE(batch_size > 0, "batch_size must be > 0");
        hipStream_t s = rlgpu::as_stream(stream);
        float bsr = (float)n / (float)batch_size;  // PPOLearner.cpp:374
        int A = h->cfg.num_actions;
        gather_obs(h, d_obs, d_index, start, n, s);  // one gathered, padded copy serves both models
        // the shared head's forward once per minibatch (PPOLearner.cpp:395-398); policy and critic read it
        const Input obs_in = obs_input(h), xin = model_input(h, 0);
        if (h->shared()) forward_train(h, 2, obs_in, n, nullptr, s);
        // the critic's pass runs on the auxiliary stream (disjoint parameters, gradients, workspace
        // and metric slots), overlapping the policy's; the caller's stream waits for both
        hipStream_t cs = h->aux;
        RLGPU_CHECK_HIP(hipEventRecord(h->ev_fork, s));
        RLGPU_CHECK_HIP(hipStreamWaitEvent(h->aux, h->ev_fork, 0));
        Model& pm = h->M[0];
        Model& cm = h->M[1];
        forward_train(h, 1, xin, n, cm.y, cs);
        hipLaunchKernelGGL(ppo::critic_loss, dim3(ceil_div(n, 256)), dim3(256), 0, cs, cm.y, d_target, d_index, start, n,
                           bsr, cm.dy, d_metrics);
        RLGPU_CHECK_HIP(hipGetLastError());
        backward(h, 1, xin, n, cm.dy, cs);
        RLGPU_CHECK_HIP(hipEventRecord(h->ev_join, h->aux));
        // policy on the caller's stream
        forward_train(h, 0, xin, n, pm.y, s);
        const int pl_blocks = (int)ceil_div(n, ppo::PL_ROWS);
        hipLaunchKernelGGL(ppo::policy_loss_any(A), dim3(pl_blocks), dim3(256), 0, s, pm.y, d_masks, d_actions, d_old_logp, d_adv,
                           d_index, start, n, A, d_adv_stats, bsr, h->cfg.clip_range, h->cfg.entropy_scale,
                           1.f / std::log((float)A), pm.dy, dout_ld(A), d_metrics, pm.lpart, amax_slot(pm, kAmaxOut));
        RLGPU_CHECK_HIP(hipGetLastError());
        backward(h, 0, xin, n, pm.dy, s, pm.lpart, pl_blocks);
        RLGPU_CHECK_HIP(hipStreamWaitEvent(s, h->ev_join, 0));
        if (h->shared()) {  // (ppoLoss + criticLoss).backward() through the shared features (:498)
            const int64_t e = (int64_t)n * h->M[2].out;
            hipLaunchKernelGGL(ppo::add2, dim3(ceil_div(ceil_div(e, 4), 256)), dim3(256), 0, s, pm.dX, cm.dX, h->dshared, e);
            RLGPU_CHECK_HIP(hipGetLastError());
            backward(h, 2, obs_in, n, h->dshared, s);
        }
    });
}

extern "C" int rlgpu_ppo_optimizer_step(rlgpu_ppo* h, float* d_metrics, void* stream) {
    return rlgpu::guarded([&] {
        RLGPU_REQUIRE(h, "null handle");
        hipStream_t s = rlgpu::as_stream(stream);
        h->step++;
        const auto& c = h->cfg;
        double bc1 = 1.0 - std::pow((double)c.beta1, (double)h->step);
        double bc2 = 1.0 - std::pow((double)c.beta2, (double)h->step);
        const int slot[3] = {RLGPU_M_GRAD_NORM_POLICY, RLGPU_M_GRAD_NORM_CRITIC, RLGPU_M_GRAD_NORM_SHARED};
        for (int mi = 0; mi < h->nm; mi++) {
            Model& m = h->M[mi];
            float* coef = h->scratch + 600 + mi;
            float* norm_out = d_metrics ? d_metrics + slot[mi] : nullptr;
            sumsq_coef(h, h->grads + m.off, m.count, c.max_grad_norm, coef, norm_out, s);
            double lr = m.lr;
            float decay_mul = (float)(1.0 - lr * (double)c.weight_decay);
            float step_size = (float)(lr / bc1);
            float bc2_sqrt = (float)std::sqrt(bc2);
            hipLaunchKernelGGL(ppo::adamw, dim3(ceil_div(m.count, 256)), dim3(256), 0, s, h->params + m.off, h->grads + m.off,
                               h->exp_avg + m.off, h->exp_avg_sq + m.off, m.count, coef, decay_mul, c.beta1,
                               c.beta2, 1.f - c.beta1, 1.f - c.beta2, step_size, bc2_sqrt, c.eps);
            RLGPU_CHECK_HIP(hipGetLastError());
        }
        refresh_half(h, s);  // Model::Forward's lazily refreshed seqHalf (Models.cpp:46-66)
    });
}

extern "C" int rlgpu_ppo_zero_grad(rlgpu_ppo* h, void* stream) {
    return rlgpu::guarded([&] {
        RLGPU_REQUIRE(h, "null handle");
        RLGPU_CHECK_HIP(hipMemsetAsync(h->grads, 0, h->nparams * sizeof(float), rlgpu::as_stream(stream)));
    });
}

extern "C" int rlgpu_ppo_optimizer_state(rlgpu_ppo* h, int64_t* step, float** d_exp_avg, float** d_exp_avg_sq) {
    return rlgpu::guarded([&] {
        RLGPU_REQUIRE(h, "null handle");
        if (step) *step = h->step;
        if (d_exp_avg) *d_exp_avg = h->exp_avg;
        if (d_exp_avg_sq) *d_exp_avg_sq = h->exp_avg_sq;
    });
}

extern "C" int rlgpu_ppo_set_optimizer_step(rlgpu_ppo* h, int64_t step) {
    return rlgpu::guarded([&] {
        RLGPU_REQUIRE(h && step >= 0, "rlgpu_ppo_set_optimizer_step: bad argument");
        h->step = step;
    });
}

extern "C" int rlgpu_permutation(int64_t n, uint64_t seed, uint64_t counter, int32_t* d_out, void* stream) {
    return rlgpu::guarded([&] {
        RLGPU_REQUIRE(d_out && n >= 0 && n < (1ll << 31), "rlgpu_permutation: bad argument");
        if (n == 0) return;
        hipStream_t s = rlgpu::as_stream(stream);
        uint32_t *k0 = nullptr, *k1 = nullptr;
        int32_t* v0 = nullptr;
        RLGPU_CHECK_HIP(hipMallocAsync((void**)&k0, n * 4, s));
        RLGPU_CHECK_HIP(hipMallocAsync((void**)&k1, n * 4, s));
        RLGPU_CHECK_HIP(hipMallocAsync((void**)&v0, n * 4, s));
        hipLaunchKernelGGL(ppo::perm_keys, dim3(ceil_div(n, 256)), dim3(256), 0, s, k0, v0, n, seed, (uint32_t)counter);
        RLGPU_CHECK_HIP(hipGetLastError());
        size_t tmp_bytes = 0;
        RLGPU_CHECK_HIP(hipcub::DeviceRadixSort::SortPairs(nullptr, tmp_bytes, k0, k1, v0, d_out, (int)n, 0, 32, s));
        void* tmp = nullptr;
        RLGPU_CHECK_HIP(hipMallocAsync(&tmp, tmp_bytes + 16, s));
        RLGPU_CHECK_HIP(hipcub::DeviceRadixSort::SortPairs(tmp, tmp_bytes, k0, k1, v0, d_out, (int)n, 0, 32, s));
        RLGPU_CHECK_HIP(hipFreeAsync(tmp, s));
        RLGPU_CHECK_HIP(hipFreeAsync(k0, s));
        RLGPU_CHECK_HIP(hipFreeAsync(k1, s));
        RLGPU_CHECK_HIP(hipFreeAsync(v0, s));
    });
}

extern "C" int rlgpu_gemm(int32_t mode, int32_t a_layout, int32_t b_layout, const float* d_A, int64_t lda, const float* d_B,
                          int64_t ldb, float* d_C, int64_t ldc, const float* d_bias, int32_t I, int32_t J, int32_t K,
                          int32_t splits, void* stream) {
    return rlgpu::guarded([&] {
        RLGPU_REQUIRE(d_A && d_B && d_C, "rlgpu_gemm: null argument");
        RLGPU_REQUIRE(mode == RLGPU_GEMM_F32X6 || mode == RLGPU_GEMM_F32 || mode == RLGPU_GEMM_F16X3,
                      "rlgpu_gemm: unknown mode");
        RLGPU_REQUIRE(I > 0 && J > 0 && K > 0 && splits >= 1, "rlgpu_gemm: bad sizes");
        RLGPU_REQUIRE((a_layout == 0 && (b_layout == 0 || b_layout == 1)) || (a_layout == 1 && b_layout == 1),
                      "rlgpu_gemm: unsupported layout pair");
        hipStream_t s = rlgpu::as_stream(stream);
        if (mode == RLGPU_GEMM_F16X3) {
            // operand scales from stand-alone max |x| passes (the training path gets them from the
            // producer kernels); B pre-split into scaled planes when the training path would be
            float* sh = nullptr;
            RLGPU_CHECK_HIP(hipMallocAsync((void**)&sh, 128 * sizeof(float), s));
            RLGPU_CHECK_HIP(hipMemsetAsync(sh, 0, 128 * sizeof(float), s));
            const int64_t ar = a_layout == 0 ? I : K, ac = a_layout == 0 ? K : I;
            hipLaunchKernelGGL(mlp::amax_rows, dim3(256), dim3(256), 0, s, d_A, ar, (int)ac, lda, sh);
            if (a_layout == 0 && splits == 1) {
                const int rows = (int)ceil_div(J, mlp::BNW) * mlp::BNW, ld = (int)ceil_div(K, mlp::XKMAX) * mlp::XKMAX;
                const int64_t plane = (int64_t)rows * ld;
                uint16_t* planes = nullptr;
                float* inv = nullptr;
                RLGPU_CHECK_HIP(hipMallocAsync((void**)&planes, 2 * plane * sizeof(uint16_t), s));
                RLGPU_CHECK_HIP(hipMallocAsync((void**)&inv, rows * sizeof(float), s));
                if (b_layout == 0)  // B [J][ldb]: W = B (out = J, in = K)
                    hipLaunchKernelGGL(mlp::split_weight_h3, dim3(rows), dim3(256), 0, s, d_B, J, K, ldb, 0, ld, planes, plane, inv);
                else  // B [K][ldb]: W^T (out = K, in = J)
                    hipLaunchKernelGGL(mlp::split_weight_h3, dim3(rows), dim3(256), 0, s, d_B, K, J, ldb, 1, ld, planes, plane, inv);
                RLGPU_CHECK_HIP(hipGetLastError());
                gemm_x6_pre(d_A, lda, planes, ld, plane, d_C, ldc, d_bias, I, J, K, s, false, sh, inv);
                RLGPU_CHECK_HIP(hipFreeAsync(planes, s));
                RLGPU_CHECK_HIP(hipFreeAsync(inv, s));
            } else {
                const int64_t br = b_layout == 0 ? J : K, bc = b_layout == 0 ? K : J;
                hipLaunchKernelGGL(mlp::amax_rows, dim3(256), dim3(256), 0, s, d_B, br, (int)bc, ldb, sh + 64);
                gemm_f32(mode, a_layout, b_layout, d_A, lda, d_B, ldb, d_C, ldc, d_bias, I, J, K, splits, s, false, false, sh,
                         sh + 64);
            }
            RLGPU_CHECK_HIP(hipGetLastError());
            RLGPU_CHECK_HIP(hipFreeAsync(sh, s));
            return;
        }
        if (mode == RLGPU_GEMM_F32X6 && a_layout == 0 && splits == 1) {
            // the training path's form: B split once into padded planes, then the pre-split kernel
            const int rows = (int)ceil_div(J, mlp::BN) * mlp::BN, ld = (int)ceil_div(K, mlp::XKMAX) * mlp::XKMAX;
            const int64_t plane = (int64_t)rows * ld;
            uint16_t* planes = nullptr;
            RLGPU_CHECK_HIP(hipMallocAsync((void**)&planes, 3 * plane * sizeof(uint16_t), s));
            if (b_layout == 0)
                hipLaunchKernelGGL(mlp::split_weight, dim3(ceil_div(plane, 256)), dim3(256), 0, s, d_B, J, (int)ldb, 0, rows, ld,
                                   planes);
            else
                hipLaunchKernelGGL(mlp::split_weight, dim3(ceil_div(plane, 256)), dim3(256), 0, s, d_B, K, (int)ldb, 1, rows, ld,
                                   planes);
            RLGPU_CHECK_HIP(hipGetLastError());
            gemm_x6_pre(d_A, lda, planes, ld, plane, d_C, ldc, d_bias, I, J, K, s);
            RLGPU_CHECK_HIP(hipFreeAsync(planes, s));
            return;
        }
        gemm_f32(mode, a_layout, b_layout, d_A, lda, d_B, ldb, d_C, ldc, d_bias, I, J, K, splits, s);
    });
}

extern "C" int rlgpu_gemm_f32(int32_t a_layout, int32_t b_layout, const float* d_A, int64_t lda, const float* d_B, int64_t ldb,
                              float* d_C, int64_t ldc, const float* d_bias, int32_t I, int32_t J, int32_t K, int32_t splits,
                              void* stream) {
    return rlgpu::guarded([&] {
        RLGPU_REQUIRE(d_A && d_B && d_C, "rlgpu_gemm_f32: null argument");
        RLGPU_REQUIRE(I > 0 && J > 0 && K > 0 && splits >= 1, "rlgpu_gemm_f32: bad sizes");
        RLGPU_REQUIRE((a_layout == 0 && (b_layout == 0 || b_layout == 1)) || (a_layout == 1 && b_layout == 1),
                      "rlgpu_gemm_f32: unsupported layout pair");
        gemm_f32(RLGPU_GEMM_F32, a_layout, b_layout, d_A, lda, d_B, ldb, d_C, ldc, d_bias, I, J, K, splits, rlgpu::as_stream(stream));
    });
}

extern "C" int rlgpu_kernel_timing(int32_t enable) {
    return rlgpu::guarded([&] {
        ktime::clear();
        ktime::g.on = enable != 0;
    });
}

extern "C" int rlgpu_kernel_timing_read(double* ms, double* work, int64_t* count, int32_t nslots) {
    return rlgpu::guarded([&] {
        RLGPU_REQUIRE(ms && work && count && nslots >= 0, "rlgpu_kernel_timing_read: null argument");
        for (int i = 0; i < nslots; i++) {
            ms[i] = work[i] = 0.0;
            count[i] = 0;
        }
        for (auto& r : ktime::g.recs) {
            if (r.slot >= nslots) continue;
            RLGPU_CHECK_HIP(hipEventSynchronize(r.b));
            float t = 0.f;
            RLGPU_CHECK_HIP(hipEventElapsedTime(&t, r.a, r.b));
            ms[r.slot] += t;
            work[r.slot] += r.work;
            count[r.slot]++;
        }
    });
}

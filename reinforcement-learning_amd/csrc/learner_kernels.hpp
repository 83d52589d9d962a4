// learner_kernels.hpp -- launchers of the host Learner's device helpers (csrc/learner_kernels.hip).
#pragma once
#include <hip/hip_runtime.h>
#include <stddef.h>
#include <stdint.h>

namespace lk {
// dst[i] = src[idx[i]]
void gather_f32(const float* src, const int32_t* idx, int64_t n, float* dst, hipStream_t s);
// dst[idx[i]] = src[i]  (index_copy)
void scatter_f32(const float* src, const int32_t* idx, int64_t n, float* dst, hipStream_t s);
// dst[r, :] = src[idx[r], :] for rows of C floats
void gather_rows(const float* src, int C, const int32_t* idx, int64_t n, float* dst, hipStream_t s);
// out[i] = rows[perm[i]]
void compose(const int32_t* rows, const int32_t* perm, int64_t n, int32_t* out, hipStream_t s);
// sample indices t * P + p of the players of `team` (p % 2 == team), [T][P / 2]
void train_rows(int T, int P, int team, int32_t* out, hipStream_t s);
// out[p] = the last t with terms[t * P + p] != 0 (the column's last trajectory end), -1 if none
void last_ends(const int8_t* terms, int T, int P, int32_t* out, hipStream_t s);
void gather_samples(const float* src, const int64_t* idx, int n, float* dst, hipStream_t s);
// (sum, sum of squares, n) in fp64 of x[idx[i]] (idx may be null), deterministic
size_t moments_scratch_bytes();
void moments_f64(const float* x, const int32_t* idx, int64_t n, double* scratch, double* out3, hipStream_t s);
// rows i (ascending) with terms[i] == 2, and their count (device)
size_t select_trunc_scratch_bytes(int64_t n);
void select_trunc(const int8_t* terms, int64_t n, void* scratch, size_t scratch_bytes, int32_t* rows, int32_t* count,
                  hipStream_t s);
// Frame stacking (BASELINE config C4): out[p] = [cur, h0, .., h(K-2)] (OBS floats each), then the
// history shifts (h0 <- cur); a trajectory that ended this step (codes[p] != 0) restarts its stack
// with the current frame repeated, and its pre-reset row out_trunc[p] = [trunc, h0, .., h(K-2)].
// hist [K-1][P][OBS].  codes == null: initialise (every stack = the current frame repeated).
void stack_frames(const float* cur, const float* trunc, const int8_t* codes, float* hist, int K, int P, int obs,
                  float* out, float* out_trunc, hipStream_t s);
}  // namespace lk

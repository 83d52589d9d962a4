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

// After a step hook (host plugins / StepCallbackFn): codes[p] = arena_terms[p / 4] (the merged terminal) or,
// where 0, the device's code; rew_out[p] = rewards[p] (rew_out may be null); the pre-reset obs rows of code-2
// players (obs [P][obs_w]) to trunc_env and trunc_out (may be null)
void host_step_finish(const uint8_t* arena_terms, int8_t* codes, const float* rewards, float* rew_out, const float* obs,
                      float* trunc_env, float* trunc_out, int P, int obs_w, hipStream_t s);

// ---- reference experience mode (complete trajectories with carry-over, Learner.cpp:504-547,823-861)
// Trajectory records, structure of arrays (capacity rows each), appended in the reference's order:
// by the step a trajectory ends, then by player index (combinedTraj.Append in the newPlayerIndices loop).
struct TrajRecs {
    int32_t* p;      // player
    int32_t* start;  // circular store row of its first step
    int32_t* len;    // steps
    int32_t* code;   // its last step's code: 1 NORMAL / 2 TRUNCATED
    int32_t* tidx;   // index into the truncation list (code 2), else -1
    int64_t* off;    // first row in the combined (flat) batch
};
// counters (device int64 [8]): [0] records, [1] truncations, [2] combined steps (finished), [3] this
// step's truncations (players in trnew)
enum { kTcRecs = 0, kTcTruncs = 1, kTcSteps = 2, kTcNewTruncs = 3, kTcCount = 8 };
// One env step's bookkeeping: for every tracked player (track[p] != 0; null = all) the step at store
// row `row` (codes[p]) extends its trajectory; a nonzero code ends it -- a record is appended and the
// next trajectory starts at row + 1 (mod Tmax).  trnew[j] = the j-th truncating player of this step.
void traj_step(const int8_t* codes, int row, int Tmax, const uint8_t* track, int P, int32_t* start, int32_t* len,
               TrajRecs recs, int64_t* counters, int32_t* trnew, hipStream_t s);
// the pre-reset obs rows of this step's truncations (src [P][W]) to dst rows counters[1] - counters[3] + j
void traj_trunc_copy(const float* src, int W, const int64_t* counters, const int32_t* trnew, float* dst, hipStream_t s);
// restart the trajectories of players with mask[p] != 0 at store row `row` (self-play: a team that acted
// with an old version)
void traj_restart(const uint8_t* mask, int P, int row, int32_t* start, int32_t* len, hipStream_t s);
// the combined batch: record k's len steps (store rows start .. start + len - 1 mod Tmax, column p) to
// combined rows off .. off + len - 1 (obs W floats, masks A bytes, action, log prob, reward, code)
void traj_gather(TrajRecs recs, int64_t K, int Tmax, int P, int W, int A, const float* obs, const uint8_t* masks,
                 const int32_t* acts, const float* logp, const float* rews, const int8_t* terms, float* c_obs,
                 uint8_t* c_masks, int32_t* c_acts, float* c_logp, float* c_rews, int8_t* c_terms, hipStream_t s);
}  // namespace lk

// hsim device buffers and launch interface (product).
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>

#include "hs_model.h"

namespace hs {

constexpr int AUXDIM = MAXDOF + 8;   // per env: qacc[nv], com[3], ncon, nefc, newton iters, solver flag
constexpr int DBGDIM = 32768;        // stage dump (env 0 only) for parity debugging
// hand-off row of a queued env step (qpos, qvel, qacc_warmstart, time, warning counters, and the
// env bookkeeping a tape launch carries from one env step to the next: step count, episode, return)
constexpr int MID_NWARN = 5;   // == NWARN (static_assert below)
constexpr int MID_Q = 0, MID_V = MAXQ, MID_WS = MAXQ + MAXDOF, MID_TIME = MAXQ + 2 * MAXDOF, MID_W = MID_TIME + 1;
constexpr int MID_SC = MID_W + MID_NWARN, MID_EP = MID_SC + 1, MID_TOT = MID_SC + 2;
// a fused rollout (hs_rollout) also hands over the next step's clipped action and the episode return
constexpr int MID_ACT = MID_TOT + 1, MID_EPACC = MID_ACT + 32;
constexpr int MIDDIM = MID_EPACC + 1;
// chunk-queue sync words (uncached device memory): claim counter, exit counter, launch epoch,
// per-pair flags.  A pair's flag holds the tag of the launch whose first chunk last handed its state
// over (tag = epoch + 1, the epoch advanced by the last wave out of every queued launch), so a flag
// left over from an earlier launch -- e.g. by a producer that arrived after its consumer timed out
// -- never matches: no reset store, no returning atomic.  QS_ABORT: a tape launch (p.nsteps > 1)
// stops when an env overflows the resident tier (the host replays the tape step by step).
constexpr int QS_HEAD = 0, QS_EXIT = 1, QS_EPOCH = 2, QS_ABORT = 3, QS_FLAG = 4;
// flag value of a queued hand-off: the launch tag (epoch + 1, 20 bits) and the hand-off's position
// in the launch (the env step of a tape launch and its stage), so a consumer waits for exactly its
// predecessor: stage 0 = first chunk of step t handed over, 1 = step t committed
constexpr int QTAG_STEPS = 511;   // most env steps per tape launch
__host__ __device__ constexpr int qtag(uint32_t epoch, int t, int stage) {
  return (int)((((epoch & 0xFFFFFu) + 1u) << 10) | (uint32_t)(2 * t + stage + 1));
}
// Cost-ordered claims: every queued launch measures each pair's duration (first chunk + last
// substep, 100 MHz realtime clock) and counts the pair into one of QNB buckets of QBIN ticks,
// heaviest first; the next queued launch claims the pairs bucket by bucket (a counting sort done
// by the previous launch), so the launch ends on the cheapest last substeps.  After the flags:
// qcost[npairs] (first-chunk durations), cnt[2][QNB] (bucket counts, by epoch parity: the launch
// reads cnt[e & 1], counts into cnt[(e + 1) & 1], and its last wave out zeroes cnt[e & 1]),
// ord[2][QNB][npairs] (the pairs of each bucket).  A launch whose read counts do not sum to npairs
// (the batch's first queued launch) claims in the fixed multiplicative permutation (p.qmul).
constexpr int QNB = 32, QBIN = 2500;   // 32 buckets of 25 us
constexpr size_t qs_cost(int npairs) { return QS_FLAG + (size_t)npairs; }
constexpr size_t qs_cnt(int npairs, int par) { return QS_FLAG + 2 * (size_t)npairs + (size_t)par * QNB; }
constexpr size_t qs_ord(int npairs, int par) {
  return QS_FLAG + 2 * (size_t)npairs + 2 * QNB + (size_t)par * QNB * npairs;
}
// sized for n_envs units: the queue's unit is an env pair, or one env in the single-env mode of
// small-batch tape launches (launch_step)
constexpr size_t qsync_words(int n_envs) { return qs_ord(n_envs, 2); }

enum StepMode { MODE_ENV_STEP = 0, MODE_RESET = 1, MODE_PHYSICS = 2 };
enum RewardId { REWARD_NONE = -1, REWARD_STAND = 0, REWARD_KNEELING = 1, REWARD_WALK = 2 };
// per-env warning counters: MuJoCo's mj_checkPos / mj_checkVel / mj_checkAcc resets, contacts past the
// wide tier, and a lost chunk-queue hand-off (a scheduling failure, not physics: the env is reset the
// same way and the trainer raises on it)
enum Warn { WARN_BADQPOS = 0, WARN_BADQVEL = 1, WARN_BADQACC = 2, WARN_OVERFLOW = 3, WARN_HANDOFF = 4, NWARN = 5 };
static_assert(NWARN == MID_NWARN, "hand-off row warning slots");

template <typename T>
struct EnvBuffers {
  T* qpos;               // [N][nq]
  T* qvel;               // [N][nv]
  T* qacc_ws;            // [N][nv]  (mjData.qacc_warmstart)
  T* ctrl;               // [N][nu]
  T* time;               // [N]
  int* step_count;       // [N]
  uint32_t* episode;     // [N]      reset counter (device RNG stream)
  T* total_reward;       // [N]
  int* warning;          // [N][NWARN]
  T* obs;                // [N][obs_dim]
  T* terminal_obs;       // [N][obs_dim]  written for envs that auto-reset this step
  T* reward;             // [N]
  uint8_t* terminated;   // [N]
  uint8_t* truncated;    // [N]
  T* aux;                // [N][AUXDIM]
  T* cfrc_ext;           // [N][nbody][6]  (full_state)
  T* subtree_linvel;     // [N][nbody][3]  (full_state)
  int* term_step_count;  // [N] or null: step_count of envs that auto-reset this step (SB3 final info)
  T* term_total_reward;  // [N] or null: their episode return
  int* redo;             // [2 + N] wide-tier work list: count, done counter, env ids (hs_batch owned)
  T* mid;                // [N][MIDDIM] state between the chunks of a queued env step (hs_batch owned)
  int* qsync;            // [qsync_words(N)] chunk queue: claim / exit counters, pair flags (hs_batch owned)
  unsigned long long* redo_total;   // cumulative number of wide-tier re-runs (diagnostics)
  T* dbg;                // [DBGDIM] or nullptr
};

struct StepParams {
  int mode;              // StepMode
  int nsub;              // substeps per call (frame_skip for env steps, n for physics)
  int max_steps;         // custom_env.py:201 truncation (750)
  int reward_id;         // RewardId
  int autoreset;         // SB3 VecEnv auto-reset semantics
  int obs_dim;
  int max_newton;        // Newton iteration cap
  int full_state;        // compute cfrc_ext / subtree_linvel; obs gains cfrc_ext[1:]
  double duration;       // custom_env.py:213 (10.0 in training)
  double init_height;    // custom_env.py:59 (1.282)
  double noise_scale;    // custom_env.py:109-110 (0.01)
  uint64_t seed;
  double kneel[9];       // target_height, min_height, max_roll_pitch, com_radius, energy_w, posture_w,
                         // com_w, foot_w, alive_w (reward_functions.py:71-81)
  int solver;            // SOLVER_NEWTON (MuJoCo default) or SOLVER_PGS: selects the kernel instance
  int outputs;           // OUT_* bits: optional per-env outputs written at commit
  int schedule;          // HS_SCHED_AUTO (0) / HS_SCHED_DIRECT (1) (hs_env_config.schedule)
  int queue;             // set by launch_step: 1 = chunk-queue schedule (persistent grid), 0 = one wave per pair
  int qmul;              // chunk-queue fallback claim order: item i -> pair (i * qmul) mod npairs (coprime)
  int qorder;            // chunk queue: 1 = cost-ordered claims (QNB buckets), 0 = the qmul permutation only
  int dbg_lose_pair1;    // test hook (hs_debug_lose_handoff): env + 1 from the host; launch_step turns it into the
                         // queue unit (pair or env) + 1 whose hand-off is treated as lost; 0 = off
  int single;            // set by launch_step: 1 = one env per wave (upper half-wave a ghost), 0 = env pairs
                         // (also the chunk queue's unit for small-batch tape launches)
  int nsteps;            // env steps per launch: 1, or a tape launch of nsteps (MODE_ENV_STEP, chunk queue)
};
// per-step outputs of a tape launch ([nsteps][N][...] each; null: the batch's own buffers, last step wins)
template <typename T>
struct TapeOut {
  T* obs;
  T* reward;
  uint8_t* terminated;
  uint8_t* truncated;
};
// hs_env_config.schedule (SCHED_FIXED_ORDER: AUTO with the chunk queue's claims in the fixed
// permutation instead of cost order -- A/B runs and tests)
enum Schedule { SCHED_AUTO = 0, SCHED_DIRECT = 1, SCHED_SINGLE = 2, SCHED_FIXED_ORDER = 3 };
// optional outputs (hs_env_config.outputs): the aux row (qacc, subtree com, ncon, nefc, solver
// iterations -- data views and stats) and the data.ctrl copy (data views / host rewards)
enum Outputs { OUT_AUX = 1, OUT_CTRL = 2 };
enum Solver { SOLVER_NEWTON = 0, SOLVER_PGS = 1 };

// actions: [N][nu] float32 (may be null in MODE_RESET); reset_mask: [N] (null = all);
// noise_qpos/noise_qvel: [N][nq]/[N][nv] host-supplied reset noise (null = device RNG).
// Fused PPO rollout (hs_rollout, fp64 engine): a tape launch whose actions come from the policy.
// After each env step the env's wave runs the SB3 MlpPolicy's pi net (2 hidden layers of 256, ReLU)
// on the new obs, draws the action (the Philox stream of ppo_act_kernel) and does the rollout
// buffer bookkeeping of ppo_post_kernel, so a K-step rollout is one launch.  Rollout buffers are
// indexed by the global step g = t_begin + t.
struct RolloutArgs {
  const float* w1;      // [D][ld1] pi layer 1 ([in][out], columns 0..255), ld1 >= 256
  const float* b1;      // [256]
  const float* w2;      // [256][256]
  const float* b2;      // [256]
  const float* w3;      // [256][A]
  const float* b3;      // [A]
  const float* log_std; // [A]
  int ld1, D, A;
  int t_begin, t_total; // global step of this launch's first step; rollout length (n_steps)
  float* obs;           // [t_total][N][D]: rows g + 1 written (row 0 is the caller's)
  float* obs_last;      // [N][D]: the obs after step t_total - 1 (the next rollout's first obs)
  float* act;           // [t_total][N][A] unclipped samples (row t_begin is the caller's)
  float* logp;          // [t_total][N]
  float* start;         // [t_total][N] episode_start before step g
  float* rew;           // [t_total][N]
  uint8_t* done;        // [t_total][N]
  double* epret;        // [t_total][N] episode return so far (ppo_post's ep_return_out)
  uint8_t* boot;        // [t_total][N] TimeLimit.truncated and not terminated
  float* tobs;          // [t_total][N][D] terminal obs of the boot envs
  double* ep_acc;       // [N] running episode return, in / out
  float* episode_start; // [N] out: done of the launch's last step
  float* act_clip;      // [N][A] in: step t_begin's clipped action; out: the next launch's
  const uint64_t* ctr_base;   // noise counter base (device); step g draws counter g + *ctr_base
  uint32_t k0, k1;            // Philox key (the 64-bit seed)
  int deterministic;
};

// p.nsteps > 1: a tape launch -- actions [nsteps][N][nu], outputs per step in `tape` (may be null), env
// steps of one env pair run back to back on the chunk queue with the state handed over through
// b.mid; no wide-tier launch follows (an overflow sets qsync[QS_ABORT], the host replays the tape).
template <typename T>
hipError_t launch_step(const DevModel<T>* dmodel, int nv, const EnvBuffers<T>& b, const float* actions,
                       const uint8_t* reset_mask, const T* noise_qpos, const T* noise_qvel,
                       const StepParams& p, int nenv, hipStream_t stream, const TapeOut<T>* tape = nullptr,
                       const RolloutArgs* ro = nullptr);

// waves of the resident step-kernel instance the current device holds at once (0 if unknown)
template <typename T>
int resident_waves(bool pgs);

// mj_kinematics/mj_comPos of one state (device qpos[nq]) -> out[KINDIM] (see kin_kernel)
constexpr int KINDIM = MAXBODY * 12 + MAXGEOM * 6 + 3;
template <typename T>
hipError_t launch_kinematics(const DevModel<T>* dmodel, int nv, const T* qpos, T* out, hipStream_t stream);

// the step kernel's reward code (reward_formula) on caller-supplied per-env fields (hs_reward_eval)
template <typename T>
struct RewardEvalArgs {
  int reward_id, n, nq, nv, nu, nbody;
  double kneel[9];            // StepParams::kneel
  const T* qpos;              // [n][nq]
  const T* qvel;              // [n][nv]
  const T* ctrl;              // [n][nu]
  const T* time;              // [n]
  const T* subtree_com0;      // [n][3]
  const T* subtree_linvel0;   // [n][3]
  const T* cfrc_ext;          // [n][nbody][6]
  const T* qfrc_actuator;     // [n][nv]
  T* out;                     // [n]
  // row strides (elements) of subtree_com0 / subtree_linvel0 / qfrc_actuator; 0 = packed (3, 3, nv) --
  // hs_reward reads the batch's own buffers in place (aux row, subtree_linvel rows, obs rows)
  int ld_com, ld_linv, ld_qfrc;
};
template <typename T>
hipError_t launch_reward_eval(const RewardEvalArgs<T>& a, hipStream_t stream);

// one step's host-bound outputs packed into one float64 buffer (hs_pack_outputs)
template <typename T>
struct PackArgs {
  int n, obs_dim, ncols, nwarn, nwarn_stride;
  const T* obs;
  const T* reward;
  const uint8_t* terminated;
  const uint8_t* truncated;
  const T* total_reward;
  const int* step_count;
  const int* term_step_count;
  const T* term_total_reward;
  const int* warning;
  double* out;
};
template <typename T>
hipError_t launch_pack(const PackArgs<T>& a, hipStream_t stream);

// PPO rollout bookkeeping around the policy GEMMs and the env step (ppo.hip)
hipError_t launch_ppo_act(const float* mean, int mean_ld, const float* value, int value_ld, const float* log_std,
                          const float* episode_start, uint64_t seed, uint64_t counter, const uint64_t* counter_base,
                          int deterministic, float* act,
                          float* act_clip, float* logp, float* val, float* start_out, int N, int A,
                          hipStream_t stream);
hipError_t launch_ppo_post(const float* reward, const uint8_t* terminated, const uint8_t* truncated,
                           const float* terminal_value, const float* terminal_obs, float* boot_obs_out,
                           uint8_t* boot_out, int obs_dim, float gamma, const float* obs, float* obs_out,
                           size_t obs_floats, float* reward_out, uint8_t* done_out, double* ep_acc,
                           double* ep_return_out, float* episode_start, int N, hipStream_t stream);
// fused 2-hidden-layer (H = 256) ReLU MLP forward of one packed policy net (ppo.hip mlp2_fwd_kernel)
hipError_t launch_mlp2_fwd(const float* X, int ldx, int D, int N, const float* W1, int ld1, const float* b1,
                           const float* W2, int ld2, const float* b2, const float* W3, int ld3, const float* b3, int A,
                           float* out, int ldo, hipStream_t stream);
// column sums of a row-major [rows][cols] float32 matrix (ppo.hip); workspace of
// colsum_workspace(rows, cols) floats (0: none needed)
size_t colsum_workspace(size_t rows, size_t cols);
hipError_t launch_colsum(const float* x, size_t rows, size_t cols, const float* row_weight, float* workspace,
                         float* out, hipStream_t stream);
// diagonal-Gaussian log-prob of given actions and its backward (ppo.hip)
hipError_t launch_gauss_logp(const float* mean, int mean_ld, const float* act, const float* log_std, float* logp, int N,
                             int A, hipStream_t stream);
hipError_t launch_gauss_logp_grad(const float* mean, int mean_ld, const float* act, const float* log_std,
                                  const float* g_logp, float* g_mean, float* gls_rows, int N, int A,
                                  hipStream_t stream);
// SB3 PPO minibatch loss (clipped surrogate + value MSE) forward / backward (ppo.hip); workspace
// of ppo_loss_workspace(B) floats, written by the forward and read by the backward
size_t ppo_loss_workspace(int B);
hipError_t launch_ppo_loss_fwd(const float* logp, const float* v, const int64_t* idx, const float* adv,
                               const float* ret, const float* old_logp, int B, float clip, int normalize, float* pg,
                               float* vf, float* ws, hipStream_t stream);
hipError_t launch_ppo_loss_bwd(const float* logp, const float* v, int B, float clip, const float* ws,
                               const float* g_pg, const float* g_vf, float* g_logp, float* g_v, hipStream_t stream);
// clip_grad_norm_ + Adam over up to 1024 tensors (ppo.hip); part: adam_partials(total numel) floats
int adam_partials(long long total);
hipError_t launch_adam_clip(int nt, float* const* p, const float* const* g, float* const* m, float* const* v,
                            float* const* step, const long long* numel, float* part, float max_norm, double lr,
                            double b1, double b2, double eps, hipStream_t stream);
// ReLU-backward + bias-gradient first pass, and a paired single-pass column sum (ppo.hip)
size_t colsum_partial_rows(size_t rows, size_t cols);
// (G W) masked by X > 0 and its per-workgroup column sums (ppo.hip dgrad_mask_*_kernel): the input
// gradient of a Linear layer fed by a ReLU, fused with that ReLU's backward; N = 256
hipError_t launch_dgrad_mask(const float* G, int ldg, int K, const float* W, int ldw, const float* X, int ldx, int B,
                             int N, float* GX, float* partial, float* workspace, hipStream_t stream);
size_t dgrad_mask_partial_rows(int B, int K);
size_t dgrad_mask_workspace(int K);
hipError_t launch_relu_colsum(const float* g, const float* y, size_t rows, size_t cols, float* gm, float* partial,
                              hipStream_t stream);
hipError_t launch_colsum_pair(const float* x0, size_t rows0, size_t cols0, float* out0, const float* x1, size_t rows1,
                              size_t cols1, float* out1, hipStream_t stream);
// GAE reverse scan over [T][N] float32 rollout arrays (gae.hip)
hipError_t launch_gae(const float* rew, const float* val, const float* start, const float* last_val,
                      const float* last_done, float* adv, float* ret, int T, int N, float gamma, float lam,
                      hipStream_t stream);

}  // namespace hs

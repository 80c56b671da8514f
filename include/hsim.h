/* hsim -- MI355X-native batched humanoid simulation: the drop-in C ABI.
 *
 * This is the boundary the reference's Python env would bind instead of the `mujoco`
 * pybind11 module + SB3's SubprocVecEnv.  Each entry point names the reference interface it
 * replaces (paths relative to the reference repo):
 *
 *   hs_model_load        <- mujoco.MjModel.from_xml_path(model_path)      custom_env.py:53
 *   hs_model_field       <- MjModel attribute reads (nq, nv, nu, body_mass, ...) custom_env.py:87,59-61
 *                           (+ "contact_bound": the 4 static worst-case counts of hs_batch_info)
 *   hs_batch_create      <- mujoco.MjData(model) per env                  custom_env.py:54
 *                           x SubprocVecEnv([make_env(...)] * n_envs)     train_sb3.py:203
 *   hs_set_seed          <- VecEnv.seed / np.random.seed(seed) of reset (custom_env.py:99-100)
 *   hs_set_config        <- env_config keys duration/frame_skip/reward_config custom_env.py:21-32,
 *                           train_sb3.py:183-200
 *   hs_reset             <- HumanoidEnv.reset: mj_resetData + noise + one mj_step  custom_env.py:97-150
 *   hs_step              <- HumanoidEnv.step: frame_skip x mj_step, _get_state, reward, done
 *                           custom_env.py:152-230 (+ SB3 auto-reset on done)
 *   hs_step_tape         <- K x HumanoidEnv.step over a given action tape (open loop), one launch
 *   hs_rollout           <- SB3 PPO.collect_rollouts' per-step loop (policy + env step + buffers), one launch
 *   hs_physics_step      <- raw `data.ctrl[:] = a; mujoco.mj_step(model, data)` custom_env.py:159-160
 *   hs_pack_outputs      <- the worker -> main-process pipe transfer of SubprocVecEnv.step_wait (obs,
 *                           rewards, dones, info values; train_sb3.py:203): one packed device buffer
 *   hs_reward_eval       <- REWARD_FUNCTIONS[type](data, params) reward_functions.py:66-269 (the device
 *                           formulas of hs_step on supplied fields)
 *   hs_reward            <- the same on the batch's current states (custom_env.py:263-271 _compute_reward)
 *   hs_debug_lose_handoff   (test hook: mj_step's warning + mj_resetData path, custom_env.py:160)
 *   hs_last_tape_ms, hs_tape_aborts, hs_stream_orders, hs_batch_counters   (diagnostics)
 *   hs_state_io          <- reads/writes of data.qpos/qvel/qacc_warmstart/time/ctrl (custom_env.py:105-117)
 *   hs_get_buffers       <- data.* arrays as device buffers (obs, reward, terminated, ...)
 *   hs_last_error        <- mujoco's error callback / MjModel load error string
 *   hs_gae               <- SB3 RolloutBuffer.compute_returns_and_advantage (stable_baselines3 2.3.2
 *                           common/buffers.py), run by PPO.learn once per rollout (train_sb3.py:229)
 *   hs_ppo_act           <- SB3 PPO.collect_rollouts per step (on_policy_algorithm.py, 2.3.2): the
 *                           DiagGaussian sample + log_prob of ActorCriticPolicy.forward, np.clip of
 *                           the actions, RolloutBuffer.add of actions/values/log_probs/episode_starts
 *   hs_ppo_post          <- the same loop after env.step: TimeLimit.truncated bootstrap of the reward,
 *                           dones, episode returns, new episode_starts, next obs into the buffer
 *   hs_gauss_logp(_grad) <- DiagGaussianDistribution.log_prob of the buffered actions in the PPO
 *                           update (SB3 ActorCriticPolicy.evaluate_actions) and its backward
 *   hs_ppo_loss(_grad)   <- SB3 PPO.train's minibatch loss: advantage normalisation, clipped
 *                           surrogate, value MSE (stable_baselines3 2.3.2 ppo/ppo.py) and its backward
 *   hs_adam_clip         <- torch.nn.utils.clip_grad_norm_(max_grad_norm) + torch.optim.Adam.step of
 *                           SB3 PPO.train (ppo.py: max_grad_norm 0.5, Adam eps 1e-5)
 *   hs_dgrad_mask        <- the input gradient of each layer fed by a ReLU, fused with that ReLU's
 *                           backward (same loss.backward())
 *   hs_relu_grad_colsum, hs_colsum_pair <- the ReLU backward + bias / weight-gradient sums of the
 *                           same loss.backward() (fewer passes and launches)
 *   hs_colsum            <- the bias-gradient and split-K weight-gradient reductions of the PPO
 *                           update's loss.backward() (SB3 PPO.train, ppo.py; train_sb3.py:229)
 *
 * Conventions: status int (0 ok, <0 error, message via hs_last_error(), thread-local); the
 * model is immutable and shareable; a batch owns (or is bound to) device buffers; every call
 * takes an optional HIP stream (NULL = default stream) and is asynchronous unless noted; a
 * batch is not re-entrant.  No torch types cross this boundary.
 * Launches of ONE batch are ordered by the library: like one mjData, a batch is a single state (two
 * unordered launches would race on every buffer, and on the chunk-queue schedule share the batch's
 * claim counters, so pairs could be stepped twice or skipped).  A call on another stream than the
 * batch's previous call first makes its stream wait for everything already issued on the old one
 * (an event; counted by hs_stream_orders).  Streams in graph capture are not joined this way: the
 * capturing framework orders a capture against its origin stream.  The library keeps the handle of a
 * batch's last stream to record that event, so a stream a batch was launched on must stay alive until
 * the batch's next call (or hs_batch_destroy).
 * Uncached memory (the chunk queue's hand-off rows and sync words, ~1.2 KB per fp64 env) is recycled
 * within the process as uncached memory only, in power-of-two size classes >= 64 KB: the process keeps
 * at most the peak of concurrently live uncached memory of each class, each block up to twice its
 * request, until it exits.
 */
#ifndef HSIM_H
#define HSIM_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef struct hs_model hs_model;
typedef struct hs_batch hs_batch;

enum { HS_FP32 = 0, HS_FP64 = 1 };
/* OR-ed into hs_batch_create's `precision` argument: the full-state option.  cfrc_ext (contact
 * wrenches, mj_rnePostConstraint) and subtree_linvel (mj_subtreeVel) are computed every substep
 * and the observation gains cfrc_ext[1:] -- the reference's commented-out obs component
 * (custom_env.py:247,255) -- so obs_dim = 352 + 6 (nbody - 1) = 448 for humanoid.xml; rewards then
 * read the real foot forces / com velocity.  Off (default) = the reference's zeros. */
enum { HS_FULL_STATE = 0x100 };
enum { HS_REWARD_NONE = -1, HS_REWARD_STAND = 0, HS_REWARD_KNEELING = 1, HS_REWARD_WALK = 2 };
/* Per-env warning counters (hs_buffers.warning): MuJoCo's mj_checkPos / mj_checkVel / mj_checkAcc
 * resets (mj_step's mju_warning + mj_resetData, custom_env.py:160), contacts dropped past the wide
 * tier, and HS_WARN_HANDOFF: a lost chunk-queue hand-off (a scheduling failure -- e.g. more concurrent
 * queued batches than the GPU holds -- after which the env was reset like a bad state). */
enum { HS_WARN_BADQPOS = 0, HS_WARN_BADQVEL = 1, HS_WARN_BADQACC = 2, HS_WARN_OVERFLOW = 3, HS_WARN_HANDOFF = 4,
       HS_NWARN = 5 };
#define HS_AUXDIM 40   /* per env aux row: qacc[32], com[3], ncon, nefc, newton iterations, pad */
/* Optional per-env outputs (hs_env_config.outputs).  HS_OUT_AUX: the aux row (qacc, subtree com,
 * contact / row counts, solver iterations) that data views and statistics read.  HS_OUT_CTRL: the
 * data.ctrl copy (the action; data views and host reward callables read it,
 * reward_functions.py:194).  A trainer on the device reward needs neither. */
enum { HS_OUT_AUX = 1, HS_OUT_CTRL = 2 };

/* Env semantics (custom_env.py defaults in brackets; train_sb3.py overrides in parentheses). */
typedef struct {
  int frame_skip;          /* [5] (3)   custom_env.py:28, train_sb3.py:199 */
  int max_steps;           /* [750]     custom_env.py:201 forced truncation */
  int reward_id;           /* HS_REWARD_*; reward_config['type'] custom_env.py:263-271 */
  int autoreset;           /* 1 = SB3 VecEnv auto-reset (terminal obs kept in terminal_obs) */
  int max_newton;          /* Newton iteration cap [100 = opt.iterations] */
  int outputs;             /* HS_OUT_* bits: optional per-env outputs [all] */
  double duration;         /* [15] (10.0) custom_env.py:23, train_sb3.py:187 */
  double init_height;      /* 1.282   custom_env.py:59 */
  double noise_scale;      /* 0.01    custom_env.py:109-110 */
  double kneel_params[9];  /* reward_functions.py:71-81: target_height, min_height, max_roll_pitch,
                              com_radius, energy_weight, posture_weight, com_weight, foot_weight,
                              alive_weight */
  int schedule;            /* HS_SCHED_*: how the step kernel maps env pairs to waves [AUTO] */
} hs_env_config;

/* hs_env_config.schedule.  AUTO: one wave per env (the upper half-wave mirrors the lower one and
 * commits nothing) when every env gets a resident wave of its own (small batches, e.g. configs[4]'s
 * 1024 envs per GPU); else one wave per env pair when every pair fits on the GPU at once; else (the
 * fp64 engine at 4096 envs) a persistent grid that runs each env step as two chunk items (substeps
 * [0, frame_skip - 1), then the last substep + obs / reward / auto-reset) from a queue.
 * The queue claims the pairs heaviest first by the durations its previous launch measured.
 * DIRECT: always one wave per pair.  SINGLE: always one wave per env.  FIXED_ORDER: AUTO with the
 * queue's claims in a fixed permutation (A/B runs, tests).  Results are bitwise identical
 * whichever schedule runs. */
enum { HS_SCHED_AUTO = 0, HS_SCHED_DIRECT = 1, HS_SCHED_SINGLE = 2, HS_SCHED_FIXED_ORDER = 3 };

/* Device buffers of a batch (row-major, env-major).  Element type of the T* entries is float
 * (HS_FP32) or double (HS_FP64). */
typedef struct {
  void* qpos;              /* [N][nq]  */
  void* qvel;              /* [N][nv]  */
  void* qacc_warmstart;    /* [N][nv]  */
  void* ctrl;              /* [N][nu]  */
  void* time;              /* [N]      */
  int32_t* step_count;     /* [N]      */
  uint32_t* episode;       /* [N]      */
  void* total_reward;      /* [N]      */
  int32_t* warning;        /* [N][HS_NWARN] */
  void* obs;               /* [N][obs_dim]  custom_env.py:242-256 layout */
  void* terminal_obs;      /* [N][obs_dim]  obs before auto-reset (SB3 info["terminal_observation"]) */
  void* reward;            /* [N]      */
  uint8_t* terminated;     /* [N]      */
  uint8_t* truncated;      /* [N]      */
  void* aux;               /* [N][HS_AUXDIM] */
  void* cfrc_ext;          /* [N][nbody][6]  (torque, force) at the root subtree com; HS_FULL_STATE only */
  void* subtree_linvel;    /* [N][nbody][3]  HS_FULL_STATE only */
  int32_t* terminal_step_count;  /* [N] or NULL: info["step_count"] of envs that auto-reset this step */
  void* terminal_total_reward;   /* [N] or NULL: their info["total_reward"] (custom_env.py:216-224) */
} hs_buffers;

typedef struct {
  int n_envs, precision, nq, nv, nu, nbody, obs_dim, elem_size;
  /* per-env contact / constraint-row capacity of the resident kernel tier (every launch) and of the
   * wide tier that re-runs the envs overflowing it; only wide-tier overflow drops contacts
   * (HS_WARN_OVERFLOW).  MuJoCo has no per-env cap (custom_env.py:160). */
  int resident_con, resident_efc, wide_con, wide_efc;
  /* waves of the resident step kernel the device holds at once (2 envs per wave); with more env
   * pairs than this, HS_SCHED_AUTO runs multi-substep calls on the chunk-queue schedule */
  int resident_waves;
  /* static worst case of one env from the model's collision pair list (most contacts per pair
   * type x rows per contact, + one row per limited joint / tendon): every pair touching at once
   * (geometric, unreachable) and every geom on the floor at once (a flat-lying body).  Models
   * whose floor bound exceeds the wide tier are rejected by hs_batch_create. */
  int bound_con_all, bound_efc_all, bound_con_floor, bound_efc_floor;
} hs_batch_info;

hs_model* hs_model_load(const char* xml_path, char* err, int errsz);
void hs_model_free(hs_model* m);
int hs_model_field(const hs_model* m, const char* name, double* out, int n);

/* external == NULL: the library allocates (hipMalloc) and owns the buffers.
 * external != NULL: every pointer must be a device buffer of the documented size on `device`;
 * the caller keeps ownership (used by the Python layer to hand in torch-allocated tensors). */
hs_batch* hs_batch_create(const hs_model* m, int n_envs, int device, uint64_t seed, int precision /* | flags */,
                          const hs_buffers* external);
void hs_batch_destroy(hs_batch* b);
int hs_batch_get_info(const hs_batch* b, hs_batch_info* out);
int hs_get_buffers(const hs_batch* b, hs_buffers* out);
int hs_set_config(hs_batch* b, const hs_env_config* cfg);
/* Base seed of the on-device reset RNG (VecEnv.seed; SB3 seeds workers with seed + rank). */
int hs_set_seed(hs_batch* b, uint64_t seed);
int hs_get_config(const hs_batch* b, hs_env_config* cfg);

/* mask: [N] uint8 device (NULL = all envs).  qpos_noise/qvel_noise: [N][nq]/[N][nv] device
 * arrays of the batch precision with the reset noise (NULL = on-device counter RNG). */
int hs_reset(hs_batch* b, const uint8_t* mask, const void* qpos_noise, const void* qvel_noise, void* stream);
/* actions: [N][nu] float32 device. Runs frame_skip substeps, writes obs/reward/terminated/truncated. */
int hs_step(hs_batch* b, const float* actions, void* stream);
/* Per-step outputs of hs_step_tape, device arrays (batch precision for obs / reward):
 * obs [K][N][obs_dim], reward [K][N], terminated / truncated [K][N] uint8. */
typedef struct hs_tape_out {
  void* obs;
  void* reward;
  uint8_t* terminated;
  uint8_t* truncated;
} hs_tape_out;
/* K = n_steps consecutive hs_step calls over an action tape: actions [K][N][nu] float32 device.
 * Same results, bitwise, as K hs_step calls (states, per-step obs / reward / done flags, auto-resets
 * and their final-step info; the terminal obs / info rows hold each env's last finished episode).
 * One launch on the chunk-queue schedule with whole env steps as items: an env pair's step t + 1
 * starts as soon as its own step t is committed, so steps of different pairs overlap and the launch
 * does not end every step on its slowest pair.  out = NULL: only the batch's buffers (last step);
 * otherwise every step's outputs, and the batch buffers as after the last step.  If an env overflows
 * the resident contact tier the launch stops and the tape is replayed step by step (counted by
 * hs_tape_aborts).  Synchronizes the stream.  K >= 1: the host splits the tape into launches of at
 * most min(the shortest episode, 511) steps (hs_rollout_max_steps).  With HS_SCHED_DIRECT / SINGLE, or
 * K = 1, it runs the K hs_step calls.  Open-loop stepping (a given action tape: benchmarks,
 * trajectory evaluation); a policy in the loop steps with hs_step. */
int hs_step_tape(hs_batch* b, const float* actions, int n_steps, const hs_tape_out* out, void* stream);
/* tape launches of this batch that were replayed step by step (resident-tier overflow) */
int hs_tape_aborts(const hs_batch* b, uint64_t* n);
/* duration in ms of the last tape / rollout kernel launch of this batch (hs_step_tape, hs_rollout), from
 * HIP events recorded around it on its stream; -1 before the first one (diagnostics: the bench's roofline) */
int hs_last_tape_ms(const hs_batch* b, double* ms);
/* cross-stream waits the library inserted to keep this batch's launches ordered (diagnostics) */
int hs_stream_orders(const hs_batch* b, uint64_t* n);

/* Fused PPO rollout (the fp64 Newton engine).  The SB3 MlpPolicy's pi net -- two hidden layers of
 * 256, ReLU, then the action head, fp32 -- with [in][out] row-major weights (w1 [obs_dim][ld1],
 * columns 0..255 the pi net's, w2 [256][256], w3 [256][act_dim]) and the DiagGaussian log_std. */
typedef struct hs_policy {
  const float *w1, *b1, *w2, *b2, *w3, *b3, *log_std;
  int ld1, obs_dim, act_dim;
} hs_policy;
/* The RolloutBuffer of SB3 PPO.collect_rollouts (on_policy_algorithm.py, 2.3.2) for t_total steps of
 * N envs, device arrays: obs [t_total][N][obs_dim] (row 0 = the rollout's first obs), obs_last
 * [N][obs_dim] (the obs after the last step), actions [t_total][N][act_dim] (unclipped samples),
 * log_probs / episode_starts / rewards [t_total][N] f32, dones / boot [t_total][N] u8 (boot:
 * TimeLimit.truncated and not terminated), episode_returns [t_total][N] f64, terminal_obs
 * [t_total][N][obs_dim] (rows of the boot envs), ep_acc [N] f64 (running return, in / out),
 * episode_start [N] f32 (out), actions_clipped [N][act_dim] (in: step t_begin's clipped action;
 * out: step t_begin + n_steps'), counter_base (device u64) and seed: the noise of hs_ppo_act. */
typedef struct hs_rollout_bufs {
  float* obs;
  float* obs_last;
  float* actions;
  float* log_probs;
  float* episode_starts;
  float* rewards;
  uint8_t* dones;
  double* episode_returns;
  uint8_t* boot;
  float* terminal_obs;
  double* ep_acc;
  float* episode_start;
  float* actions_clipped;
  const uint64_t* counter_base;
  uint64_t seed;
  int deterministic;
} hs_rollout_bufs;
/* Steps [t_begin, t_begin + n_steps) of a PPO rollout in ONE launch: hs_step with the given clipped
 * action for step t_begin, then for every later step the policy forward on the returned obs, the
 * Gaussian sample (hs_ppo_act's Philox stream, counter step + *counter_base), the clip, and
 * hs_ppo_post's bookkeeping (rewards, dones, episode returns, bootstrap flags / terminal obs, the
 * next obs row, episode_start) -- on each env's wave, each env pair's step t + 1 starting when its
 * own step t is done.  Replaces the per-step loop of SB3 collect_rollouts (train_sb3.py:229 ->
 * on_policy_algorithm.py) for envs stepped by this engine; values are evaluated after the rollout.
 * n_steps <= hs_rollout_max_steps(b) (the shortest episode, at most 511 steps).  Returns 0, or 1 when an env overflowed
 * the resident contact tier: the env state, ep_acc, episode_start and actions_clipped are restored
 * to the call's start, and the caller collects these steps step by step (hs_step).  Synchronizes. */
int hs_rollout(hs_batch* b, const hs_policy* pol, const hs_rollout_bufs* rb, int t_begin, int n_steps, int t_total,
               void* stream);
int hs_rollout_max_steps(const hs_batch* b);
/* Auto-reset noise source of hs_step: [N][nq] / [N][nv] device arrays of the batch precision with
 * the raw U(-noise_scale, noise_scale) draws of the NEXT reset of each env (the kernel applies the
 * x0.1 height factor and zeroes the quaternion part, custom_env.py:109-114); NULL, NULL = the
 * on-device counter RNG (default).  The caller refreshes an env's row after it auto-resets -- the
 * SubprocVecEnv-exact mode where worker i continues its own np.random stream seeded with
 * seed + i (custom_env.py:99-110, SB3 VecEnv.seed).  The arrays stay owned by the caller. */
int hs_set_autoreset_noise(hs_batch* b, const void* qpos_noise, const void* qvel_noise);
/* One step's host-bound outputs in ONE launch, for a single device-to-host copy (the SubprocVecEnv
 * step_wait / Gym step() return values, custom_env.py:216-230, train_sb3.py:203): writes the float64
 * device buffer out = [obs N x obs_dim][ncols x N columns of reward, terminated, truncated,
 * total_reward, step_count, terminal_step_count, terminal_total_reward (first ncols of them)]
 * [warnings ? HS_NWARN x N warning counters (kind-major) : nothing].  Asynchronous on `stream`. */
int hs_pack_outputs(hs_batch* b, double* out, int ncols, int warnings, void* stream);
/* ctrl: [N][nu] float32 device (NULL = keep current ctrl).  nsub raw mj_step's, obs refreshed.
 * Resets and raw physics calls always write data.ctrl; env steps (hs_step) only with HS_OUT_CTRL.
 * After an hs_step with HS_OUT_CTRL off the ctrl buffer no longer holds data.ctrl, and until it is
 * rewritten (a full hs_reset, an hs_physics_step with ctrl, an hs_state_io set of ctrl) both
 * hs_physics_step(ctrl = NULL) and an hs_state_io get of ctrl fail instead of using it. */
int hs_physics_step(hs_batch* b, const float* ctrl, int nsub, void* stream);
/* Test hook of the chunk-queue schedule (never used on the product path): from the next launch on,
 * the hand-off of env `env`'s pair (env / 2) is treated as lost by its consumer item, exactly as
 * if its bounded wait had timed out -- both envs of the pair are reset as mj_checkPos resets a bad
 * state (qpos0, qvel 0, time 0), HS_WARN_HANDOFF += 1, and the step continues from there.
 * env = -1 turns it off.  Only launches on the queued schedule consult it. */
int hs_debug_lose_handoff(hs_batch* b, int env);

/* Synchronous host<->device state copy in fp64.  dir 0: device -> host, 1: host -> device.
 * Any pointer may be NULL.  Arrays are [N][nq], [N][nv], [N][nv], [N], [N][nu]. */
int hs_state_io(hs_batch* b, int dir, double* qpos, double* qvel, double* qacc_warmstart, double* time,
                double* ctrl);
/* mj_kinematics + mj_comPos of env `env` (visualisation; the pose data mujoco.Renderer.update_scene
 * reads from mjData at custom_env.py:284-288).  qpos: nq fp64 values to pose instead of the env's
 * current state (NULL = current).  Outputs, each nullable: xpos [nbody][3], xmat [nbody][9],
 * geom_xpos [ngeom][3], geom_zaxis [ngeom][3] (capsule axis), com [3] (subtree_com of the root).
 * Synchronous; not on the step path. */
int hs_kinematics(hs_batch* b, int env, const double* qpos, double* xpos, double* xmat, double* geom_xpos,
                  double* geom_zaxis, double* com);
/* Stage dump of env 0 after its last substep (parity debugging); n >= 16384 doubles. */
int hs_set_debug(hs_batch* b, int enable);
int hs_get_debug(hs_batch* b, double* out, int n);
int hs_synchronize(hs_batch* b);
/* Diagnostics (synchronous): *wide_reruns = cumulative count of env steps whose contacts or
 * constraint rows overflowed the resident kernel tier (32 contacts / 128 rows) and were re-run by
 * the wide tier (64 / 256); contacts are only dropped (HS_WARN_OVERFLOW) past the wide tier. */
int hs_batch_counters(const hs_batch* b, uint64_t* wide_reruns);

/* The device reward plug-ins on supplied fields <- REWARD_FUNCTIONS[type](env_data, params)
 * (reward_functions.py:66-269, utils.py:3-21; called at custom_env.py:263-271).  Runs the SAME device
 * code the step kernel inlines after each env step (reward_formula + numpy-order sums), on n states
 * given as device arrays of the `precision` type (HS_FP32 / HS_FP64): qpos [n][nq], qvel [n][nv],
 * ctrl [n][nu], time [n], subtree_com0 / subtree_linvel0 [n][3] (subtree_com[0], subtree_linvel[0]),
 * cfrc_ext [n][nbody][6], qfrc_actuator [n][nv]; writes out [n].  reward_id: HS_REWARD_STAND ("default",
 * "stand"), HS_REWARD_KNEELING, HS_REWARD_WALK; kneel_params: 9 host doubles in hs_env_config's order
 * (NULL = the reference defaults, reward_functions.py:71-81).  The step kernel itself passes zeros for
 * cfrc_ext / subtree_linvel unless HS_FULL_STATE (mj_step leaves them uncomputed).  Asynchronous. */
int hs_reward_eval(const hs_model* m, int precision, int reward_id, const double* kneel_params, int n,
                   const void* qpos, const void* qvel, const void* ctrl, const void* time, const void* subtree_com0,
                   const void* subtree_linvel0, const void* cfrc_ext, const void* qfrc_actuator, void* out,
                   void* stream);

/* The reward of every env's current state under any built-in reward <- REWARD_FUNCTIONS[type](data, params)
 * on each env's data (custom_env.py:263-271): hs_reward_eval on the batch's own buffers (qpos, qvel,
 * data.ctrl, time, the aux row's subtree com, subtree_linvel / cfrc_ext -- zeros unless HS_FULL_STATE,
 * as mj_step leaves them -- and the obs row's qfrc_actuator), so it needs HS_OUT_AUX | HS_OUT_CTRL written
 * by the last step.  out: [N] of the batch precision (device).  kneel_params NULL = the batch's.  After an
 * hs_step with reward_id r it equals the step's reward buffer bitwise, except for truncated envs (which
 * the step rewards 0, custom_env.py:201-211) and envs that auto-reset (whose buffers hold the reset
 * state).  Asynchronous. */
int hs_reward(hs_batch* b, int reward_id, const double* kneel_params, void* out, void* stream);

/* GAE(gamma, lambda) reverse scan over a device rollout buffer, SB3 semantics: [T][N] float32
 * rewards, values, episode_starts; [N] last_values, last_dones; writes [T][N] advantages and
 * returns (= advantages + values).  All pointers are device memory on the current device;
 * asynchronous on `stream`.  advantages / returns must not overlap the inputs or each other (checked:
 * an error, not wrong advantages): for T >= 256 the scan runs as three launches that keep their
 * per-chunk maps and carries in those output rows. */
int hs_gae(const float* rewards, const float* values, const float* episode_starts, const float* last_values,
           const float* last_dones, float* advantages, float* returns, int T, int N, float gamma, float gae_lambda,
           void* stream);
/* One PPO rollout step's policy sampling and buffer writes over N envs (A <= 32 actions):
 * mean [N][mean_ld] (first A columns), value [N] at stride value_ld, log_std [A], episode_start
 * [N] (all float32 device memory).  actions = mean + exp(log_std) * z with z ~ N(0, 1) from the
 * counter-based Philox4x32-10 stream (seed, counter + *counter_base when counter_base (a device
 * uint64) is not NULL -- graph replays then draw fresh noise; z = 0 when deterministic != 0); writes
 * actions [N][A] (unclipped, the buffer copy), actions_clipped [N][A] (clip to [-1, 1], what the
 * env steps with), log_prob [N], values [N] and episode_starts_out [N].  Asynchronous on `stream`. */
/* Fused forward of one 2-hidden-layer ReLU MLP (H = 256): out[N][A] = relu(relu(X W1' + b1) W2' + b2)
 * W3' + b3, weights as nn.Linear stores them, [out][in] row-major (W1 [256][ld1 >= D], W2 [256][ld2],
 * W3 [A][ld3], ld2 / ld3 >= 256); D <= 512, A <= 32.  16-byte weight loads when every weight row
 * is 16-byte aligned, element loads otherwise.  Replaces the three GEMMs of SB3's MlpPolicy forward (ActorCriticPolicy.forward ->
 * mlp_extractor -> action_net / value_net, policies.py, SB3 2.3.2) in the rollout: the pi net's mean
 * per env step and the vf net's values over the rollout buffer.  fp32 in, fp32 MFMA accumulation.
 * Asynchronous on `stream`. */
int hs_mlp2_forward(const float* X, int ldx, int D, int N, const float* W1, int ld1, const float* b1, const float* W2,
                    int ld2, const float* b2, const float* W3, int ld3, const float* b3, int A, float* out, int ldo,
                    void* stream);
int hs_ppo_act(const float* mean, int mean_ld, const float* value, int value_ld, const float* log_std,
               const float* episode_start, uint64_t seed, uint64_t counter, const uint64_t* counter_base,
               int deterministic, float* actions,
               float* actions_clipped, float* log_prob, float* values, float* episode_starts_out, int N, int A,
               void* stream);
/* The rest of the PPO rollout step after the env step, over N envs: reward [N] float32,
 * terminated / truncated [N] uint8.  boot = truncated && !terminated (TimeLimit.truncated).
 * Immediate bootstrap: terminal_value [N] = V(terminal obs) given -> reward_out = reward +
 * gamma * terminal_value where boot (else reward).  Deferred bootstrap: terminal_value NULL ->
 * reward_out = reward, boot_out [N] uint8 = boot, and for boot envs the terminal_obs row (obs_dim
 * float32) is copied to boot_obs_out (row n); the caller adds gamma V(row) at the end of the
 * rollout.  Both: done_out = terminated || truncated (uint8), ep_acc += reward (float64, zeroed
 * where done, after ep_return_out = the accumulated value is written), episode_start = done
 * (float32), and obs_floats float32 copied from obs to obs_out (the next rollout-buffer slot;
 * NULL obs skips it).  Asynchronous on `stream`. */
int hs_ppo_post(const float* reward, const uint8_t* terminated, const uint8_t* truncated, const float* terminal_value,
                const float* terminal_obs, float* boot_obs_out, uint8_t* boot_out, int obs_dim, float gamma,
                const float* obs, float* obs_out, uint64_t obs_floats, float* reward_out, uint8_t* done_out,
                double* ep_acc, double* ep_return_out, float* episode_start, int N, void* stream);
/* logp[n] = sum_j (-z^2/2 - log_std[j]) - A log(sqrt(2 pi)), z = (actions[n][j] - mean[n][j]) /
 * exp(log_std[j]); mean [N][mean_ld], actions [N][A] contiguous, A <= 32.  The backward, given
 * g_logp [N]: g_mean[n][j] = g z / sigma and gls_rows[n][j] = g (z^2 - 1), whose column sums
 * (hs_colsum) are dL/dlog_std.  Asynchronous on `stream`. */
int hs_gauss_logp(const float* mean, int mean_ld, const float* actions, const float* log_std, float* logp, int N,
                  int A, void* stream);
int hs_gauss_logp_grad(const float* mean, int mean_ld, const float* actions, const float* log_std,
                       const float* g_logp, float* g_mean, float* gls_rows, int N, int A, void* stream);
/* SB3 PPO minibatch loss over B samples gathered by idx [B] (int64) from the rollout arrays
 * advantages / returns / old_log_prob [M]: log_prob [B] and values [B] are the policy's on the
 * minibatch.  a = advantages[idx] normalised (mean, unbiased std + 1e-8; not when B == 1, nor when
 * normalize_advantage == 0: SB3's PPO(normalize_advantage=False)),
 * r = exp(log_prob - old_log_prob[idx]); writes policy_loss = -mean(min(a r, a clip(r, 1 -+ clip)))
 * and value_loss = mean((returns[idx] - values)^2) (device scalars).  `workspace` holds
 * hs_ppo_loss_workspace(B) floats: the forward leaves the gathered minibatch and the
 * normalisation there for the backward, which, given the upstream device scalars g_pg, g_vf,
 * writes dL/dlog_prob [B] and dL/dvalues [B] with torch's min/clamp derivative conventions.
 * Fixed reduction order (deterministic); asynchronous on `stream`. */
uint64_t hs_ppo_loss_workspace(int B);
int hs_ppo_loss(const float* log_prob, const float* values, const int64_t* idx, const float* advantages,
                const float* returns, const float* old_log_prob, int B, float clip, int normalize_advantage,
                float* policy_loss, float* value_loss, float* workspace, void* stream);
int hs_ppo_loss_grad(const float* log_prob, const float* values, int B, float clip, const float* workspace,
                     const float* g_pg, const float* g_vf, float* g_log_prob, float* g_values, void* stream);
/* Gradient-norm clipping + one Adam step over nt <= 1024 float32 device tensors: params[i],
 * grads[i], exp_avg[i], exp_avg_sq[i] (numel[i] elements each) and step[i] (a float32 device
 * scalar per tensor, torch's capturable Adam state; all tensors share one step count).  With
 * c = min(1, max_norm / (||grads||_2 + 1e-6)) (max_norm <= 0: c = 1) and t = step + 1:
 * m = b1 m + (1-b1) c g; v = b2 v + (1-b2) (c g)^2; p -= lr / (1 - b1^t) * m / (sqrt(v) /
 * sqrt(1 - b2^t) + eps); step = t (1 - beta rounded to float from double, as torch's scalar
 * arguments are).  Grads are read, not modified.  `workspace` holds
 * hs_adam_workspace(sum numel) floats.  Pointer tables are host arrays (copied into the kernel
 * arguments); asynchronous on `stream`. */
uint64_t hs_adam_workspace(uint64_t total_numel);
int hs_adam_clip(int nt, float* const* params, const float* const* grads, float* const* exp_avg,
                 float* const* exp_avg_sq, float* const* step, const int64_t* numel, float* workspace, float max_norm,
                 double lr, double beta1, double beta2, double eps, void* stream);
/* out[c] = sum_r w[r] x[r][c] over a row-major [rows][cols] float32 device matrix (w = row_weight
 * [rows], or 1 when NULL -- the weighted form is a rank-1 weight gradient g'x), in a fixed
 * summation order (deterministic).  `workspace` must hold hs_colsum_workspace(rows, cols) floats
 * (may be NULL when that is 0).  Asynchronous on `stream`. */
/* ReLU backward fused with the bias gradient's first reduction pass, for a [rows][cols] float32
 * upstream gradient g and the layer's ReLU output y: writes gm = (y > 0) ? g : 0 and per-chunk
 * column sums of gm to partial [hs_colsum_partial_rows(rows, cols)][cols]. */
uint64_t hs_colsum_partial_rows(uint64_t rows, uint64_t cols);
int hs_relu_grad_colsum(const float* g, const float* y, uint64_t rows, uint64_t cols, float* gm, float* partial,
                        void* stream);
/* Input gradient of a Linear layer fed by a ReLU, fused with that ReLU's backward and the first
 * pass of its bias gradient: GX[B][N] = (G W) masked by X > 0, partial[p][N] = column sums of GX
 * over row block p, p < hs_dgrad_mask_partial_rows(B, K).  G [B][K] (row stride ldg) is the layer's
 * output gradient, W [K][N] its weight as nn.Linear stores it ([out][in], row stride ldw), X [B][N]
 * (ldx) its input = the previous layer's ReLU output; GX is contiguous.  N = 256; K <= 32 (a policy
 * or value head) or K % 16 == 0, K <= 512 (a hidden layer: fp32 MFMA, G rows 16-byte aligned, and
 * `workspace` of hs_dgrad_mask_workspace(K) floats for W transposed; may be NULL when that is 0).
 * Replaces `g @ w` + threshold_backward + the bias sum's first read of SB3's loss.backward() through
 * mlp_extractor (policies.py, SB3 2.3.2).  Asynchronous on `stream`. */
uint64_t hs_dgrad_mask_partial_rows(int B, int K);
uint64_t hs_dgrad_mask_workspace(int K);
int hs_dgrad_mask(const float* G, int ldg, int K, const float* W, int ldw, const float* X, int ldx, int B, int N,
                  float* GX, float* partial, float* workspace, void* stream);
/* Two single-pass column sums in one launch: out0[c] = sum_r x0[r][c] ([rows0][cols0]) and
 * out1[c] = sum_r x1[r][c] ([rows1][cols1]) -- for short matrices (split-K slices, partials). */
int hs_colsum_pair(const float* x0, uint64_t rows0, uint64_t cols0, float* out0, const float* x1, uint64_t rows1,
                   uint64_t cols1, float* out1, void* stream);
uint64_t hs_colsum_workspace(uint64_t rows, uint64_t cols);
int hs_colsum(const float* x, uint64_t rows, uint64_t cols, const float* row_weight, float* workspace, float* out,
              void* stream);
const char* hs_last_error(void);
const char* hs_version(void);

#ifdef __cplusplus
}
#endif
#endif

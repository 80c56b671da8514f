// hsim PPO rollout kernels for gfx950 (MI355X).  PRODUCT CODE.
//
// The per-step bookkeeping of SB3 2.3.2 PPO.collect_rollouts (stable_baselines3/common/
// on_policy_algorithm.py), which the reference's PPO.learn runs n_steps times per rollout
// (train_sb3.py:229), as two launches per env step around the policy GEMMs and the env kernel:
//
//   ppo_act_kernel   ActorCriticPolicy.forward's DiagGaussianDistribution.sample() + log_prob()
//                    (common/distributions.py) on the policy heads, the clip of the actions to
//                    the action space (on_policy_algorithm.py: np.clip(actions, low, high)) and
//                    the rollout-buffer writes of step t (actions, values, log_probs,
//                    episode_starts; common/buffers.py RolloutBuffer.add)
//   ppo_post_kernel  the step's reward bookkeeping: time-limit bootstrap
//                    r += gamma V(terminal_obs) for envs with TimeLimit.truncated (or, deferred,
//                    the boot flags and terminal-obs rows for one batched V at rollout end)
//                    (on_policy_algorithm.py: infos[idx]["TimeLimit.truncated"]), dones,
//                    episode-return accumulation, the new episode_starts, and the copy of the
//                    next observation into the rollout buffer's slot t+1
//
// Both are HBM/launch-bound elementwise work (no GEMM shape), so they are laid out for
// coalescing: ppo_act maps a half-wave (32 lanes) onto one env's action vector (A <= 32), so
// a wave touches two consecutive 84 B head rows and the log-prob sum is a 5-step DPP/swizzle
// reduction within the half-wave; ppo_post moves the [N][D] observation copy as 16 B vectors.
//
// Noise: Philox4x32-10 (Salmon et al., SC'11) keyed by the 64-bit seed, counter =
// (env * 32 + action index, rollout-step counter), and a Box-Muller transform of two of its
// words: a counter-based stream, so every (env, step, action) draw is independent of the
// launch shape and reproducible from (seed, counter).
#include <hip/hip_runtime.h>

#include <algorithm>

#include <cstdint>
#include <cstdlib>

#include "hs_philox.h"

namespace hs {
namespace {

__global__ __launch_bounds__(256) void ppo_act_kernel(const float* __restrict__ mean, int mean_ld,
                                                      const float* __restrict__ value, int value_ld,
                                                      const float* __restrict__ log_std,
                                                      const float* __restrict__ episode_start, uint32_t k0,
                                                      uint32_t k1, uint64_t counter,
                                                      const uint64_t* __restrict__ counter_base, int deterministic,
                                                      float* __restrict__ act, float* __restrict__ act_clip,
                                                      float* __restrict__ logp, float* __restrict__ val,
                                                      float* __restrict__ start_out, int N, int A) {
  const int gid = blockIdx.x * blockDim.x + threadIdx.x;
  const int n = gid >> 5, j = gid & 31;
  if (n >= N) return;                         // whole half-waves exit together (N*32 lanes)
  float term = 0.f;
  if (j < A) {
    const float m = mean[(size_t)n * mean_ld + j];
    const float ls = log_std[j];
    float z = 0.f;
    if (!deterministic) {
      const uint64_t c = counter + (counter_base ? *counter_base : 0ull);
      z = policy_noise((uint32_t)n, (uint32_t)j, c, k0, k1);   // counter block (env * 32 + j, env >> 27, c)
    }
    const float a = m + __expf(ls) * z;
    const size_t i = (size_t)n * A + j;
    act[i] = a;
    act_clip[i] = fminf(fmaxf(a, -1.0f), 1.0f);
    // DiagGaussian log_prob: sum_j -((a-m)^2 / (2 sigma^2)) - log sigma - log(sqrt(2 pi))
    term = -0.5f * z * z - ls - 0.91893853320467274f;
  }
  const float lp = half_sum(term);
  if (j == 0) {
    logp[n] = lp;
    val[n] = value[(size_t)n * value_ld];
    start_out[n] = episode_start[n];
  }
}

__global__ __launch_bounds__(256) void ppo_post_kernel(const float* __restrict__ reward,
                                                       const uint8_t* __restrict__ terminated,
                                                       const uint8_t* __restrict__ truncated,
                                                       const float* __restrict__ terminal_value,
                                                       const float* __restrict__ terminal_obs,
                                                       float* __restrict__ boot_obs_out,
                                                       uint8_t* __restrict__ boot_out, float gamma,
                                                       const float* __restrict__ obs, float* __restrict__ obs_out,
                                                       size_t obs_n, int vec4, float* __restrict__ reward_out,
                                                       uint8_t* __restrict__ done_out, double* __restrict__ ep_acc,
                                                       double* __restrict__ ep_return_out,
                                                       float* __restrict__ episode_start, int N, int obs_dim) {
  const size_t gid = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  const size_t stride = (size_t)gridDim.x * blockDim.x;
  if (vec4) {   // 16 B-aligned pointers, obs_n = floats / 4
    const float4* __restrict__ src = reinterpret_cast<const float4*>(obs);
    float4* __restrict__ dst = reinterpret_cast<float4*>(obs_out);
    for (size_t i = gid; i < obs_n; i += stride) dst[i] = src[i];
  } else {
    for (size_t i = gid; i < obs_n; i += stride) obs_out[i] = obs[i];
  }
  if (gid < (size_t)N) {
    const bool term = terminated[gid] != 0, trunc = truncated[gid] != 0;
    const float r = reward[gid];
    // TimeLimit.truncated = truncated and not terminated: bootstrap from V(terminal obs), now
    // (terminal_value given) or deferred to the end of the rollout (boot flag + the terminal obs
    // row kept in boot_obs_out; rows are copied only for the rare boot envs)
    const bool boot = trunc && !term;
    if (terminal_value) {
      reward_out[gid] = boot ? r + gamma * terminal_value[gid] : r;
    } else {
      reward_out[gid] = r;
      boot_out[gid] = boot;
      if (boot)
        for (int k = 0; k < obs_dim; k++)
          boot_obs_out[gid * obs_dim + k] = terminal_obs[gid * obs_dim + k];
    }
    const bool done = term || trunc;
    const double acc = ep_acc[gid] + (double)r;
    done_out[gid] = done;
    ep_return_out[gid] = acc;
    ep_acc[gid] = done ? 0.0 : acc;
    episode_start[gid] = done ? 1.0f : 0.0f;
  }
}


// DiagGaussianDistribution.log_prob of given actions (SB3 common/distributions.py), the PPO
// update's evaluate_actions, and its backward: with z = (a - mean) / sigma and upstream g = dL/dlogp,
//   logp       = sum_j (-z_j^2 / 2 - log sigma_j) - A log(sqrt(2 pi))
//   dL/dmean_j = g z_j / sigma_j
//   dL/dlog sigma_j = sum_rows g (z_j^2 - 1)     (the per-row terms are written to `gls_rows`;
//                                                the batch sum is colsum_kernel's)
// Half-wave per row (A <= 32), as ppo_act_kernel.
__global__ __launch_bounds__(256) void gauss_logp_kernel(const float* __restrict__ mean, int mean_ld,
                                                         const float* __restrict__ act,
                                                         const float* __restrict__ log_std,
                                                         float* __restrict__ logp, int N, int A) {
  const int gid = blockIdx.x * blockDim.x + threadIdx.x;
  const int n = gid >> 5, j = gid & 31;
  if (n >= N) return;
  float term = 0.f;
  if (j < A) {
    const float ls = log_std[j];
    const float z = (act[(size_t)n * A + j] - mean[(size_t)n * mean_ld + j]) * __expf(-ls);
    term = -0.5f * z * z - ls - 0.91893853320467274f;
  }
  const float lp = half_sum(term);
  if (j == 0) logp[n] = lp;
}

__global__ __launch_bounds__(256) void gauss_logp_grad_kernel(const float* __restrict__ mean, int mean_ld,
                                                              const float* __restrict__ act,
                                                              const float* __restrict__ log_std,
                                                              const float* __restrict__ g_logp,
                                                              float* __restrict__ g_mean,
                                                              float* __restrict__ gls_rows, int N, int A) {
  const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;   // element of [N][A]
  if (i >= (size_t)N * A) return;
  const size_t n = i / A;
  const int j = (int)(i - n * A);
  const float ls = log_std[j];
  const float inv = __expf(-ls);
  const float z = (act[i] - mean[n * mean_ld + j]) * inv;
  const float g = g_logp[n];
  g_mean[i] = g * z * inv;
  gls_rows[i] = g * (z * z - 1.0f);
}

// SB3 PPO.train's per-minibatch loss terms (stable_baselines3 2.3.2 ppo/ppo.py) over a minibatch
// gathered by idx from the rollout arrays (the torch restatement is ~25 small kernels):
//   a     = adv[idx];  a_n = (a - mean(a)) / (std(a) + 1e-8)       (std unbiased; skipped if B = 1)
//   r     = exp(logp - old_logp[idx])
//   pg    = -mean(min(a_n r, a_n clamp(r, 1 - clip, 1 + clip)))
//   vf    = mean((ret[idx] - v)^2)
// Backward (torch's derivative conventions: min splits ties, clamp passes its closed interval):
//   dpg/dlogp_i = -(1/B) r_i dmin_i,  dmin_i = a_n [s1 < s2] + a_n [r in range] [s1 > s2] + ties / 2
//   dvf/dv_i    = 2 (v_i - ret_i) / B
// The random gathers bound the work (each lane of a gather touches its own cache line), so they
// are spread over LOSS_BLOCKS-wide grids: loss_gather writes the gathered a / old_logp / ret
// compactly (the backward reads those coalesced) with per-block sums of a - a_0 and (a - a_0)^2
// (shifted by the minibatch's first advantage against cancellation); loss_terms reduces those
// partials in a fixed order (deterministic) and forms per-block surrogate / MSE sums; loss_final
// writes the two scalars.  Workspace: 3 B + 4 blocks floats + 2 stats.
constexpr int LOSS_TPB = 256;

__device__ inline float block_sum256(float v, float* red) {
  for (int o = 32; o >= 1; o >>= 1) v += __shfl_xor(v, o);
  const int w = threadIdx.x >> 6, l = threadIdx.x & 63;
  __syncthreads();
  if (l == 0) red[w] = v;
  __syncthreads();
  return (red[0] + red[1]) + (red[2] + red[3]);
}

__global__ __launch_bounds__(LOSS_TPB) void loss_gather_kernel(const int64_t* __restrict__ idx,
                                                               const float* __restrict__ adv,
                                                               const float* __restrict__ ret,
                                                               const float* __restrict__ old_logp, int B,
                                                               float* __restrict__ ws) {
  __shared__ float red[LOSS_TPB / 64];
  const int i = blockIdx.x * LOSS_TPB + threadIdx.x;
  float* a_g = ws;
  float* old_g = ws + B;
  float* ret_g = ws + 2 * (size_t)B;
  float* part = ws + 3 * (size_t)B;            // [blocks][4]: sum d, sum d^2, sum pg, sum vf
  const float a0 = adv[idx[0]];
  float d = 0.f;
  if (i < B) {
    const int64_t j = idx[i];
    const float a = adv[j];
    a_g[i] = a;
    old_g[i] = old_logp[j];
    ret_g[i] = ret[j];
    d = a - a0;
  }
  const float s1 = block_sum256(d, red);
  const float s2 = block_sum256(d * d, red);
  if (threadIdx.x == 0) {
    part[4 * blockIdx.x + 0] = s1;
    part[4 * blockIdx.x + 1] = s2;
  }
}

// sum over blocks of part[4 k + c], by one full wave (lane-strided, then a fixed xor tree: the
// same order in every block and every run)
__device__ inline float wave_part_sum(const float* part, int nblk, int c) {
  const int l = threadIdx.x & 63;
  float t = 0.f;
  for (int k = l; k < nblk; k += 64) t += part[4 * k + c];
  for (int o = 32; o >= 1; o >>= 1) t += __shfl_xor(t, o);
  return t;
}

// mean and 1 / (std + 1e-8) from the per-block shifted sums (called by a whole wave)
// (norm == 0: SB3's normalize_advantage=False -- mean 0, scale 1)
__device__ inline void loss_stats(const float* ws, int B, int nblk, float a0, int norm, float& mean, float& inv) {
  const float* part = ws + 3 * (size_t)B;
  const float s1 = wave_part_sum(part, nblk, 0), s2 = wave_part_sum(part, nblk, 1);
  if (B > 1 && norm) {
    mean = a0 + s1 / (float)B;
    float var = (s2 - s1 * s1 / (float)B) / (float)(B - 1);
    inv = 1.f / (sqrtf(fmaxf(var, 0.f)) + 1e-8f);
  } else {
    mean = 0.f;
    inv = 1.f;
  }
}

__global__ __launch_bounds__(LOSS_TPB) void loss_terms_kernel(const float* __restrict__ logp,
                                                              const float* __restrict__ v, int B, float clip,
                                                              int norm, float* __restrict__ ws, int nblk) {
  __shared__ float red[LOSS_TPB / 64];
  __shared__ float st[2];
  const float* a_g = ws;
  const float* old_g = ws + B;
  const float* ret_g = ws + 2 * (size_t)B;
  float* part = ws + 3 * (size_t)B;
  if (threadIdx.x < 64) {
    float mu, iv;
    loss_stats(ws, B, nblk, a_g[0], norm, mu, iv);
    if (threadIdx.x == 0) { st[0] = mu; st[1] = iv; }
  }
  __syncthreads();
  const float mean = st[0], inv = st[1];
  const int i = blockIdx.x * LOSS_TPB + threadIdx.x;
  float pg = 0.f, vf = 0.f;
  if (i < B) {
    const float an = (a_g[i] - mean) * inv;
    const float r = expf(logp[i] - old_g[i]);
    const float rc = fminf(fmaxf(r, 1.f - clip), 1.f + clip);
    pg = fminf(an * r, an * rc);
    const float e = ret_g[i] - v[i];
    vf = e * e;
  }
  pg = block_sum256(pg, red);
  vf = block_sum256(vf, red);
  if (threadIdx.x == 0) {
    part[4 * blockIdx.x + 2] = pg;
    part[4 * blockIdx.x + 3] = vf;
    if (blockIdx.x == 0) {                    // stats for the backward
      float* stats = part + 4 * nblk;
      stats[0] = mean;
      stats[1] = inv;
    }
  }
}

__global__ void loss_final_kernel(const float* __restrict__ ws, int B, int nblk, float* __restrict__ pg_out,
                                  float* __restrict__ vf_out) {
  const float* part = ws + 3 * (size_t)B;
  const float pg = wave_part_sum(part, nblk, 2), vf = wave_part_sum(part, nblk, 3);
  if (threadIdx.x != 0) return;
  pg_out[0] = -pg / (float)B;
  vf_out[0] = vf / (float)B;
}

__global__ __launch_bounds__(256) void ppo_loss_bwd_kernel(const float* __restrict__ logp,
                                                           const float* __restrict__ v, int B, float clip,
                                                           const float* __restrict__ ws, int nblk,
                                                           const float* __restrict__ g_pg,
                                                           const float* __restrict__ g_vf,
                                                           float* __restrict__ g_logp, float* __restrict__ g_v) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= B) return;
  const float* a_g = ws;
  const float* old_g = ws + B;
  const float* ret_g = ws + 2 * (size_t)B;
  const float* stats = ws + 3 * (size_t)B + 4 * nblk;
  const float an = (a_g[i] - stats[0]) * stats[1];
  const float r = expf(logp[i] - old_g[i]);
  const float lo = 1.f - clip, hi = 1.f + clip;
  const float rc = fminf(fmaxf(r, lo), hi);
  const float s1 = an * r, s2 = an * rc;
  const float d1 = an, d2 = (r >= lo && r <= hi) ? an : 0.f;
  const float dmin = s1 < s2 ? d1 : (s1 > s2 ? d2 : 0.5f * (d1 + d2));
  g_logp[i] = g_pg[0] * (-1.f / (float)B) * dmin * r;
  g_v[i] = g_vf[0] * 2.f * (v[i] - ret_g[i]) / (float)B;
}

// clip_grad_norm_(max_norm) + Adam (torch.optim.Adam, capturable/fused formula) over up to
// ADAM_MAXT parameter tensors per chunk in three launches (torch: a multi-tensor norm, stack, norm, clamp,
// foreach mul and the fused Adam kernel):
//   adam_sqsum   per-block sums of g^2 over the concatenated gradients (fixed order)
//   adam_update  every block reduces those partials (same order) to the clip coefficient
//                min(1, max_norm / (||g|| + 1e-6)), then updates its chunk:
//                  m = b1 m + (1-b1) g c;  v = b2 v + (1-b2) (g c)^2
//                  p -= lr / (1 - b1^t) * m / (sqrt(v) / sqrt(1 - b2^t) + eps),  t = step + 1
//   adam_step    step[i] = t for every tensor (after all blocks have read the old step)
// All tensors take the same number of steps (one optimizer), so tensor 0's step is the clock.
constexpr int ADAM_MAXT = 16, ADAM_TPB = 256, ADAM_PER = 4;
constexpr int ADAM_MAXCHUNK = 64;   // launch_adam_clip handles up to ADAM_MAXT * ADAM_MAXCHUNK tensors

struct AdamArgs {
  float* p[ADAM_MAXT];
  const float* g[ADAM_MAXT];
  float* m[ADAM_MAXT];
  float* v[ADAM_MAXT];
  float* step[ADAM_MAXT];
  long long start[ADAM_MAXT + 1];   // prefix offsets of the tensors in the concatenation
  int nt;
};

__device__ inline int adam_tensor(const AdamArgs& a, long long e) {
  int t = 0;
  while (t + 1 < a.nt && e >= a.start[t + 1]) t++;
  return t;
}

__global__ __launch_bounds__(ADAM_TPB) void adam_sqsum_kernel(AdamArgs a, float* __restrict__ part) {
  __shared__ float red[ADAM_TPB / 64];
  float acc = 0.f;
  const long long base = (long long)blockIdx.x * ADAM_TPB * ADAM_PER;
  for (int k = 0; k < ADAM_PER; k++) {
    const long long e = base + (long long)k * ADAM_TPB + threadIdx.x;
    if (e < a.start[a.nt]) {
      const int t = adam_tensor(a, e);
      const float g = a.g[t][e - a.start[t]];
      acc += g * g;
    }
  }
  for (int o = 32; o >= 1; o >>= 1) acc += __shfl_xor(acc, o);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = acc;
  __syncthreads();
  if (threadIdx.x == 0) part[blockIdx.x] = (red[0] + red[1]) + (red[2] + red[3]);
}

__global__ __launch_bounds__(ADAM_TPB) void adam_update_kernel(AdamArgs a, const float* __restrict__ part, int nblk,
                                                               float max_norm, float lr, float b1, float b2,
                                                               float omb1, float omb2, float eps) {
  __shared__ float coef_s;
  if (threadIdx.x < 64) {
    float t = 0.f;
    for (int k = threadIdx.x; k < nblk; k += 64) t += part[k];
    for (int o = 32; o >= 1; o >>= 1) t += __shfl_xor(t, o);
    if (threadIdx.x == 0) coef_s = max_norm > 0.f ? fminf(1.f, max_norm / (sqrtf(t) + 1e-6f)) : 1.f;
  }
  __syncthreads();
  const float c = coef_s;
  const float step = a.step[0][0] + 1.f;
  const float bc1 = 1.f - powf(b1, step), bc2s = sqrtf(1.f - powf(b2, step));
  const float step_size = lr / bc1;
  const long long base = (long long)blockIdx.x * ADAM_TPB * ADAM_PER;
  for (int k = 0; k < ADAM_PER; k++) {
    const long long e = base + (long long)k * ADAM_TPB + threadIdx.x;
    if (e >= a.start[a.nt]) break;
    const int t = adam_tensor(a, e);
    const long long i = e - a.start[t];
    const float g = a.g[t][i] * c;
    const float m = b1 * a.m[t][i] + omb1 * g;        // omb = 1 - beta, rounded once from double
    const float v = b2 * a.v[t][i] + omb2 * g * g;
    a.m[t][i] = m;
    a.v[t][i] = v;
    a.p[t][i] -= step_size * m / (sqrtf(v) / bc2s + eps);
  }
}

__global__ void adam_step_kernel(AdamArgs a) {
  const float step = a.step[0][0] + 1.f;
  __syncthreads();
  if ((int)threadIdx.x < a.nt) a.step[threadIdx.x][0] = step;
}

// Column sums of a row-major [rows][cols] float32 matrix: out[c] = sum_r x[r][c].  The PPO
// update's bias gradients (sum of the output gradient over the minibatch, [32768][256]) and the
// split-K weight-gradient finish (sum over S slices of [S][out*in]).  A workgroup is a tile of
// 64 columns (a wave reads 256 contiguous bytes of a row per load) x 16 row phases (waves); each
// lane runs 4 independent accumulation chains over its rows, then the 16 phases are combined
// through LDS.  grid.y splits the rows into chunks whose partial rows a second launch
// (grid.y = 1) sums: fixed summation order, so results are run-to-run deterministic (no float
// atomics), and every lane's dependent-load chain stays short.
constexpr int CS_COLS = 64, CS_PHASES = 16, CS_PAIR_COLS1 = 16;

__global__ __launch_bounds__(CS_COLS* CS_PHASES) void colsum_kernel(const float* __restrict__ x, size_t rows,
                                                                     size_t cols, size_t rows_per_chunk,
                                                                     const float* __restrict__ rw,
                                                                     float* __restrict__ out) {
  __shared__ float part[CS_PHASES][CS_COLS];
  const int lane = threadIdx.x, ph = threadIdx.y;
  const size_t c = (size_t)blockIdx.x * CS_COLS + lane;
  const size_t r0 = (size_t)blockIdx.y * rows_per_chunk;
  const size_t r1 = r0 + rows_per_chunk < rows ? r0 + rows_per_chunk : rows;
  float a0 = 0.f, a1 = 0.f, a2 = 0.f, a3 = 0.f;
  if (c < cols) {
    const float* __restrict__ p = x + c;
    const size_t step = (size_t)CS_PHASES * cols;
    size_t r = r0 + ph;
    if (rw) {     // weighted rows: out[c] = sum_r rw[r] x[r][c] (a rank-1 weight gradient g' x)
      for (; r + 3 * CS_PHASES < r1; r += 4 * CS_PHASES) {
        const float* q = p + r * cols;
        a0 += rw[r] * q[0];
        a1 += rw[r + CS_PHASES] * q[step];
        a2 += rw[r + 2 * CS_PHASES] * q[2 * step];
        a3 += rw[r + 3 * CS_PHASES] * q[3 * step];
      }
      for (; r < r1; r += CS_PHASES) a0 += rw[r] * p[r * cols];
    } else {
      for (; r + 3 * CS_PHASES < r1; r += 4 * CS_PHASES) {
        const float* q = p + r * cols;
        a0 += q[0];
        a1 += q[step];
        a2 += q[2 * step];
        a3 += q[3 * step];
      }
      for (; r < r1; r += CS_PHASES) a0 += p[r * cols];
    }
  }
  part[ph][lane] = (a0 + a1) + (a2 + a3);
  __syncthreads();
  if (ph == 0 && c < cols) {
    float t = 0.f;
#pragma unroll
    for (int k = 0; k < CS_PHASES; k++) t += part[k][lane];
    out[(size_t)blockIdx.y * cols + c] = t;
  }
}

// ReLU backward fused with the bias gradient's first reduction pass: gm = (y > 0) ? g : 0 is
// written for the GEMMs that follow, and its per-chunk column sums go to `partial`
// ([gridDim.y][cols], the same tiling as colsum_kernel), finished by colsum_pair_kernel together
// with the split-K weight-gradient slices -- one pass over g instead of threshold_backward + a
// separate colsum read.
__global__ __launch_bounds__(CS_COLS* CS_PHASES) void relu_colsum_kernel(const float* __restrict__ g,
                                                                          const float* __restrict__ y,
                                                                          size_t rows, size_t cols,
                                                                          size_t rows_per_chunk,
                                                                          float* __restrict__ gm,
                                                                          float* __restrict__ partial) {
  __shared__ float part[CS_PHASES][CS_COLS];
  const int lane = threadIdx.x, ph = threadIdx.y;
  const size_t c = (size_t)blockIdx.x * CS_COLS + lane;
  const size_t r0 = (size_t)blockIdx.y * rows_per_chunk;
  const size_t r1 = r0 + rows_per_chunk < rows ? r0 + rows_per_chunk : rows;
  float a0 = 0.f, a1 = 0.f;
  if (c < cols) {
    size_t r = r0 + ph;
    for (; r + CS_PHASES < r1; r += 2 * CS_PHASES) {
      const size_t i0 = r * cols + c, i1 = (r + CS_PHASES) * cols + c;
      const float v0 = y[i0] > 0.f ? g[i0] : 0.f, v1 = y[i1] > 0.f ? g[i1] : 0.f;
      gm[i0] = v0;
      gm[i1] = v1;
      a0 += v0;
      a1 += v1;
    }
    for (; r < r1; r += CS_PHASES) {
      const size_t i = r * cols + c;
      const float v = y[i] > 0.f ? g[i] : 0.f;
      gm[i] = v;
      a0 += v;
    }
  }
  part[ph][lane] = a0 + a1;
  __syncthreads();
  if (ph == 0 && c < cols) {
    float t = 0.f;
#pragma unroll
    for (int k = 0; k < CS_PHASES; k++) t += part[k][lane];
    partial[(size_t)blockIdx.y * cols + c] = t;
  }
}

// Two single-pass column sums in one launch (blocks [0, tiles0) do x0, the rest x1): a layer's
// split-K weight-gradient finish (S rows, many columns: 64 columns x 16 row phases per block) and its
// bias-gradient finish (hundreds of partial rows of 256 columns: 16 columns x 64 row phases per
// block, so that 16 blocks share the rows instead of 4 walking them).  Four independent
// accumulators per thread keep four loads in flight.
__global__ __launch_bounds__(CS_COLS* CS_PHASES) void colsum_pair_kernel(const float* __restrict__ x0, size_t rows0,
                                                                          size_t cols0, float* __restrict__ out0,
                                                                          const float* __restrict__ x1, size_t rows1,
                                                                          size_t cols1, float* __restrict__ out1,
                                                                          unsigned tiles0) {
  __shared__ float part[CS_COLS * CS_PHASES];
  const bool second = blockIdx.x >= tiles0;
  const float* __restrict__ x = second ? x1 : x0;
  const size_t rows = second ? rows1 : rows0, cols = second ? cols1 : cols0;
  float* __restrict__ out = second ? out1 : out0;
  const int t = threadIdx.y * CS_COLS + threadIdx.x;
  const int w = second ? CS_PAIR_COLS1 : CS_COLS, nph = CS_COLS * CS_PHASES / w;   // columns, row phases per block
  const int lane = t % w, ph = t / w;
  const size_t c = (size_t)(second ? blockIdx.x - tiles0 : blockIdx.x) * w + lane;
  float a0 = 0.f, a1 = 0.f, a2 = 0.f, a3 = 0.f;
  if (c < cols) {
    size_t r = ph;
    for (; r + 3 * nph < rows; r += 4 * nph) {
      a0 += x[r * cols + c];
      a1 += x[(r + nph) * cols + c];
      a2 += x[(r + 2 * nph) * cols + c];
      a3 += x[(r + 3 * nph) * cols + c];
    }
    for (; r < rows; r += nph) a0 += x[r * cols + c];
  }
  part[ph * w + lane] = (a0 + a1) + (a2 + a3);
  __syncthreads();
  if (ph == 0 && c < cols) {
    float s = 0.f;
    for (int k = 0; k < nph; k++) s += part[k * w + lane];
    out[c] = s;
  }
}

// ------------------------------------------------------------------ fused 2-hidden-layer MLP forward
// out = relu(relu(X W1' + b1) W2' + b2) W3' + b3 for one policy net (PPO rollout: the pi net's mean per
// env step, the vf net's values once per rollout).  The weights come as nn.Linear stores them,
// [out][in] row-major (W1 [256][ld1], W2 [256][ld2], W3 [A][ld3]): the reduction index k is
// contiguous, so one 16-byte load fetches a lane's B operand for four v_mfma_f32_16x16x4_f32 steps.
// Within each group of 16 k the MFMA steps run over a permuted k (step j of lane group ak takes
// k = 16 q + 4 ak + j) so that A (from LDS) and B (from global) are both one b128 per lane per
// group -- the sum over k is the same, only its order differs from the GEMM's.
// One workgroup per 16 RB rows, 8 waves: wave w owns output columns [32 w, 32 w + 32) of a hidden
// layer for all the rows (RB row blocks x 2 column tiles of accumulators).  Its weight rows are read
// by no other wave, so they stream straight into VGPRs (the MI355X guide's GEMV rule: no LDS round
// trip), MLP_PF groups ahead of the MFMAs in a register ring, and each 16-byte weight load feeds RB
// row blocks; the input tile and the hidden activations live in LDS (dynamic: sized to D).
// RB = 1 for the per-step pi forward (4096 rows: 256 workgroups, every CU busy), RB = 2 for the
// rollout-buffer vf pass (half the weight traffic per row).
// Replaces three library GEMM launches and their two [N][256] HBM round trips.
constexpr int MLP_H = 256, MLP_WAVES = 8, MLP_TPB = 64 * MLP_WAVES, MLP_MAXD = 512, MLP_PF = 4;
// above this many rows two row blocks per wave (A/B with each forced, tools/probes/gpu_mlp2_fwd.py,
// profiles/r5i: 4096 rows 23.5 vs 26.6 us, 8192 rows 40.2 vs 26.4 us)
constexpr int MLP_RB2_ROWS = 6144;
constexpr int MLP_SH = MLP_H + 4;   // LDS row stride (floats) of the hidden tiles: 16-byte aligned rows
typedef float f32x4 __attribute__((ext_vector_type(4)));

template <bool VEC>
__device__ __forceinline__ f32x4 mlp_ld4(const float* __restrict__ p) {
  if constexpr (VEC) return *reinterpret_cast<const f32x4*>(p);
  else return f32x4{p[0], p[1], p[2], p[3]};
}

// acc[rb][t] += A_rb[16 x 16] . B_t[16 x 16] for k-group g: a = LDS base of this lane's A row in
// row block 0 (+ 4 ak), sa = the row-block stride (16 rows) in floats
template <int RB>
__device__ __forceinline__ void mlp_group(const float* a, int sa, int g, const f32x4& b0, const f32x4& b1,
                                          f32x4 (&acc)[RB][2]) {
  f32x4 x[RB];
#pragma unroll
  for (int rb = 0; rb < RB; rb++) x[rb] = *reinterpret_cast<const f32x4*>(a + rb * sa + 16 * g);
#pragma unroll
  for (int s = 0; s < 4; s++)
#pragma unroll
    for (int rb = 0; rb < RB; rb++) {
      acc[rb][0] = __builtin_amdgcn_mfma_f32_16x16x4f32(x[rb][s], b0[s], acc[rb][0], 0, 0, 0);
      acc[rb][1] = __builtin_amdgcn_mfma_f32_16x16x4f32(x[rb][s], b1[s], acc[rb][1], 0, 0, 0);
    }
}
// the full k-groups [0, G) of one wave's two column tiles; w0 / w1 = this lane's weight rows (+ 4 ak).
// Every ring refill is unconditional (the group index clamped to G - 1: the last refills re-read
// it) and follows the MFMAs that consumed the slot, so the compiler's wait before a slot's use
// counts only the loads issued after it and the ring needs no register copies.
template <bool VEC, int RB>
__device__ __forceinline__ void mlp_groups(const float* a, int sa, const float* __restrict__ w0,
                                           const float* __restrict__ w1, int G, f32x4 (&acc)[RB][2]) {
  if (G <= 0) return;
  f32x4 bq[MLP_PF][2];
#pragma unroll
  for (int j = 0; j < MLP_PF; j++) {
    const int g = j < G - 1 ? j : G - 1;
    bq[j][0] = mlp_ld4<VEC>(w0 + 16 * g);
    bq[j][1] = mlp_ld4<VEC>(w1 + 16 * g);
  }
  const int Gm = G - G % MLP_PF;
  for (int g0 = 0; g0 < Gm; g0 += MLP_PF) {
#pragma unroll
    for (int j = 0; j < MLP_PF; j++) {
      const int g = g0 + j;
      mlp_group<RB>(a, sa, g, bq[j][0], bq[j][1], acc);
      const int gn = g + MLP_PF < G - 1 ? g + MLP_PF : G - 1;
      bq[j][0] = mlp_ld4<VEC>(w0 + 16 * gn);
      bq[j][1] = mlp_ld4<VEC>(w1 + 16 * gn);
      __builtin_amdgcn_sched_barrier(0);   // keep each refill in its group (the scheduler would batch them)
    }
  }
#pragma unroll
  for (int j = 0; j < MLP_PF - 1; j++)   // the last G % MLP_PF groups, already in slots 0..
    if (Gm + j < G) mlp_group<RB>(a, sa, Gm + j, bq[j][0], bq[j][1], acc);
}

// dynamic LDS of one workgroup: the input tile (row stride roundup16(D) + 4), later layer 2's output
// (stride MLP_SH), then layer 1's output
__host__ __device__ constexpr int mlp_xs_stride(int D) { return ((D + 15) & ~15) + 4 > MLP_SH ? ((D + 15) & ~15) + 4 : MLP_SH; }
__host__ __device__ constexpr size_t mlp_lds_bytes(int RB, int D) { return (size_t)16 * RB * (mlp_xs_stride(D) + MLP_SH) * 4; }

template <bool VEC, int RB>
__global__ __launch_bounds__(MLP_TPB) void mlp2_fwd_kernel(const float* __restrict__ X, int ldx, int D, int N,
                                                           const float* __restrict__ W1, int ld1,
                                                           const float* __restrict__ b1,
                                                           const float* __restrict__ W2, int ld2,
                                                           const float* __restrict__ b2,
                                                           const float* __restrict__ W3, int ld3,
                                                           const float* __restrict__ b3, int A,
                                                           float* __restrict__ out, int ldo) {
  constexpr int R = 16 * RB;
  extern __shared__ __attribute__((aligned(16))) float mlp_lds[];
  const int sx = mlp_xs_stride(D);
  float* xs = mlp_lds;                 // X tile, then layer 2's output
  float* hs = mlp_lds + R * sx;        // layer 1's output, then the head's partial sums
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int ar = lane & 15, ak = lane >> 4;   // A: row ar, k 4 ak..; B: column ar, k 4 ak..; C: rows 4 ak.., column ar
  const int row0 = blockIdx.x * R;
  const int Gf = D >> 4, Dp = (D + 15) & ~15;
  if ((D & 3) == 0 && (ldx & 3) == 0 && ((uintptr_t)X & 15) == 0) {   // 16-byte staging: 32 threads per row
    for (int r = threadIdx.x >> 5; r < R; r += MLP_TPB / 32) {
      const bool live = row0 + r < N;
      const float* xr = X + (size_t)(live ? row0 + r : 0) * ldx;
      for (int c = 4 * (threadIdx.x & 31); c < Dp; c += 128) {
        const f32x4 v = (live && c < D) ? *reinterpret_cast<const f32x4*>(xr + c) : f32x4{0, 0, 0, 0};
        *reinterpret_cast<f32x4*>(xs + r * sx + c) = v;
      }
    }
  } else {
    for (int e = threadIdx.x; e < R * Dp; e += MLP_TPB) {
      const int r = e / Dp, c = e - r * Dp;
      xs[r * sx + c] = (row0 + r < N && c < D) ? X[(size_t)(row0 + r) * ldx + c] : 0.f;
    }
  }
  __syncthreads();
  const int c0 = wave * 32 + ar;   // this lane's column of tile 0 (tile 1: + 16)
  auto epilogue = [&](const f32x4 (&acc)[RB][2], const float* __restrict__ bias, float* dst) {
#pragma unroll
    for (int t = 0; t < 2; t++) {
      const float bb = bias[c0 + 16 * t];
#pragma unroll
      for (int rb = 0; rb < RB; rb++)
#pragma unroll
        for (int r = 0; r < 4; r++)
          dst[(16 * rb + 4 * ak + r) * MLP_SH + c0 + 16 * t] = fmaxf(acc[rb][t][r] + bb, 0.f);
    }
  };
  {   // layer 1: K = D (full groups pipelined, a partial last group with masked loads)
    f32x4 acc[RB][2] = {};
    const float* w0 = W1 + (size_t)c0 * ld1 + 4 * ak;
    const float* w1 = w0 + (size_t)16 * ld1;
    const float* a = xs + ar * sx + 4 * ak;
    mlp_groups<VEC, RB>(a, 16 * sx, w0, w1, Gf, acc);
    if (D & 15) {
      const int kb = 16 * Gf + 4 * ak;
      f32x4 b0, b1v;
#pragma unroll
      for (int i = 0; i < 4; i++) {
        b0[i] = kb + i < D ? w0[16 * Gf + i] : 0.f;
        b1v[i] = kb + i < D ? w1[16 * Gf + i] : 0.f;
      }
      mlp_group<RB>(a, 16 * sx, Gf, b0, b1v, acc);
    }
    epilogue(acc, b1, hs);
  }
  __syncthreads();
  {   // layer 2: K = 256, into xs (the X tile is dead)
    f32x4 acc[RB][2] = {};
    const float* w0 = W2 + (size_t)c0 * ld2 + 4 * ak;
    mlp_groups<VEC, RB>(hs + ar * MLP_SH + 4 * ak, 16 * MLP_SH, w0, w0 + (size_t)16 * ld2, MLP_H / 16, acc);
    epilogue(acc, b2, xs);
  }
  __syncthreads();
  // head: A <= 32 columns = 2 tiles x 4 quarters of k over the 8 waves (every wave's 4 weight loads in
  // flight at once), the quarters' partial sums added through LDS (hs is free after layer 2); a lane
  // whose column is >= A reads row A - 1 and multiplies zeros
  {
    const int t = wave & 1, kq = wave >> 1, col = 16 * t + ar;
    if (16 * t < A) {
      const float* w = W3 + (size_t)(col < A ? col : A - 1) * ld3 + 4 * ak + 64 * kq;
      const float keep = col < A ? 1.f : 0.f;
      const float* a = xs + ar * MLP_SH + 4 * ak + 64 * kq;
      f32x4 bw[4];
#pragma unroll
      for (int g = 0; g < 4; g++) bw[g] = mlp_ld4<VEC>(w + 16 * g) * keep;
      f32x4 acc[RB] = {};
#pragma unroll
      for (int g = 0; g < 4; g++)
#pragma unroll
        for (int rb = 0; rb < RB; rb++) {
          const f32x4 x = *reinterpret_cast<const f32x4*>(a + 16 * rb * MLP_SH + 16 * g);
#pragma unroll
          for (int s = 0; s < 4; s++) acc[rb] = __builtin_amdgcn_mfma_f32_16x16x4f32(x[s], bw[g][s], acc[rb], 0, 0, 0);
        }
#pragma unroll
      for (int rb = 0; rb < RB; rb++)
#pragma unroll
        for (int r = 0; r < 4; r++) hs[(kq * R + 16 * rb + 4 * ak + r) * 32 + col] = acc[rb][r];
    }
  }
  __syncthreads();
  for (int e = threadIdx.x; e < R * A; e += MLP_TPB) {
    const int r = e / A, c = e - r * A;
    if (row0 + r < N)
      out[(size_t)(row0 + r) * ldo + c] = b3[c] + ((hs[r * 32 + c] + hs[(R + r) * 32 + c]) +
                                                   (hs[(2 * R + r) * 32 + c] + hs[(3 * R + r) * 32 + c]));
  }
}

// ------------------------------------------------------------------ input gradient + ReLU mask
// The backward of a Linear layer whose input x is the previous layer's ReLU output:
//   GX = (G W) ⊙ (X > 0),  partial[wg][n] = sum of GX over the workgroup's rows
// G [B][K] (ldg) is the layer's output gradient, W [K][N] its nn.Linear weight ([out][in]), X [B][N]
// (ldx) its input.  The mask is the previous layer's ReLU backward and the partial sums its bias
// gradient's first pass, so that layer needs no separate pass over [B][N] (autograd writes G W,
// then threshold_backward reads it with X and writes it again, then the bias sum reads it).
// N = 256 (the hidden width).
// K % 16 == 0 (hidden layers, K = 256): the MFMA tiles of mlp2_fwd_kernel on Wt = W' ([N][K], k
// contiguous: dg_transpose_kernel, once per call) so that a lane's B operand of a k-group is one
// 16-byte load; the accumulators go through LDS so that the mask read of X, the GX store and the
// column sums run on whole rows (16-byte accesses) instead of the MFMA's 64-byte column slivers.
// K <= 32 (the heads: 21 actions, 1 value): VALU, the G tile in LDS, a float4 of columns per thread.
constexpr int DG_N = 256, DG_RB4_ROWS = 16384;

// Wt[n][k] = W[k][n] (W [K][ldw], Wt [N][K]): 32 x 32 tiles through LDS
__global__ __launch_bounds__(256) void dg_transpose_kernel(const float* __restrict__ W, int ldw, int K, int N,
                                                           float* __restrict__ Wt) {
  __shared__ float t[32][33];
  const int k0 = blockIdx.y * 32, n0 = blockIdx.x * 32, tx = threadIdx.x & 31, ty = threadIdx.x >> 5;
  for (int r = ty; r < 32; r += 8)
    if (k0 + r < K && n0 + tx < N) t[r][tx] = W[(size_t)(k0 + r) * ldw + n0 + tx];
  __syncthreads();
  for (int r = ty; r < 32; r += 8)
    if (n0 + r < N && k0 + tx < K) Wt[(size_t)(n0 + r) * K + k0 + tx] = t[tx][r];
}

// mask, store and column-sum an [R][DG_N] gradient tile held in LDS (row stride st): thread t owns
// columns 4 (t % 64) .. + 3 of rows t / 64 + TPB / 64 i; the per-thread sums reduce through `red`
// ([TPB / 64][64] float4, may alias the tile after the barrier)
template <int R, int TPB, bool XVEC>
__device__ __forceinline__ void dg_finish(const float* tile, int st, const float* __restrict__ X, int ldx, int B,
                                          int row0, float* __restrict__ GX, float* __restrict__ part, f32x4* red) {
  constexpr int P = TPB / 64;
  const int c4 = threadIdx.x & 63, rp = threadIdx.x >> 6;
  f32x4 xv[R / P], gv[R / P];
#pragma unroll
  for (int i = 0; i < R / P; i++) {   // every X load of the thread in flight at once
    const int row = row0 + rp + P * i;
    const float* xr = X + (size_t)(row < B ? row : 0) * ldx + 4 * c4;
    xv[i] = mlp_ld4<XVEC>(xr);
    gv[i] = *reinterpret_cast<const f32x4*>(tile + (rp + P * i) * st + 4 * c4);
  }
  f32x4 cs = {0, 0, 0, 0};
#pragma unroll
  for (int i = 0; i < R / P; i++) {
    const int row = row0 + rp + P * i;
    f32x4 v;
#pragma unroll
    for (int q = 0; q < 4; q++) v[q] = xv[i][q] > 0.f ? gv[i][q] : 0.f;
    if (row < B) {
      *reinterpret_cast<f32x4*>(GX + (size_t)row * DG_N + 4 * c4) = v;
      cs += v;
    }
  }
  __syncthreads();   // the tile is read: red may alias it
  red[rp * 64 + c4] = cs;
  __syncthreads();
  if (rp == 0) {
    f32x4 tsum = red[c4];
#pragma unroll
    for (int p = 1; p < P; p++) tsum += red[p * 64 + c4];
    *reinterpret_cast<f32x4*>(part + (size_t)blockIdx.x * DG_N + 4 * c4) = tsum;
  }
}

__host__ __device__ constexpr int dg_stride(int K) { return (K > DG_N ? K : DG_N) + 4; }

template <int RB, bool XVEC>
__global__ __launch_bounds__(MLP_TPB) void dgrad_mask_mfma_kernel(const float* __restrict__ G, int ldg, int K,
                                                                  const float* __restrict__ Wt,
                                                                  const float* __restrict__ X, int ldx, int B,
                                                                  float* __restrict__ GX, float* __restrict__ part) {
  constexpr int R = 16 * RB;
  extern __shared__ __attribute__((aligned(16))) float dg_lds[];
  const int sg = dg_stride(K);                // G tile, then the output tile: 16-byte aligned rows
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int ar = lane & 15, ak = lane >> 4;
  const int row0 = blockIdx.x * R;
  for (int r = threadIdx.x >> 5; r < R; r += MLP_TPB / 32) {   // 32 threads per row, 16-byte loads
    const bool live = row0 + r < B;
    const float* gr = G + (size_t)(live ? row0 + r : 0) * ldg;
    for (int c = 4 * (threadIdx.x & 31); c < K; c += 128)
      *reinterpret_cast<f32x4*>(dg_lds + r * sg + c) = live ? *reinterpret_cast<const f32x4*>(gr + c)
                                                            : f32x4{0, 0, 0, 0};
  }
  __syncthreads();
  const int c0 = wave * 32 + ar;
  f32x4 acc[RB][2] = {};
  const float* w0 = Wt + (size_t)c0 * K + 4 * ak;
  mlp_groups<true, RB>(dg_lds + ar * sg + 4 * ak, 16 * sg, w0, w0 + (size_t)16 * K, K >> 4, acc);
  __syncthreads();   // every wave is done with the G tile
#pragma unroll
  for (int t = 0; t < 2; t++)
#pragma unroll
    for (int rb = 0; rb < RB; rb++)
#pragma unroll
      for (int r = 0; r < 4; r++) dg_lds[(16 * rb + 4 * ak + r) * sg + c0 + 16 * t] = acc[rb][t][r];
  __syncthreads();
  dg_finish<R, MLP_TPB, XVEC>(dg_lds, sg, X, ldx, B, row0, GX, part, reinterpret_cast<f32x4*>(dg_lds));
}

// K <= 32: 32 rows per workgroup; the G tile in LDS (each wave's row of it read as a broadcast),
// W[k][4 c4 .. + 3] one load per k, k outer over the thread's 8 rows
constexpr int DG_SMALL_K = 32, DG_SMALL_R = 32, DG_SMALL_TPB = 256;
template <bool XVEC>
__global__ __launch_bounds__(DG_SMALL_TPB) void dgrad_mask_small_kernel(const float* __restrict__ G, int ldg, int K,
                                                                        const float* __restrict__ W, int ldw,
                                                                        const float* __restrict__ X, int ldx, int B,
                                                                        float* __restrict__ GX,
                                                                        float* __restrict__ part) {
  __shared__ __attribute__((aligned(16))) float gs[DG_SMALL_R][DG_SMALL_K + 1];
  __shared__ __attribute__((aligned(16))) f32x4 tile[DG_SMALL_R * 64];   // [R][256] floats, row stride 256
  const int c4 = threadIdx.x & 63, rp = threadIdx.x >> 6;
  const int row0 = blockIdx.x * DG_SMALL_R;
  for (int e = threadIdx.x; e < DG_SMALL_R * K; e += DG_SMALL_TPB) {
    const int r = e / K, k = e - r * K;
    gs[r][k] = row0 + r < B ? G[(size_t)(row0 + r) * ldg + k] : 0.f;
  }
  __syncthreads();
  constexpr int P = DG_SMALL_TPB / 64, RR = DG_SMALL_R / P;
  f32x4 v[RR] = {};
  for (int k = 0; k < K; k++) {
    const f32x4 w = mlp_ld4<XVEC>(W + (size_t)k * ldw + 4 * c4);
#pragma unroll
    for (int i = 0; i < RR; i++) v[i] += gs[rp + P * i][k] * w;
  }
#pragma unroll
  for (int i = 0; i < RR; i++) tile[(rp + P * i) * 64 + c4] = v[i];
  __syncthreads();
  dg_finish<DG_SMALL_R, DG_SMALL_TPB, XVEC>(reinterpret_cast<const float*>(tile), DG_N, X, ldx, B, row0, GX, part,
                                            tile);
}

}  // namespace

// row chunks for colsum: enough workgroups to fill the chip (~1024) with >= 32 rows each;
// one chunk (a single launch) when the column tiles alone give that parallelism
static size_t colsum_chunks(size_t rows, size_t cols) {
  const size_t ctiles = (cols + CS_COLS - 1) / CS_COLS;
  if (ctiles >= 512 || rows <= 4 * CS_PHASES) return 1;
  size_t chunks = 512 / ctiles;                 // ~512 workgroups of 16 waves
  const size_t maxc = rows / (4 * CS_PHASES);   // >= 4 rows per lane
  if (chunks > maxc) chunks = maxc;
  return chunks < 1 ? 1 : chunks;
}

hipError_t launch_ppo_act(const float* mean, int mean_ld, const float* value, int value_ld, const float* log_std,
                          const float* episode_start, uint64_t seed, uint64_t counter, const uint64_t* counter_base,
                          int deterministic, float* act,
                          float* act_clip, float* logp, float* val, float* start_out, int N, int A,
                          hipStream_t stream) {
  if (N <= 0) return hipSuccess;
  const size_t threads = (size_t)N * 32;
  const int block = 256;
  const dim3 grid((unsigned)((threads + block - 1) / block));
  hipLaunchKernelGGL(ppo_act_kernel, grid, dim3(block), 0, stream, mean, mean_ld, value, value_ld, log_std,
                     episode_start, (uint32_t)seed, (uint32_t)(seed >> 32), counter, counter_base, deterministic, act,
                     act_clip, logp, val, start_out, N, A);
  return hipGetLastError();
}

hipError_t launch_ppo_post(const float* reward, const uint8_t* terminated, const uint8_t* truncated,
                           const float* terminal_value, const float* terminal_obs, float* boot_obs_out,
                           uint8_t* boot_out, int obs_dim, float gamma, const float* obs, float* obs_out,
                           size_t obs_floats, float* reward_out, uint8_t* done_out, double* ep_acc,
                           double* ep_return_out, float* episode_start, int N, hipStream_t stream) {
  if (N <= 0) return hipSuccess;
  const int vec4 = obs_floats % 4 == 0 && ((uintptr_t)obs | (uintptr_t)obs_out) % 16 == 0;
  const size_t obs_n = vec4 ? obs_floats / 4 : obs_floats;
  const size_t work = obs_n > (size_t)N ? obs_n : (size_t)N;
  const int block = 256;
  // one 16 B vector per lane per pass, at most 8 passes' worth of workgroups resident
  size_t blocks = (work + block - 1) / block;
  if (blocks > 2048) blocks = 2048;
  if (blocks * block < (size_t)N) blocks = ((size_t)N + block - 1) / block;
  hipLaunchKernelGGL(ppo_post_kernel, dim3((unsigned)blocks), dim3(block), 0, stream, reward, terminated, truncated,
                     terminal_value, terminal_obs, boot_obs_out, boot_out, gamma, obs, obs_out, obs_n, vec4,
                     reward_out, done_out, ep_acc, ep_return_out, episode_start, N, obs_dim);
  return hipGetLastError();
}

size_t colsum_workspace(size_t rows, size_t cols) {
  const size_t chunks = colsum_chunks(rows, cols);
  return chunks > 1 ? chunks * cols : 0;
}

hipError_t launch_colsum(const float* x, size_t rows, size_t cols, const float* row_weight, float* workspace,
                         float* out, hipStream_t stream) {
  if (cols == 0) return hipSuccess;
  const dim3 block(CS_COLS, CS_PHASES);
  const unsigned ctiles = (unsigned)((cols + CS_COLS - 1) / CS_COLS);
  const size_t chunks = colsum_chunks(rows, cols);
  if (rows == 0) return hipMemsetAsync(out, 0, cols * sizeof(float), stream);
  if (chunks <= 1) {
    hipLaunchKernelGGL(colsum_kernel, dim3(ctiles, 1), block, 0, stream, x, rows, cols, rows, row_weight, out);
    return hipGetLastError();
  }
  const size_t rpc = (rows + chunks - 1) / chunks;
  hipLaunchKernelGGL(colsum_kernel, dim3(ctiles, (unsigned)chunks), block, 0, stream, x, rows, cols, rpc,
                     row_weight, workspace);
  hipLaunchKernelGGL(colsum_kernel, dim3(ctiles, 1), block, 0, stream, (const float*)workspace, chunks, cols,
                     chunks, (const float*)nullptr, out);
  return hipGetLastError();
}

hipError_t launch_gauss_logp(const float* mean, int mean_ld, const float* act, const float* log_std, float* logp, int N,
                             int A, hipStream_t stream) {
  if (N <= 0) return hipSuccess;
  const size_t threads = (size_t)N * 32;
  hipLaunchKernelGGL(gauss_logp_kernel, dim3((unsigned)((threads + 255) / 256)), dim3(256), 0, stream, mean, mean_ld,
                     act, log_std, logp, N, A);
  return hipGetLastError();
}

hipError_t launch_gauss_logp_grad(const float* mean, int mean_ld, const float* act, const float* log_std,
                                  const float* g_logp, float* g_mean, float* gls_rows, int N, int A,
                                  hipStream_t stream) {
  if (N <= 0) return hipSuccess;
  const size_t el = (size_t)N * A;
  hipLaunchKernelGGL(gauss_logp_grad_kernel, dim3((unsigned)((el + 255) / 256)), dim3(256), 0, stream, mean, mean_ld,
                     act, log_std, g_logp, g_mean, gls_rows, N, A);
  return hipGetLastError();
}

size_t ppo_loss_workspace(int B) {
  const size_t nblk = B > 0 ? ((size_t)B + LOSS_TPB - 1) / LOSS_TPB : 0;
  return 3 * (size_t)B + 4 * nblk + 2;
}

hipError_t launch_ppo_loss_fwd(const float* logp, const float* v, const int64_t* idx, const float* adv,
                               const float* ret, const float* old_logp, int B, float clip, int normalize, float* pg,
                               float* vf, float* ws, hipStream_t stream) {
  if (B <= 0) return hipSuccess;
  const int nblk = (B + LOSS_TPB - 1) / LOSS_TPB;
  hipLaunchKernelGGL(loss_gather_kernel, dim3(nblk), dim3(LOSS_TPB), 0, stream, idx, adv, ret, old_logp, B, ws);
  hipLaunchKernelGGL(loss_terms_kernel, dim3(nblk), dim3(LOSS_TPB), 0, stream, logp, v, B, clip, normalize, ws,
                     nblk);
  hipLaunchKernelGGL(loss_final_kernel, dim3(1), dim3(64), 0, stream, (const float*)ws, B, nblk, pg, vf);
  return hipGetLastError();
}

hipError_t launch_ppo_loss_bwd(const float* logp, const float* v, int B, float clip, const float* ws,
                               const float* g_pg, const float* g_vf, float* g_logp, float* g_v, hipStream_t stream) {
  if (B <= 0) return hipSuccess;
  const int nblk = (B + LOSS_TPB - 1) / LOSS_TPB;
  hipLaunchKernelGGL(ppo_loss_bwd_kernel, dim3(nblk), dim3(256), 0, stream, logp, v, B, clip, ws, nblk, g_pg, g_vf,
                     g_logp, g_v);
  return hipGetLastError();
}

// partial sums of the squared-gradient pass: one per ADAM_TPB * ADAM_PER elements of each chunk of
// ADAM_MAXT tensors (the per-chunk rounding adds at most one partial per chunk)
int adam_partials(long long total) {
  return (int)((total + (long long)ADAM_TPB * ADAM_PER - 1) / ((long long)ADAM_TPB * ADAM_PER)) + ADAM_MAXCHUNK;
}

// Any number of tensors (<= ADAM_MAXT * ADAM_MAXCHUNK): chunks of ADAM_MAXT share one partials
// array, so every update block reduces the partials of ALL chunks to the same clip coefficient;
// the step counters advance after every chunk's update has read them.
hipError_t launch_adam_clip(int nt, float* const* p, const float* const* g, float* const* m, float* const* v,
                            float* const* step, const long long* numel, float* part, float max_norm, double lr,
                            double b1, double b2, double eps, hipStream_t stream) {
  if (nt <= 0 || nt > ADAM_MAXT * ADAM_MAXCHUNK) return hipErrorInvalidValue;
  const int nchunk = (nt + ADAM_MAXT - 1) / ADAM_MAXT;
  AdamArgs a[ADAM_MAXCHUNK];
  int nblk[ADAM_MAXCHUNK], off[ADAM_MAXCHUNK + 1];
  off[0] = 0;
  for (int c = 0; c < nchunk; c++) {
    a[c] = AdamArgs{};
    a[c].nt = std::min(ADAM_MAXT, nt - c * ADAM_MAXT);
    a[c].start[0] = 0;
    for (int j = 0; j < a[c].nt; j++) {
      const int t = c * ADAM_MAXT + j;
      a[c].p[j] = p[t];
      a[c].g[j] = g[t];
      a[c].m[j] = m[t];
      a[c].v[j] = v[t];
      a[c].step[j] = step[t];
      a[c].start[j + 1] = a[c].start[j] + numel[t];
    }
    nblk[c] = (int)((a[c].start[a[c].nt] + (long long)ADAM_TPB * ADAM_PER - 1) / ((long long)ADAM_TPB * ADAM_PER));
    off[c + 1] = off[c] + nblk[c];
  }
  if (off[nchunk] <= 0) return hipSuccess;
  for (int c = 0; c < nchunk; c++)
    if (nblk[c]) hipLaunchKernelGGL(adam_sqsum_kernel, dim3(nblk[c]), dim3(ADAM_TPB), 0, stream, a[c], part + off[c]);
  for (int c = 0; c < nchunk; c++)
    if (nblk[c])
      hipLaunchKernelGGL(adam_update_kernel, dim3(nblk[c]), dim3(ADAM_TPB), 0, stream, a[c], (const float*)part,
                         off[nchunk], max_norm, (float)lr, (float)b1, (float)b2, (float)(1.0 - b1), (float)(1.0 - b2),
                         (float)eps);
  for (int c = 0; c < nchunk; c++) hipLaunchKernelGGL(adam_step_kernel, dim3(1), dim3(64), 0, stream, a[c]);
  return hipGetLastError();
}

size_t colsum_partial_rows(size_t rows, size_t cols) { return colsum_chunks(rows, cols); }

hipError_t launch_relu_colsum(const float* g, const float* y, size_t rows, size_t cols, float* gm, float* partial,
                              hipStream_t stream) {
  if (cols == 0 || rows == 0) return hipSuccess;
  const size_t chunks = colsum_chunks(rows, cols);
  const size_t rpc = (rows + chunks - 1) / chunks;
  const unsigned ctiles = (unsigned)((cols + CS_COLS - 1) / CS_COLS);
  hipLaunchKernelGGL(relu_colsum_kernel, dim3(ctiles, (unsigned)chunks), dim3(CS_COLS, CS_PHASES), 0, stream, g, y,
                     rows, cols, rpc, gm, partial);
  return hipGetLastError();
}

hipError_t launch_colsum_pair(const float* x0, size_t rows0, size_t cols0, float* out0, const float* x1, size_t rows1,
                              size_t cols1, float* out1, hipStream_t stream) {
  const unsigned t0 = (unsigned)((cols0 + CS_COLS - 1) / CS_COLS),
                 t1 = (unsigned)((cols1 + CS_PAIR_COLS1 - 1) / CS_PAIR_COLS1);
  if (t0 + t1 == 0) return hipSuccess;
  hipLaunchKernelGGL(colsum_pair_kernel, dim3(t0 + t1), dim3(CS_COLS, CS_PHASES), 0, stream, x0, rows0, cols0, out0, x1,
                     rows1, cols1, out1, t0);
  return hipGetLastError();
}


hipError_t launch_mlp2_fwd(const float* X, int ldx, int D, int N, const float* W1, int ld1, const float* b1,
                           const float* W2, int ld2, const float* b2, const float* W3, int ld3, const float* b3, int A,
                           float* out, int ldo, hipStream_t stream) {
  if (D < 1 || D > MLP_MAXD || A < 1 || A > 32 || N < 0 || ld1 < D || ld2 < MLP_H || ld3 < MLP_H || ldx < D || ldo < A)
    return hipErrorInvalidValue;
  if (N == 0) return hipSuccess;
  // 16-byte weight loads when every weight row starts 16-byte aligned; two row blocks per wave for
  // large row counts (half the weight traffic; one-block workgroups keep every CU busy below)
  auto al = [](const float* p, int ld) { return ((uintptr_t)p & 15) == 0 && (ld & 3) == 0; };
  const bool vec = al(W1, ld1) && al(W2, ld2) && al(W3, ld3);
  const int RB = N > MLP_RB2_ROWS ? 2 : 1;
  const dim3 grid((N + 16 * RB - 1) / (16 * RB));
  const size_t lds = mlp_lds_bytes(RB, D);
  // dynamic LDS above 64 KiB needs the per-kernel opt-in (once per instance)
#define MLP_LAUNCH(V, B)                                                                                     \
  do {                                                                                                      \
    static const hipError_t attr = hipFuncSetAttribute(reinterpret_cast<const void*>(&mlp2_fwd_kernel<V, B>), \
                                                       hipFuncAttributeMaxDynamicSharedMemorySize,          \
                                                       (int)mlp_lds_bytes(B, MLP_MAXD));                    \
    if (attr != hipSuccess) return attr;                                                                    \
    mlp2_fwd_kernel<V, B><<<grid, MLP_TPB, lds, stream>>>(X, ldx, D, N, W1, ld1, b1, W2, ld2, b2, W3, ld3, b3, \
                                                          A, out, ldo);                                     \
  } while (0)
  if (vec) { if (RB == 2) MLP_LAUNCH(true, 2); else MLP_LAUNCH(true, 1); }
  else { if (RB == 2) MLP_LAUNCH(false, 2); else MLP_LAUNCH(false, 1); }
#undef MLP_LAUNCH
  return hipGetLastError();
}

// row blocks per workgroup of the MFMA instance: 16 rows below MLP_RB2_ROWS, 32 to DG_RB4_ROWS,
// 64 above (each workgroup streams all of Wt: more rows per workgroup, less L2 traffic per row).
// HSIM_DG_RB=1|2|4 forces one (A/B probes).
static int dg_rb(int B) {
  static const int forced = [] {
    const char* e = getenv("HSIM_DG_RB");
    const int v = e ? atoi(e) : 0;
    return v == 1 || v == 2 || v == 4 ? v : 0;
  }();
  if (forced) return forced;
  return B > DG_RB4_ROWS ? 4 : B > MLP_RB2_ROWS ? 2 : 1;
}

size_t dgrad_mask_partial_rows(int B, int K) {
  if (B <= 0) return 0;
  const int R = K <= DG_SMALL_K ? DG_SMALL_R : 16 * dg_rb(B);
  return (size_t)((B + R - 1) / R);
}

size_t dgrad_mask_workspace(int K) { return K <= DG_SMALL_K ? 0 : (size_t)DG_N * K; }

hipError_t launch_dgrad_mask(const float* G, int ldg, int K, const float* W, int ldw, const float* X, int ldx, int B,
                             int N, float* GX, float* partial, float* workspace, hipStream_t stream) {
  if (B < 0 || N != DG_N || K < 1 || (K > DG_SMALL_K && (K % 16 != 0 || K > MLP_MAXD)) || ldg < K || ldw < N ||
      ldx < N)
    return hipErrorInvalidValue;
  if (B == 0) return hipSuccess;
  const bool xvec = ((uintptr_t)X & 15) == 0 && (ldx & 3) == 0;
  if (K <= DG_SMALL_K) {
    const bool vec = xvec && ((uintptr_t)W & 15) == 0 && (ldw & 3) == 0;   // X and W rows 16-byte aligned
    if (vec)
      hipLaunchKernelGGL(dgrad_mask_small_kernel<true>, dim3((B + DG_SMALL_R - 1) / DG_SMALL_R), dim3(DG_SMALL_TPB), 0,
                         stream, G, ldg, K, W, ldw, X, ldx, B, GX, partial);
    else
      hipLaunchKernelGGL(dgrad_mask_small_kernel<false>, dim3((B + DG_SMALL_R - 1) / DG_SMALL_R), dim3(DG_SMALL_TPB),
                         0, stream, G, ldg, K, W, ldw, X, ldx, B, GX, partial);
    return hipGetLastError();
  }
  if (((uintptr_t)G & 15) || (ldg & 3) || !workspace) return hipErrorInvalidValue;
  hipLaunchKernelGGL(dg_transpose_kernel, dim3(DG_N / 32, (K + 31) / 32), dim3(256), 0, stream, W, ldw, K, N, workspace);
  const int RB = dg_rb(B);
  const size_t lds = (size_t)16 * RB * dg_stride(K) * 4;
#define DG_LAUNCH(BB, XV)                                                                                     \
  do {                                                                                                        \
    static const hipError_t attr =                                                                            \
        hipFuncSetAttribute(reinterpret_cast<const void*>(&dgrad_mask_mfma_kernel<BB, XV>),                   \
                            hipFuncAttributeMaxDynamicSharedMemorySize, (int)((size_t)16 * BB * dg_stride(MLP_MAXD) * 4)); \
    if (attr != hipSuccess) return attr;                                                                      \
    dgrad_mask_mfma_kernel<BB, XV><<<dim3((B + 16 * BB - 1) / (16 * BB)), MLP_TPB, lds, stream>>>(            \
        G, ldg, K, workspace, X, ldx, B, GX, partial);                                                        \
  } while (0)
  if (RB == 4) {
    if (xvec) DG_LAUNCH(4, true);
    else DG_LAUNCH(4, false);
  } else if (RB == 2) {
    if (xvec) DG_LAUNCH(2, true);
    else DG_LAUNCH(2, false);
  } else {
    if (xvec) DG_LAUNCH(1, true);
    else DG_LAUNCH(1, false);
  }
#undef DG_LAUNCH
  return hipGetLastError();
}

}  // namespace hs

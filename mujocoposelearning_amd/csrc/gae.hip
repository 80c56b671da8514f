// hsim GAE reverse scan for gfx950 (MI355X).  PRODUCT CODE.
//
// Replaces SB3 2.3.2 RolloutBuffer.compute_returns_and_advantage (stable_baselines3/common/
// buffers.py), which the reference's PPO.learn runs once per rollout (train_sb3.py:229):
//   for t = T-1 .. 0:
//     nonterm = 1 - (t == T-1 ? last_dones : episode_starts[t+1])
//     nextv   =      (t == T-1 ? last_values : values[t+1])
//     delta   = rewards[t] + gamma * nextv * nonterm - values[t]
//     gae     = delta + gamma * lambda * nonterm * gae
//     adv[t]  = gae ; ret[t] = gae + values[t]
//
// Layout: [T][N] row-major float32 (the rollout buffer of ppo.PPO), so a wavefront's 64 lanes
// (64 consecutive envs) read/write 256 contiguous bytes per time step.  One lane per env, the
// recurrence runs backwards in time; the per-step loads do not depend on the carried value, so
// an unrolled block of UNROLL steps is loaded before it is consumed (UNROLL x 3 loads in flight
// per lane).  Algorithmic traffic: 12 B read + 8 B written per (t, env).
#include <hip/hip_runtime.h>

#include <cstdint>

namespace hs {
namespace {

constexpr int UNROLL = 8;
constexpr int CHUNKS = 16;   // time chunks per workgroup (one wave each): 64 envs x 16 waves

// One workgroup = 64 consecutive envs (lanes) x CHUNKS waves, wave w owning time steps
// [w L, (w+1) L).  Pass 1: each wave reduces its chunk to the affine map gae_start = A + B gae_next.
// Pass 2 (after one barrier): wave w composes the maps of the chunks after it (<= CHUNKS-1 LDS
// reads) to get its true carry-in.  Pass 3: the wave re-runs its chunk and writes adv / ret.
// Reads twice (24 B) + writes 8 B per element (algorithmic: 20 B); 16x the parallelism of one
// lane per env (1024 waves for 4096 envs instead of 64).
__global__ __launch_bounds__(64 * CHUNKS) void gae_kernel(const float* __restrict__ rew,
                                                          const float* __restrict__ val,
                                                          const float* __restrict__ start,
                                                          const float* __restrict__ last_val,
                                                          const float* __restrict__ last_done,
                                                          float* __restrict__ adv, float* __restrict__ ret, int T,
                                                          int N, float gamma, float lam) {
  __shared__ float mapA[CHUNKS][64], mapB[CHUNKS][64];
  const int lane = threadIdx.x, w = threadIdx.y;
  const int n = blockIdx.x * 64 + lane;
  const bool live = n < N;
  const size_t N_ = (size_t)N;
  const int L = (T + CHUNKS - 1) / CHUNKS;
  const int t0 = w * L, t1 = min(T, t0 + L);      // this wave's steps [t0, t1)
  const float gl = gamma * lam;
  // the step after the chunk: (values, nonterm) of t1, or the rollout's last_values / last_dones
  auto boundary = [&](float& nextv, float& nonterm) {
    if (t1 >= T) {
      nextv = last_val[n];
      nonterm = 1.f - last_done[n];
    } else {
      const size_t i = (size_t)t1 * N_ + n;
      nextv = val[i];
      nonterm = 1.f - start[i];
    }
  };
  // run the chunk backwards (gae_t = delta_t + c_t gae_{t+1}, c_t = gamma lambda nonterm_t);
  // `emit` receives (t, gae, v_t); bprod accumulates the product of the c_t
  auto run = [&](float gae, float& bprod, auto&& emit) {
    float nextv, nonterm;
    boundary(nextv, nonterm);
    int t = t1 - 1;
    for (; t - (UNROLL - 1) >= t0; t -= UNROLL) {
      float r[UNROLL], v[UNROLL], st[UNROLL];
#pragma unroll
      for (int u = 0; u < UNROLL; u++) {
        const size_t i = (size_t)(t - u) * N_ + n;
        r[u] = rew[i];
        v[u] = val[i];
        st[u] = start[i];
      }
#pragma unroll
      for (int u = 0; u < UNROLL; u++) {
        gae = r[u] + gamma * nextv * nonterm - v[u] + gl * nonterm * gae;
        bprod *= gl * nonterm;
        emit(t - u, gae, v[u]);
        nextv = v[u];
        nonterm = 1.f - st[u];
      }
    }
    for (; t >= t0; t--) {
      const size_t i = (size_t)t * N_ + n;
      const float vt = val[i];
      gae = rew[i] + gamma * nextv * nonterm - vt + gl * nonterm * gae;
      bprod *= gl * nonterm;
      emit(t, gae, vt);
      nextv = vt;
      nonterm = 1.f - start[i];
    }
    return gae;
  };
  // pass 1: A = chunk result with carry-in 0, B = product of the chunk's c_t
  float A = 0.f, B = 1.f;
  if (live && t0 < t1) A = run(0.f, B, [](int, float, float) {});
  mapA[w][lane] = A;
  mapB[w][lane] = B;
  __syncthreads();
  if (!live || t0 >= t1) return;
  float g = 0.f;                                    // gae after the last step of the rollout
  for (int c = CHUNKS - 1; c > w; c--) g = mapA[c][lane] + mapB[c][lane] * g;
  float unused = 1.f;
  run(g, unused, [&](int t, float gae, float vt) {
    const size_t i = (size_t)t * N_ + n;
    adv[i] = gae;
    ret[i] = gae + vt;
  });
}

// Long rollouts (T >= GAE_SPLIT_T, e.g. the README config's n_steps 2048): the kernel above gets only
// N / 64 workgroups (64 of 256 CUs at N = 4096), so the scan runs as three launches over
// (env group, time chunk) waves instead, with no workspace: the chunk maps and then the carries live
// in the output rows the last launch overwrites.
//   maps:  wave (g, c) reduces chunk c of envs [64 g, 64 g + 64) to gae_start = A + B gae_next and
//          stores A in adv and B in ret at the chunk's last row;
//   carry: one thread per env composes the maps from the last chunk back and stores each chunk's
//          carry-in over its A (each slot is read before it is written, by the same thread);
//   apply: wave (g, c) re-runs its chunk from that carry and writes adv / ret (its first write is the
//          carry slot it has just read).
// Reads twice (24 B) + writes 8 B per element, as the one-launch kernel; the second read of the
// 100 MB rollout buffer can be served by the 256 MB MALL.
constexpr int GAE_SPLIT_T = 256;

__device__ __forceinline__ float gae_run_chunk(const float* __restrict__ rew, const float* __restrict__ val,
                                               const float* __restrict__ start, const float* __restrict__ last_val,
                                               const float* __restrict__ last_done, float* __restrict__ adv,
                                               float* __restrict__ ret, size_t N_, int n, int T, int t0, int t1,
                                               float gamma, float gl, float gae, float& bprod, bool emit) {
  float nextv, nonterm;
  if (t1 >= T) {
    nextv = last_val[n];
    nonterm = 1.f - last_done[n];
  } else {
    const size_t i = (size_t)t1 * N_ + n;
    nextv = val[i];
    nonterm = 1.f - start[i];
  }
  int t = t1 - 1;
  for (; t - (UNROLL - 1) >= t0; t -= UNROLL) {
    float r[UNROLL], v[UNROLL], st[UNROLL];
#pragma unroll
    for (int u = 0; u < UNROLL; u++) {
      const size_t i = (size_t)(t - u) * N_ + n;
      r[u] = rew[i];
      v[u] = val[i];
      st[u] = start[i];
    }
#pragma unroll
    for (int u = 0; u < UNROLL; u++) {
      gae = r[u] + gamma * nextv * nonterm - v[u] + gl * nonterm * gae;
      bprod *= gl * nonterm;
      if (emit) {
        const size_t i = (size_t)(t - u) * N_ + n;
        adv[i] = gae;
        ret[i] = gae + v[u];
      }
      nextv = v[u];
      nonterm = 1.f - st[u];
    }
  }
  for (; t >= t0; t--) {
    const size_t i = (size_t)t * N_ + n;
    const float vt = val[i];
    gae = rew[i] + gamma * nextv * nonterm - vt + gl * nonterm * gae;
    bprod *= gl * nonterm;
    if (emit) {
      adv[i] = gae;
      ret[i] = gae + vt;
    }
    nextv = vt;
    nonterm = 1.f - start[i];
  }
  return gae;
}

__global__ __launch_bounds__(64) void gae_maps_kernel(const float* __restrict__ rew, const float* __restrict__ val,
                                                      const float* __restrict__ start,
                                                      const float* __restrict__ last_val,
                                                      const float* __restrict__ last_done, float* __restrict__ adv,
                                                      float* __restrict__ ret, int T, int N, int L, float gamma,
                                                      float lam) {
  const int n = blockIdx.x * 64 + threadIdx.x, t0 = blockIdx.y * L, t1 = min(T, t0 + L);
  if (n >= N || t0 >= t1) return;
  float B = 1.f;
  const float A = gae_run_chunk(rew, val, start, last_val, last_done, adv, ret, (size_t)N, n, T, t0, t1, gamma,
                                gamma * lam, 0.f, B, false);
  const size_t i = (size_t)(t1 - 1) * N + n;
  adv[i] = A;
  ret[i] = B;
}

__global__ __launch_bounds__(256) void gae_carry_kernel(float* __restrict__ adv, const float* __restrict__ ret,
                                                        int T, int N, int L) {
  const int n = blockIdx.x * 256 + threadIdx.x;
  if (n >= N) return;
  const int C = (T + L - 1) / L;
  float g = 0.f;
  int c = C - 1;
  for (; c - (UNROLL - 1) >= 0; c -= UNROLL) {   // the maps' loads do not depend on the carry
    float a[UNROLL], b[UNROLL];
#pragma unroll
    for (int u = 0; u < UNROLL; u++) {
      const size_t i = (size_t)(min(T, (c - u + 1) * L) - 1) * N + n;
      a[u] = adv[i];
      b[u] = ret[i];
    }
#pragma unroll
    for (int u = 0; u < UNROLL; u++) {
      adv[(size_t)(min(T, (c - u + 1) * L) - 1) * N + n] = g;
      g = a[u] + b[u] * g;
    }
  }
  for (; c >= 0; c--) {
    const size_t i = (size_t)(min(T, (c + 1) * L) - 1) * N + n;
    const float a = adv[i], b = ret[i];
    adv[i] = g;
    g = a + b * g;
  }
}

__global__ __launch_bounds__(64) void gae_apply_kernel(const float* __restrict__ rew, const float* __restrict__ val,
                                                       const float* __restrict__ start,
                                                       const float* __restrict__ last_val,
                                                       const float* __restrict__ last_done, float* __restrict__ adv,
                                                       float* __restrict__ ret, int T, int N, int L, float gamma,
                                                       float lam) {
  const int n = blockIdx.x * 64 + threadIdx.x, t0 = blockIdx.y * L, t1 = min(T, t0 + L);
  if (n >= N || t0 >= t1) return;
  const float g = adv[(size_t)(t1 - 1) * N + n];   // this chunk's carry-in (gae_carry_kernel)
  float unused = 1.f;
  gae_run_chunk(rew, val, start, last_val, last_done, adv, ret, (size_t)N, n, T, t0, t1, gamma, gamma * lam, g,
                unused, true);
}

}  // namespace

hipError_t launch_gae(const float* rew, const float* val, const float* start, const float* last_val,
                      const float* last_done, float* adv, float* ret, int T, int N, float gamma, float lam,
                      hipStream_t stream) {
  if (T <= 0 || N <= 0) return hipSuccess;
  if (T >= GAE_SPLIT_T) {
    // ~4096 (env group, chunk) waves: chunks of L >= 16 steps
    const int groups = (N + 63) / 64;
    int L = (int)(((long long)T * groups + 4095) / 4096);
    L = L < 16 ? 16 : L;
    const int C = (T + L - 1) / L;
    const dim3 grid(groups, C);
    hipLaunchKernelGGL(gae_maps_kernel, grid, dim3(64), 0, stream, rew, val, start, last_val, last_done, adv, ret, T,
                       N, L, gamma, lam);
    hipLaunchKernelGGL(gae_carry_kernel, dim3((N + 255) / 256), dim3(256), 0, stream, adv, ret, T, N, L);
    hipLaunchKernelGGL(gae_apply_kernel, grid, dim3(64), 0, stream, rew, val, start, last_val, last_done, adv, ret, T,
                       N, L, gamma, lam);
    return hipGetLastError();
  }
  const dim3 block(64, CHUNKS);
  const dim3 grid((N + 63) / 64);
  hipLaunchKernelGGL(gae_kernel, grid, block, 0, stream, rew, val, start, last_val, last_done, adv, ret, T, N,
                     gamma, lam);
  return hipGetLastError();
}

}  // namespace hs

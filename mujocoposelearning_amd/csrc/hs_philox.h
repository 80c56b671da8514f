// Counter-based Gaussian noise of the PPO rollout (product): Philox4x32-10 (Salmon et al., SC'11)
// keyed by the 64-bit seed, and a Box-Muller transform of two of its words.  Shared by the per-step
// sampler (ppo.hip ppo_act_kernel) and the fused rollout (hs_kernels.hip), so both draw bitwise the
// same z for the same (env, action index, rollout step).
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>

namespace hs {

struct U4 {
  uint32_t x, y, z, w;
};

__device__ inline U4 philox4x32_10(U4 c, uint32_t k0, uint32_t k1) {
  constexpr uint32_t M0 = 0xD2511F53u, M1 = 0xCD9E8D57u, W0 = 0x9E3779B9u, W1 = 0xBB67AE85u;
#pragma unroll
  for (int r = 0; r < 10; r++) {
    const uint32_t hi0 = __umulhi(M0, c.x), lo0 = M0 * c.x;
    const uint32_t hi1 = __umulhi(M1, c.z), lo1 = M1 * c.z;
    c = U4{hi1 ^ c.y ^ k0, lo1, hi0 ^ c.w ^ k1, lo0};
    k0 += W0;
    k1 += W1;
  }
  return c;
}

// standard normal from two uniform words (Box-Muller, u1 in (0, 1])
__device__ inline float box_muller(uint32_t a, uint32_t b) {
  const float u1 = ((float)(a >> 8) + 1.0f) * (1.0f / 16777216.0f);
  const float u2 = (float)(b >> 8) * (1.0f / 16777216.0f);
  return sqrtf(-2.0f * __logf(u1)) * __cosf(6.283185307179586f * u2);
}

// z of (env n, action index j, rollout-step counter c): the counter block is (n * 32 + j, n >> 27, c)
__device__ inline float policy_noise(uint32_t n, uint32_t j, uint64_t c, uint32_t k0, uint32_t k1) {
  const U4 r = philox4x32_10(U4{n * 32u + j, n >> 27, (uint32_t)c, (uint32_t)(c >> 32)}, k0, k1);
  return box_muller(r.x, r.y);
}

// sum over the 32 lanes of a half-wave (xor butterfly stays inside the half)
__device__ inline float half_sum(float v) {
#pragma unroll
  for (int o = 16; o >= 1; o >>= 1) v += __shfl_xor(v, o, 32);
  return v;
}

}  // namespace hs

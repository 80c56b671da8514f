// hsim step kernel for gfx950 (MI355X).  PRODUCT CODE.
//
// Replaces, for a whole batch of envs at once:
//   custom_env.py:152-230  HumanoidEnv.step   (frame_skip x {ctrl = a; mj_step}, obs, reward, done)
//   custom_env.py:97-150   HumanoidEnv.reset  (mj_resetData, noise, one ctrl=0 mj_step, obs)
//   custom_env.py:232-261  _get_state         (352-dim obs, stale derived fields)
//   reward_functions.py:66-261 stand / kneeling / walk rewards (device plug-ins)
//   SB3 SubprocVecEnv auto-reset semantics (train_sb3.py:203)
// and MuJoCo 3.2.5's mj_step pipeline (custom_env.py:121,160): kinematics, com, collision, CRB,
// RNE, actuation, constraint assembly, primal Newton solver (pyramidal cones; MuJoCo's default) or,
// in the <option solver="PGS"> instance, projected Gauss-Seidel on the dual, Euler with implicit
// joint damping.
//
// Execution model: TWO ENVS PER WAVEFRONT.  Lanes 0-31 step env 2w, lanes 32-63 env 2w+1; a
// half-wave maps its 32 lanes to bodies / dofs / geoms / joints / contacts / constraint rows
// stage by stage (humanoid: 17 bodies, 27 dofs, <= 32 contacts), so a wave64 instruction does
// useful work for both envs.  Per-env state lives in LDS (phase-local arrays aliased in a union
// so one wave = 2 envs fits 20 KB: all 4096 envs of configs[1] are resident at once).  Dense
// nv x nv matrices (M, the Newton Hessian, M + h*B) live row-per-lane in VGPRs and are factored
// with per-half v_readlane broadcasts.  The contact part of the Newton Hessian uses the
// tree-structured form H_ij += jp_j' U jp_i (O(nv * ncon), no nefc x nv Jacobian in memory).
// HBM traffic is only the per-env state in/out; the model is read through L1/L2.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdint>
#include <type_traits>

#include "hs_kernels.h"
#include "hs_philox.h"
#include "hs_model.h"

namespace hs {
namespace {

constexpr int WAVE = 64;
constexpr int HL = 32;            // lanes per env
static_assert(MAXDOF == HL, "one dof per sub-lane (lim_row slots, dof masks)");

// Per-env contact / constraint-row capacity of a kernel instance (hs_model.h): the resident tier
// every launch runs with and the wide tier that re-runs the (rare) envs overflowing it.
template <int NCON, int NEFC, bool W = false>
struct Cap {
  static constexpr int CON = NCON;        // contacts (at most one slot per lane per HL-slot pass)
  static constexpr int EFC = NEFC;        // constraint rows
  static constexpr int RPL = NEFC / HL;   // rows per lane (kept in registers by the row's lane)
  static constexpr bool WIDE = W;         // the wide (re-run) tier
  static_assert((NCON % HL == 0 || HL % NCON == 0) && NEFC % HL == 0, "capacity in whole half-waves");
};
// resident tier per precision (hs_model.h)
template <typename T>
using Resident = std::conditional_t<sizeof(T) == 8, Cap<MAXCON_F64, MAXEFC_F64>, Cap<MAXCON, MAXEFC>>;
using Wide = Cap<MAXCON_WIDE, MAXEFC_WIDE, true>;

// scheduling fence: keeps the machine scheduler from hoisting loads across iterations of fully
// unrolled loops (which otherwise inflates VGPR pressure far past the occupancy target)
#define SCHED_FENCE() __builtin_amdgcn_sched_barrier(0)
// Cholesky pivot block by DPP broadcast instead of LDS read-back, per precision (bit 0 the fp32
// engine, bit 1 the fp64 engine).  A/B, ms per configs[1] launch: fp64 0.720 -> 0.714 (with the
// normal-range sqrt below 0.701); fp32 0.423 -> 0.433 (2 waves per SIMD hide the LDS round trip,
// and the extra VALU ops cost issue slots): fp64 only.
// contact aggregates over a contact's rows as straight-line code: all LDS operands read up front
// instead of a row loop whose every iteration waits on its own reads (fp64 0.662 -> 0.634 ms per
// configs[1] launch)
// fp64 1/x as rcp + one cubic correction (e + e^2) instead of two Newton steps: 4 dependent
// operations instead of 5, the same ~1 ulp (0.662 -> 0.656 ms)
// fp64 1/sqrt without the denormal / class handling of the library sqrt (development A/B knob)
// CRB and Newton-Hessian rows software-pipelined: the next column (group)'s LDS reads are issued
// before the current one's arithmetic, behind the per-column scheduling fence, so each LDS round trip
// overlaps the previous column's FMAs (A/B, fp64 ms per configs[1] launch: 0.681 -> CRB 0.674,
// Hessian 0.661, both 0.659; the fp64 queue kernel drops from 510 to 482 unified registers)
// Cholesky, per precision (bit 0 fp32, bit 1 fp64): trailing-column LDS reads issued before the pivot math, behind a
// scheduling fence (the machine scheduler otherwise sinks the column publish and its read-back below
// the pivot chain, exposing the LDS round trip): 0.691 -> 0.682 ms per fp64 configs[1] launch; fp32
// (pivots from LDS too, so one round trip instead of two): 0.390 -> 0.387 ms
// M·v with two accumulators: no change.  Removing the per-loop scheduling fences
// costs 1136 / 564 B/lane of scratch (Cholesky / CRB).
// columns per scheduling group in the Hessian / CRB row loops (A/B, fp64 configs[1] ms per launch:
// Hessian 2 columns 0.720 vs 1 column 0.724, 3 spill; CRB 2 or 3 columns: no change)
// (the fp32 engine at 2 waves per SIMD has no registers for a second column: 148 B/lane of scratch)

// single-wave workgroup: LDS ops of a wave execute in order, so a compiler-only barrier suffices to
// keep LDS accesses from moving across phase boundaries (no s_barrier, and no s_waitcnt that a
// workgroup-scope fence would add).
#define WSYNC() asm volatile("" ::: "memory")

// ------------------------------------------------------------------ cross-lane helpers
// compile-time loop: f(std::integral_constant<int, i>) for i in [B, E)
template <int B, int E, typename F>
__device__ __forceinline__ void static_for(F&& f) {
  if constexpr (B < E) {
    f(std::integral_constant<int, B>{});
    static_for<B + 1, E>(f);
  }
}
// bound_ctrl set: every pattern used here reads in-bounds lanes only, and with it the DPP combiner
// folds the move into its consumer (hsum's adds become single v_add_f32_dpp instructions)
template <int CTRL>
__device__ __forceinline__ uint32_t dpp32(uint32_t v) {
  return (uint32_t)__builtin_amdgcn_mov_dpp((int)v, CTRL, 0xF, 0xF, true);
}
// v_permlane16_swap(v, v): .first = rows {0,0,2,2}, .second = rows {1,1,3,3} (row = 16 lanes),
// i.e. every lane of a 32-lane half sees the half's low row in .first and its high row in .second.
struct RowPair { uint32_t lo, hi; };
__device__ __forceinline__ RowPair rowswap(uint32_t v) {
  auto r = __builtin_amdgcn_permlane16_swap(v, v, false, false);
  return {r[0], r[1]};
}
// value of sub-lane K (compile-time) of the caller's 32-lane half: DPP row_newbcast + one
// permlane16 swap -- 3 VALU ops, no SGPR round trip, and bcast<K> / bcast<K+16> share both ops.
template <int K>
__device__ __forceinline__ uint32_t bcast32(uint32_t v) {
  RowPair r = rowswap(dpp32<0x150 + (K & 15)>(v));
  return K < 16 ? r.lo : r.hi;
}
template <int K>
__device__ __forceinline__ float bcast(float v) {
  return __uint_as_float(bcast32<K>(__float_as_uint(v)));
}
template <int K>
__device__ __forceinline__ double bcast(double v) {
  uint64_t x = (uint64_t)__double_as_longlong(v);
  uint64_t lo = bcast32<K>((uint32_t)x), hi = bcast32<K>((uint32_t)(x >> 32));
  return __longlong_as_double((long long)((hi << 32) | lo));
}
template <int CTRL>
__device__ __forceinline__ float dpp(float v) {
  return __uint_as_float(dpp32<CTRL>(__float_as_uint(v)));
}
template <int CTRL>
__device__ __forceinline__ double dpp(double v) {
  uint64_t x = (uint64_t)__double_as_longlong(v);
  uint64_t lo = dpp32<CTRL>((uint32_t)x), hi = dpp32<CTRL>((uint32_t)(x >> 32));
  return __longlong_as_double((long long)((hi << 32) | lo));
}
__device__ __forceinline__ float rows_sum(float v) {
  RowPair r = rowswap(__float_as_uint(v));
  return __uint_as_float(r.lo) + __uint_as_float(r.hi);
}
__device__ __forceinline__ double rows_sum(double v) {
  uint64_t x = (uint64_t)__double_as_longlong(v);
  RowPair l = rowswap((uint32_t)x), h = rowswap((uint32_t)(x >> 32));
  return __longlong_as_double((long long)(((uint64_t)h.lo << 32) | l.lo)) +
         __longlong_as_double((long long)(((uint64_t)h.hi << 32) | l.hi));
}
// the value of the same position in the half's high 16-lane row (valid on the low row's lanes)
__device__ __forceinline__ float up_row(float v) { return __uint_as_float(rowswap(__float_as_uint(v)).hi); }
__device__ __forceinline__ double up_row(double v) {
  uint64_t x = (uint64_t)__double_as_longlong(v);
  const uint64_t lo = rowswap((uint32_t)x).hi, hi = rowswap((uint32_t)(x >> 32)).hi;
  return __longlong_as_double((long long)((hi << 32) | lo));
}
// sum over each 32-lane half (result in every lane of the half); all-VALU, no LDS permute
template <typename T>
__device__ __forceinline__ T hsum(T v) {
  v += dpp<0xB1>(v);    // quad_perm [1,0,3,2]
  v += dpp<0x4E>(v);    // quad_perm [2,3,0,1]
  v += dpp<0x141>(v);   // row_half_mirror
  v += dpp<0x140>(v);   // row_mirror
  return rows_sum(v);   // + the other 16-lane row of the half
}
__device__ __forceinline__ uint32_t hballot(bool p, bool upper) {
  uint64_t m = __ballot(p);
  return upper ? (uint32_t)(m >> 32) : (uint32_t)m;
}
// f(j, ld(j)) for each set bit j of mk, ascending (the chain / subtree sums).  AHEAD: the loads of the
// next bit's operands are issued before the current bit's arithmetic, so one LDS round trip overlaps
// the FMAs (the same operations in the same order) -- the contact loops take it; for the chain /
// subtree sums it measured slower in both engines (fp64 0.697 vs 0.691 ms, fp32 0.411 vs 0.408 ms
// per configs[1] launch).
template <typename T, bool AHEAD = false, typename LD, typename F>
__device__ __forceinline__ void for_bits(uint32_t mk, LD&& ld, F&& f) {
  if constexpr (AHEAD) {
    if (mk == 0u) return;
    int j = __builtin_ctz(mk);
    mk &= mk - 1u;
    auto cur = ld(j);
    for (; mk; mk &= mk - 1u) {
      const int jn = __builtin_ctz(mk);
      auto nxt = ld(jn);
      f(j, cur);
      cur = nxt;
      j = jn;
    }
    f(j, cur);
  } else {
    for (; mk; mk &= mk - 1u) {
      const int j = __builtin_ctz(mk);
      f(j, ld(j));
    }
  }
}
template <typename T, int N>
struct Vals { T v[N]; };
template <typename T, int N>
struct ValsX { T x; T v[N]; };

// Hide a (uniform) pointer's value from the optimiser.  The model pointer is const __restrict__,
// so without this LICM hoists every per-lane model load (m->dof_bodyid[sl], ...) out of the
// substep / Newton loops and keeps each one live in a VGPR for the whole kernel.
// (The value is wave-uniform by construction; readfirstlane only tells the uniformity analysis so,
// where control flow hides it -- e.g. across the chunk-queue loop -- and folds away otherwise.)
template <typename P>
__device__ __forceinline__ P opaque(P p) {
  uint64_t v = (uint64_t)p;
  uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)v), hi = __builtin_amdgcn_readfirstlane((uint32_t)(v >> 32));
  v = ((uint64_t)hi << 32) | lo;
  asm volatile("" : "+s"(v));
  return (P)v;
}
// The model lives in the constant address space: it is never written by the kernel, so reads at
// a wave-uniform index become scalar loads (s_load via the scalar cache) even through an
// opaque()-laundered pointer; lane-varying reads stay vector loads.
template <typename T>
using MPtr = const __attribute__((address_space(4))) DevModel<T>*;
template <typename T>
using CPtr = const __attribute__((address_space(4))) T*;      // pointer into the model
// All launch arguments travel as ONE by-value struct, so it sits at offset 0 of the kernarg
// segment.  The kernel reads it through an opaque()-laundered constant-address-space pointer to
// that segment: every use is a fresh scalar load (scalar cache) instead of ~80 SGPRs kept live
// for the whole kernel (which spill to VGPR lanes, and the per-lane buffer addresses derived
// from them to scratch -- 150 B/lane of spill traffic written back to HBM every launch).
template <typename T>
struct KArgs {
  MPtr<T> m;
  EnvBuffers<T> b;
  const float* actions;       // [N][nu] f32 (null in MODE_RESET)
  const uint8_t* reset_mask;  // [N] or null
  const T* nz_q;              // [N][nq] host reset noise or null (device RNG)
  const T* nz_v;              // [N][nv] or null
  StepParams p;
  int nenv;
  TapeOut<T> tape;            // per-step outputs of a tape launch (p.nsteps > 1), or all null
  RolloutArgs ro;             // fused rollout (ro.obs != null): actions from the policy, see hs_kernels.h
};
template <typename T>
using KPtr = const __attribute__((address_space(4))) KArgs<T>*;
// Same for a per-lane value: stops lane-invariant compare masks (j <= sl, bit(mask, sl), ...)
// being hoisted out of the loops as dozens of 64-bit SGPR masks (which then spill).
__device__ __forceinline__ int opaque_v(int x) {
  asm volatile("" : "+v"(x));
  return x;
}
__device__ __forceinline__ int below(uint32_t m, int sl) { return __popc(m & ((1u << sl) - 1u)); }
__device__ __forceinline__ bool bit(uint32_t mask, int i) { return i < 32 && ((mask >> i) & 1u); }
template <typename T>
__device__ __forceinline__ bool isbad(T x) {
  return !(x <= T(1e10) && x >= T(-1e10));   // NaN or |x| > mjMAXVAL
}

// Chunk-queue hand-off rows (b.mid, uncached) are written and read at agent scope.  A row is rewritten
// by one CU and read by another, and a tape launch reads env e's row once per env step, often on a CU
// whose vector L1 still holds the line from an earlier step: plain loads could return that stale line
// (measured: tape launches were nondeterministic with plain loads, tests/test_gpu_tape.py).
template <typename T>
__device__ __forceinline__ T row_ld(const T* p) {
  return __hip_atomic_load(const_cast<T*>(p), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
template <typename T>
__device__ __forceinline__ void row_st(T* p, T v) {
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// ------------------------------------------------------------------ small algebra
// sin/cos: fp64 libm for the parity mode; the fp32 engine uses the hardware v_sin/v_cos
// (|error| ~1e-6 on the half joint angles, inside the fp32 tolerance)
__device__ __forceinline__ void sincos_t(double x, double& s, double& c) { sincos(x, &s, &c); }
__device__ __forceinline__ void sincos_t(float x, float& s, float& c) { s = __sinf(x); c = __cosf(x); }
template <typename T>
__device__ __forceinline__ void quat2mat(const T* q, T* R) {
  T w = q[0], x = q[1], y = q[2], z = q[3];
  R[0] = 1 - 2 * (y * y + z * z); R[1] = 2 * (x * y - w * z); R[2] = 2 * (x * z + w * y);
  R[3] = 2 * (x * y + w * z); R[4] = 1 - 2 * (x * x + z * z); R[5] = 2 * (y * z - w * x);
  R[6] = 2 * (x * z - w * y); R[7] = 2 * (y * z + w * x); R[8] = 1 - 2 * (x * x + y * y);
}
template <typename T>
__device__ __forceinline__ void mulq(const T* a, const T* b, T* r) {
  T t0 = a[0] * b[0] - a[1] * b[1] - a[2] * b[2] - a[3] * b[3];
  T t1 = a[0] * b[1] + a[1] * b[0] + a[2] * b[3] - a[3] * b[2];
  T t2 = a[0] * b[2] - a[1] * b[3] + a[2] * b[0] + a[3] * b[1];
  T t3 = a[0] * b[3] + a[1] * b[2] - a[2] * b[1] + a[3] * b[0];
  r[0] = t0; r[1] = t1; r[2] = t2; r[3] = t3;
}
template <typename T>
__device__ __forceinline__ void mv3(const T* R, const T* v, T* r) {
  T a = R[0] * v[0] + R[1] * v[1] + R[2] * v[2];
  T b = R[3] * v[0] + R[4] * v[1] + R[5] * v[2];
  T c = R[6] * v[0] + R[7] * v[1] + R[8] * v[2];
  r[0] = a; r[1] = b; r[2] = c;
}
template <typename T>
__device__ __forceinline__ void cross3(const T* a, const T* b, T* r) {
  T x = a[1] * b[2] - a[2] * b[1], y = a[2] * b[0] - a[0] * b[2], z = a[0] * b[1] - a[1] * b[0];
  r[0] = x; r[1] = y; r[2] = z;
}
template <typename T>
__device__ __forceinline__ T dot3(const T* a, const T* b) { return a[0] * b[0] + a[1] * b[1] + a[2] * b[2]; }
template <typename T>
__device__ __forceinline__ T dot6(const T* a, const T* b) {
  return a[0] * b[0] + a[1] * b[1] + a[2] * b[2] + a[3] * b[3] + a[4] * b[4] + a[5] * b[5];
}
template <typename T>
__device__ __forceinline__ T rsqrt_t(T x);
template <>
__device__ __forceinline__ float rsqrt_t<float>(float x) { return __builtin_amdgcn_rsqf(x); }
// fp64: below recip()
// 1/x: fp32 is v_rcp_f32 under -fno-hip-fp32-correctly-rounded-divide-sqrt; fp64 is v_rcp_f64 +
// two Newton steps (within 1-2 ulp of the correctly rounded divide, for normal nonzero x)
__device__ __forceinline__ float recip(float x) { return 1.0f / x; }
__device__ __forceinline__ double recip(double x) {
  double y = __builtin_amdgcn_rcp(x);
  // y (1 + e + e^2) with e = 1 - x y: relative error cubed in one step (4 dependent operations)
  const double e = fma(-x, y, 1.0);
  return fma(fma(e, e, e), y, y);
}
// fp64 1/sqrt(x), x >= 1e-30 at every call site (the Cholesky pivots are clamped to it, the
// normalizations branch below it), so no denormal scaling or zero / infinity class check:
// v_rsq_f64, one Goldschmidt step (h ~ 1/(2 sqrt x)), one Newton step on y = 2h -- within ~1 ulp,
// 7 dependent operations.  A/B, fp64 ms per configs[1] launch (with the DPP pivots of chol_rows):
// recip(sqrt(x)) (18 operations) 0.714, the library sqrt sequence without its scaling / class check
// then recip() (13) 0.701, this 0.690.  (Round 2 measured a v_rsq_f64 + two-Newton-step variant
// slower, 305k vs 298k cycles per env substep, under the default machine scheduler.)
template <>
__device__ __forceinline__ double rsqrt_t<double>(double x) {
  const double y = __builtin_amdgcn_rsq(x);
  double g = x * y, h = 0.5 * y;
  const double r = fma(-h, g, 0.5);
  h = fma(h, r, h);
  const double y1 = h + h;
  const double e = fma(-(x * y1), y1, 1.0);
  return fma(h, e, y1);
}
template <typename T>
__device__ __forceinline__ T normalize3(T* v) {
  const T n2 = dot3(v, v);
  if (n2 < T(1e-30)) { v[0] = 1; v[1] = 0; v[2] = 0; return sqrt(n2); }
  const T i = rsqrt_t(n2);
  v[0] *= i; v[1] *= i; v[2] *= i;
  return n2 * i;
}
template <typename T>
__device__ __forceinline__ void normalize4(T* q) {
  const T n2 = q[0] * q[0] + q[1] * q[1] + q[2] * q[2] + q[3] * q[3];
  if (n2 < T(1e-30)) { q[0] = 1; q[1] = q[2] = q[3] = 0; }
  else { const T i = rsqrt_t(n2); q[0] *= i; q[1] *= i; q[2] *= i; q[3] *= i; }
}
// spatial inertia (10-param cinert layout) times motion vector (mju_mulInertVec)
template <typename T>
__device__ __forceinline__ void mul_inert(const T* i, const T* v, T* r) {
  r[0] = i[0] * v[0] + i[3] * v[1] + i[4] * v[2] - i[8] * v[4] + i[7] * v[5];
  r[1] = i[3] * v[0] + i[1] * v[1] + i[5] * v[2] + i[8] * v[3] - i[6] * v[5];
  r[2] = i[4] * v[0] + i[5] * v[1] + i[2] * v[2] - i[7] * v[3] + i[6] * v[4];
  r[3] = i[8] * v[1] - i[7] * v[2] + i[9] * v[3];
  r[4] = i[6] * v[2] - i[8] * v[0] + i[9] * v[4];
  r[5] = i[7] * v[0] - i[6] * v[1] + i[9] * v[5];
}
template <typename T>
__device__ __forceinline__ void cross_motion(const T* v, const T* m, T* r) {
  r[0] = -v[2] * m[1] + v[1] * m[2];
  r[1] = v[2] * m[0] - v[0] * m[2];
  r[2] = -v[1] * m[0] + v[0] * m[1];
  r[3] = -v[2] * m[4] + v[1] * m[5] - v[5] * m[1] + v[4] * m[2];
  r[4] = v[2] * m[3] - v[0] * m[5] + v[5] * m[0] - v[3] * m[2];
  r[5] = -v[1] * m[3] + v[0] * m[4] - v[4] * m[0] + v[3] * m[1];
}
template <typename T>
__device__ __forceinline__ void cross_force(const T* v, const T* f, T* r) {
  r[0] = -v[2] * f[1] + v[1] * f[2] - v[5] * f[4] + v[4] * f[5];
  r[1] = v[2] * f[0] - v[0] * f[2] + v[5] * f[3] - v[3] * f[5];
  r[2] = -v[1] * f[0] + v[0] * f[1] - v[4] * f[3] + v[3] * f[4];
  r[3] = -v[2] * f[4] + v[1] * f[5];
  r[4] = v[2] * f[3] - v[0] * f[5];
  r[5] = -v[1] * f[3] + v[0] * f[4];
}

// ------------------------------------------------------------------ row-per-lane dense algebra
// Cholesky A = L L' of an NV x NV SPD matrix held row-per-lane in each half (sub-lane i: row i);
// on return A holds L's strictly lower part (diagonal and upper part zeroed, so the substitutions
// below need no lane selects) and dinv (sub-lane i) = 1 / L_ii.  Step k
// publishes column k (a_ik, one ds_write) in the env's LDS vector `col`; every lane reads the
// pivot and a_jk (j > k) back as broadcast ds_reads, so the update is pure FMAs:
//   A_ij -= (a_ik / a_kk) a_jk.

// LDL: return the factor as L D L' instead (unit lower L's strictly lower part in A, dinv = 1/d_i,
// *diag = d_i): the same elimination, each finished column scaled by its pivot's 1/L_kk on the way.
template <int NV, typename T, bool LDL = false>
__device__ __forceinline__ void chol_rows(T (&A)[NV], T& dinv, int sl, T (*cb)[2], T* diag = nullptr) {
  constexpr bool CDPP = sizeof(T) == 8;   // pivot block by DPP: the fp64 engine only (see above)
  // two columns per LDS round trip: every lane publishes (a_ik, a_i,k+1) as one ds_write and reads
  // the 2x2 pivot block and (a_jk, a_j,k+1) back as broadcasts.  With L_P the pivot block's
  // Cholesky factor (1/L_kk = r1, L_k+1,k = l10, 1/L_k+1,k+1 = r2), row i gets
  //   z = L_P^-1 (a_ik, a_i,k+1)   (its L entries)    f = L_P^-T z   (its Schur coefficients)
  //   A_ij -= f0 a_jk + f1 a_j,k+1   (j >= k+2)
  // and the pivot rows' own z are their L entries (L_kk, and l10, L_k+1,k+1).
  static_for<0, NV / 2>([&](auto bc) {
    constexpr int k = 2 * decltype(bc)::value;
    const int sl_k = opaque_v(sl);     // fresh compare per step (no 64-bit mask kept live)
    cb[sl_k][0] = A[k];
    cb[sl_k][1] = A[k + 1];
    T p, q, t;
    if constexpr (CDPP) {   // the pivot block by DPP broadcast from lanes k, k+1: the LDS round trip
      // of the column publish leaves the pivot chain (the trailing update still reads a_jk from LDS);
      // the pivot is clamped before the broadcast (an FMA result: no NaN canonicalization for v_max)
      p = bcast<k>(A[k] > T(1e-30) ? A[k] : T(1e-30));
      q = bcast<k + 1>(A[k]);
      t = bcast<k + 1>(A[k + 1]);
    } else {
      p = cb[k][0];
      q = cb[k + 1][0];
      t = cb[k + 1][1];
      p = p > T(1e-30) ? p : T(1e-30);
    }
    // the trailing columns' broadcast reads issued before the pivot math (fenced), so their LDS round
    // trip overlaps the pivot chain instead of following it
    T cj[NV][2];
    static_for<k + 2, NV>([&](auto jc) {
      constexpr int j = decltype(jc)::value;
      cj[j][0] = cb[j][0];
      cj[j][1] = cb[j][1];
    });
    SCHED_FENCE();
    T r1 = rsqrt_t(p);
    T l10 = q * r1;
    T s11 = t - l10 * l10;
    s11 = s11 > T(1e-30) ? s11 : T(1e-30);
    T r2 = rsqrt_t(s11);
    T z0 = A[k] * r1;
    T z1 = (sl_k == k + 1) ? s11 * r2 : (A[k + 1] - l10 * z0) * r2;
    T f1 = z1 * r2;
    T f0 = (z0 - l10 * f1) * r1;
    if constexpr (LDL) {   // L~_ik = L_ik / L_kk, d = L_kk^2 (the pivots' own entries are zeroed below)
      A[k] = z0 * r1;
      A[k + 1] = z1 * r2;
      dinv = (sl_k == k) ? r1 * r1 : ((sl_k == k + 1) ? r2 * r2 : dinv);
      *diag = (sl_k == k) ? p : ((sl_k == k + 1) ? s11 : *diag);
    } else {
      A[k] = (sl_k == k) ? p * r1 : z0;
      A[k + 1] = z1;
      dinv = (sl_k == k) ? r1 : ((sl_k == k + 1) ? r2 : dinv);
    }
    static_for<k + 2, NV>([&](auto jc) {
      constexpr int j = decltype(jc)::value;
      A[j] = fma(-f0, cj[j][0], fma(-f1, cj[j][1], A[j]));
    });
    SCHED_FENCE();
  });
  if constexpr (NV % 2 == 1) {         // trailing single column
    constexpr int k = NV - 1;
    const int sl_k = opaque_v(sl);
    T akk;
    if constexpr (CDPP) {
      akk = bcast<k>(A[k]);
    } else {
      cb[sl_k][0] = A[k];
      akk = cb[k][0];
    }
    akk = akk > T(1e-30) ? akk : T(1e-30);
    if constexpr (LDL) {
      const T r = rsqrt_t(akk);
      A[k] = A[k] * r * r;
      dinv = (sl_k == k) ? r * r : dinv;
      *diag = (sl_k == k) ? akk : *diag;
    } else {
      const T r = rsqrt_t(akk);
      A[k] = (sl_k == k) ? akk * r : A[k] * r;
      dinv = (sl_k == k) ? r : dinv;
    }
  }
  const int sl_z = opaque_v(sl);
  static_for<0, NV>([&](auto jc) {
    constexpr int j = decltype(jc)::value;
    A[j] = sl_z > j ? A[j] : T(0);
  });
}
// solve (L L') x = b (L from chol_rows: strictly lower part, 1/L_ii in dinv); sub-lane i holds b_i;
// returns x_i.  Forward: at step k every lane subtracts L_ik y_k (zero unless i > k), so lane k's b
// stops changing once y_k = b_k / L_kk is broadcast, and y = b / L_ii at the end.
// UNIT: L D L' form instead (unit lower L, 1/d_i in dinv): forward with L, scale by 1/d, back with L'.
template <int NV, typename T, bool UNIT = false>
__device__ __forceinline__ T chol_solve(const T (&L)[NV], T dinv, T b, int sl) {
  static_for<0, NV - 1>([&](auto kc) {      // column NV - 1 has no row below it: skipped
    constexpr int k = decltype(kc)::value;
    b = fma(-L[k], bcast<k>(UNIT ? b : b * dinv), b);
  });
  b *= dinv;
  // back substitution x_k = (y_k - sum_{i>k} L_ik x_i) / L_kk in blocks of BS columns, top block
  // first: the sums over the rows below the block are BS independent half-wave sums (their latencies
  // overlap), the block's own rows follow as a short chain of broadcasts of L_ik x_i from lane i
  // (block size A/B, fp64 configs[1] ms per launch: BS 1 0.726, 2 0.728, 3 0.731, 4 0.738,
  // 5 0.747; fp32: BS 2 0.424 vs 3 0.426, BS 1 within noise of 2)
  constexpr int BS = sizeof(T) == 8 ? 1 : 2;
  T x = 0;
  static_for<0, (NV + BS - 1) / BS>([&](auto bc) {
    constexpr int hi = NV - BS * decltype(bc)::value;        // block = columns [lo, hi)
    constexpr int lo = hi - BS > 0 ? hi - BS : 0;
    const int sl_k = opaque_v(sl);
    T ssum[BS];
    static_for<lo, hi>([&](auto cc) {
      constexpr int c = decltype(cc)::value;
      ssum[c - lo] = hsum(L[c] * x);                           // x = 0 on lanes < hi still
    });
    static_for<0, hi - lo>([&](auto tc) {
      constexpr int c = hi - 1 - decltype(tc)::value;         // top of the block down
      T xc = UNIT ? b - ssum[c - lo] : (b - ssum[c - lo]) * dinv;   // lane c's value is x_c
      x = (sl_k == c) ? xc : x;
      static_for<lo, c>([&](auto dc) {                       // lane c's L_cd x_c to the block's lanes d < c
        constexpr int d = decltype(dc)::value;
        ssum[d - lo] += bcast<c>(L[d] * x);
      });
    });
  });
  return x;
}
// forward substitution y = L^-1 b for G right-hand sides at once (sub-lane i holds b_i of each; the
// G broadcast chains are independent, so their latencies overlap); returns y_i in place (0 on
// sub-lanes >= NV, where dinv = 0)
template <int NV, int G, typename T>
__device__ __forceinline__ void chol_fwd_multi(const T (&L)[NV], T dinv, T (&b)[G], int sl) {
  static_for<0, NV - 1>([&](auto kc) {      // the last column changes no row: skipped
    constexpr int k = decltype(kc)::value;
    static_for<0, G>([&](auto gc) {
      constexpr int g = decltype(gc)::value;
      b[g] = fma(-L[k], bcast<k>(b[g] * dinv), b[g]);
    });
  });
  static_for<0, G>([&](auto gc) { b[decltype(gc)::value] *= dinv; });
}
template <int NV, typename T>
__device__ __forceinline__ T chol_fwd(const T (&L)[NV], T dinv, T b, int sl) {
  T bb[1] = {b};
  chol_fwd_multi<NV, 1>(L, dinv, bb, sl);
  return bb[0];
}
// Gauss-Jordan solve of an SPD system A x = b held row-per-lane (sub-lane i: row i in A[], b_i in b),
// without pivoting (SPD: positive pivot blocks), two pivots per LDS round trip -- the Newton direction
// of the HS_NEWTON_GJ A/B build (12 % fewer VALU instructions than chol_rows + chol_solve,
// 8 % slower: the kernel is latency-bound, and the solve needs the Hessian's upper triangle).  No
// substitutions: every other lane eliminates the pivot columns from its own row, rows above the pivots
// included.  Step s eliminates columns k = 2s, k + 1 with the 2 x 2 pivot
// block P (rows k, k + 1 of the current matrix; its trailing block is symmetric, but the two
// off-diagonal entries are used as computed, so every row's update is exact Gauss-Jordan):
//   (f0, f1) = (a_ik, a_i,k+1) P^-1,   a_ij -= f0 a_kj + f1 a_k+1,j  (j > k + 1),   b_i likewise.
// Rows k and k + 1 keep only their block at the end; each lane records its block's entries at its
// own step and takes its partner's right-hand side by DPP (lanes k, k + 1 are a quad pair): x from
// the 2 x 2 solve.  `buf` >= 64 T: row k at [0, NV), row k + 1 at [32, 32 + NV), their b at 28 / 60.
template <int NV, typename T>
__device__ __forceinline__ T gj_solve2(T (&A)[NV], T b, int sl, T* buf) {
  static_assert(NV + 1 <= 28, "two pivot rows + their b in 64 slots");
  using V2 = HIP_vector_type<T, 2>;
  T qd = T(0), qo = T(0), qr = T(0);     // own block: the other row's diagonal, own off-diagonal, 1 / det
  T dinv1 = T(0);                        // (a trailing single column, NV odd)
  static_for<0, NV / 2>([&](auto sc) {
    constexpr int k = 2 * decltype(sc)::value;
    const int sl_k = opaque_v(sl);
    const bool piv = sl_k == k || sl_k == k + 1;
    if (piv) {                           // lanes k, k + 1 publish their rows' columns >= k and b
      T* row = buf + (sl_k == k ? 0 : 32);
      static_for<k / 2, (NV + 1) / 2>([&](auto pc) {
        constexpr int p = decltype(pc)::value;
        if constexpr (2 * p + 1 < NV) *reinterpret_cast<V2*>(row + 2 * p) = V2(A[2 * p], A[2 * p + 1]);
        else row[2 * p] = A[2 * p];
      });
      *reinterpret_cast<V2*>(row + 28) = V2(b, T(0));
    }
    WSYNC();
    const V2 r0 = *reinterpret_cast<const V2*>(buf + k), r1 = *reinterpret_cast<const V2*>(buf + 32 + k);
    const T p00 = r0.x, p01 = r0.y, p10 = r1.x, p11 = r1.y;
    const T det = p00 * p11 - p01 * p10;
    const T rdet = recip(det > T(1e-30) ? det : T(1e-30));
    qd = (sl_k == k) ? p11 : (sl_k == k + 1) ? p00 : qd;
    qo = (sl_k == k) ? p01 : (sl_k == k + 1) ? p10 : qo;
    qr = piv ? rdet : qr;
    const T f0 = piv ? T(0) : (A[k] * p11 - A[k + 1] * p10) * rdet;
    const T f1 = piv ? T(0) : (A[k + 1] * p00 - A[k] * p01) * rdet;
    const T b0 = buf[28], b1 = buf[60];
    static_for<(k + 2) / 2, (NV + 1) / 2>([&](auto pc) {
      constexpr int p = decltype(pc)::value;
      if constexpr (2 * p + 1 < NV) {
        const V2 u = *reinterpret_cast<const V2*>(buf + 2 * p), w = *reinterpret_cast<const V2*>(buf + 32 + 2 * p);
        A[2 * p] = fma(-f1, w.x, fma(-f0, u.x, A[2 * p]));
        A[2 * p + 1] = fma(-f1, w.y, fma(-f0, u.y, A[2 * p + 1]));
      } else {
        A[2 * p] = fma(-f1, buf[32 + 2 * p], fma(-f0, buf[2 * p], A[2 * p]));
      }
    });
    b = fma(-f1, b1, fma(-f0, b0, b));
    WSYNC();
  });
  if constexpr (NV % 2 == 1) {           // the last column: a single pivot
    constexpr int k = NV - 1;
    const int sl_k = opaque_v(sl);
    const T piv = A[k] > T(1e-30) ? A[k] : T(1e-30);
    const T r = recip(piv);
    dinv1 = (sl_k == k) ? r : T(0);
    if (sl_k == k) *reinterpret_cast<V2*>(buf + 28) = V2(b, r);
    WSYNC();
    const V2 br = *reinterpret_cast<const V2*>(buf + 28);
    const T f = (sl_k == k) ? T(0) : A[k] * br.y;
    b = fma(-f, br.x, b);
    WSYNC();
  }
  const T bp = dpp<0xB1>(b);             // the pair partner's right-hand side (quad_perm [1,0,3,2])
  const int sl_e = opaque_v(sl);
  const T x2 = qr * (qd * b - qo * bp);
  return (NV % 2 == 1 && sl_e == NV - 1) ? b * dinv1 : x2;
}

// (A v)_i for a row-per-lane matrix and a vector in LDS (broadcast ds_reads)
template <int NV, typename T>
__device__ __forceinline__ T matvec_lds(const T (&A)[NV], const T* v) {
  T acc = 0;
  static_for<0, NV>([&](auto jc) {
    constexpr int j = decltype(jc)::value;
    acc = fma(A[j], v[j], acc);
  });
  return acc;
}

// ------------------------------------------------------------------ per-env LDS scratch
enum RowKind { RK_JLO = 0, RK_JHI = 1, RK_TLO = 2, RK_THI = 3, RK_CN = 4, RK_P0 = 5 };   // P0..P0+3: pyramid
__device__ __forceinline__ int rk_kind(int kid) { return kid >> 16; }
__device__ __forceinline__ int rk_id(int kid) { return kid & 0xffff; }

template <typename T, typename C>
struct Scratch {
  T qpos[MAXQ];
  T qvel[MAXDOF];
  T ctrl[MAXU];
  alignas(16) T vx[MAXDOF];   // generalized vector for J x; Cholesky column buffer
  T com[4];
  T cinert[MAXBODY][10];
  T cdof[MAXDOF][6];
  T cvel[MAXBODY][6];
  T con_pos[C::CON][3];
  T con_n[C::CON][3];
  T con_t1[C::CON][3];
  T con_dist[C::CON];
  T con_v[C::CON][3];
  T con_U[C::CON][6];
  T con_F[C::CON][3];
  int con_pair[C::CON];
  int con_adr[C::CON];
  uint32_t con_bb[C::CON];    // b1 | b2 << 8 | condim << 16 of the contact's pair (no model lookups per use)
  uint32_t con_m1[C::CON];    // dof chain masks of the contact's bodies (m1 = 0: world)
  uint32_t con_m2[C::CON];
  T con_mu[C::CON];
  uint32_t con_act[(C::CON + HL - 1) / HL];   // contacts with a nonzero force (contact_aggregates)
  uint16_t lim_row[MAXDOF];   // joint-limit rows of a dof: (lo row + 1) | (hi row + 1) << 8
  uint32_t dense_mask[C::RPL];   // rows added as dense rank-1 Hessian terms (tendons, body-body)
  int row_kid[C::EFC];
  T row_D[C::EFC];
  T row_f[C::EFC];
  int ncon, nefc, nlim, njl;   // njl: joint-limit rows (tendon rows are [njl, nlim))
  int niter;                   // this env's Newton iterations (the wave's loop runs for the slower env)
  struct Kin { T xpos[MAXBODY][3]; T xmat[MAXBODY][9]; T xquat[MAXBODY][4]; T xanchor[MAXJNT][3];
               T xaxis[MAXJNT][3]; T gpos[MAXGEOM][3]; T gax[MAXGEOM][3]; };
  union {   // phase-local arrays (aliased)
    Kin k;                                                        // kinematics + collision
    struct { T crb[MAXBODY][10]; T buf[MAXDOF][6]; } c;          // composite rigid body
    struct { T cdofdot[MAXDOF][6]; T cfrc[MAXBODY][6]; T csub[MAXBODY][6]; } r;   // RNE
    struct { T bvel[MAXBODY][6];                                  // J x mapping (rows, Newton)
             alignas(16) T cb[MAXDOF][2];                         // Cholesky column pairs / Gauss-Jordan pivot row
             union {
               struct { T cfrc[MAXBODY][6], linv[MAXBODY][3], mv[MAXBODY][3]; };   // full_state (after solve)
               alignas(16) T aug[MAXDOF][6];   // Newton: each dof's contact Hessian aggregate (upper triangle)
             }; } n;
    // fused rollout's policy forward (fp64 engine only: inside the union's 4 KB there; the fp32
    // engine's union is smaller and must not grow, so its member is a stub)
    struct { alignas(16) float x[sizeof(T) == 8 ? 512 : 4]; alignas(16) float h[sizeof(T) == 8 ? 256 : 4]; } pol;
  } u;
};

// PGS solver scratch (the <option solver="PGS"> kernel instance only; the Newton instance never
// allocates it).  With M = L L', row r's u_r = L^-1 J_r' (one nv-vector per row) gives the whole dual:
// AR = J M^-1 J' + R has AR_ik = u_i . u_k + R_i [i == k], and J_r qacc = u_r . (L' qacc).  Rows
// [0, NC) keep u_r in LDS (later rows rebuild it per use); every row keeps b_r = -aref_r, R_r, AR_rr,
// 1 / AR_rr and its lookahead Gram terms.
// Row sweep lookahead: row r's residual u_r . z is started PGS_LA rows early, on a z that still lacks the
// updates of rows r-PGS_LA .. r-1, and corrected with delta_{r-j} (u_r . u_{r-j}) when row r's turn
// comes (the Gram terms G_rj are computed once per substep).  The half-wave sum thus leaves the
// serial chain, which shrinks to a few scalar FMAs per row.
constexpr int PGS_LA = 3;
// cached rows: 40 in fp32 keep the resident PGS instance at 4 workgroups per CU; fp64 (48) runs at 2
template <typename T>
constexpr int pgs_cache_rows() { return sizeof(T) == 4 ? 40 : 48; }
template <typename T>
struct alignas(4 * sizeof(T)) PgsRow {
  T b, R, ar, ai;                 // -aref_r, R_r, AR_rr, 1 / max(AR_rr, MINVAL)
  T g[4];                         // G_rj = u_r . u_{r-j}, j = 1..PGS_LA (0 past the first row)
};
template <typename T, typename C>
struct PgsCache {
  static constexpr int NC = pgs_cache_rows<T>();
  T u[NC][MAXDOF];
  PgsRow<T> row[C::EFC];
};

// ------------------------------------------------------------------ narrow phase
template <typename T>
struct Con {
  T pos[3], n[3], t1[3], dist;
};

template <typename T>
__device__ __forceinline__ bool plane_sphere(const T* pp, const T* pn, const T* c, T r, Con<T>& o) {
  T d[3] = {c[0] - pp[0], c[1] - pp[1], c[2] - pp[2]};
  T cd = dot3(d, pn);
  if (cd > r) return false;
  o.dist = cd - r;
  for (int k = 0; k < 3; k++) { o.n[k] = pn[k]; o.pos[k] = c[k] - pn[k] * (o.dist * T(0.5) + r); o.t1[k] = 0; }
  return true;
}
template <typename T>
__device__ __forceinline__ bool sphere_sphere(const T* p1, T r1, const T* p2, T r2, Con<T>& o) {
  T d[3] = {p2[0] - p1[0], p2[1] - p1[1], p2[2] - p1[2]};
  T len = sqrt(dot3(d, d));
  T dist = len - r1 - r2;
  if (dist > 0) return false;
  o.dist = dist;
  if (len < T(1e-15)) { o.n[0] = 1; o.n[1] = 0; o.n[2] = 0; }
  else { T i = recip(len); for (int k = 0; k < 3; k++) o.n[k] = d[k] * i; }
  for (int k = 0; k < 3; k++) { o.pos[k] = p1[k] + o.n[k] * (r1 + dist * T(0.5)); o.t1[k] = 0; }
  return true;
}
// mju_makeFrame: complete (n, t1 hint) -> orthonormal t1
template <typename T>
__device__ __forceinline__ void make_frame(Con<T>& c) {
  normalize3(c.n);
  if (sqrt(dot3(c.t1, c.t1)) < T(0.5)) {
    if (fabs(c.n[1]) < T(0.5)) { c.t1[0] = 0; c.t1[1] = 1; c.t1[2] = 0; }
    else { c.t1[0] = 0; c.t1[1] = 0; c.t1[2] = 1; }
  }
  T d = dot3(c.n, c.t1);
  for (int k = 0; k < 3; k++) c.t1[k] -= c.n[k] * d;
  normalize3(c.t1);
}

// number of contacts (0..2) for static pair p (mjc_* primitives)
template <typename T, typename C>
__device__ __forceinline__ int collide_pair(const Scratch<T, C>& s, const int4 info, const T (&sz)[4], Con<T>& c0,
                                           Con<T>& c1) {
  const int g1 = info.x, g2 = info.y, fn = info.z;
  const T* p1 = s.u.k.gpos[g1];
  const T* p2 = s.u.k.gpos[g2];
  const T* a1 = s.u.k.gax[g1];
  const T* a2 = s.u.k.gax[g2];
  const T r1 = sz[0], h1 = sz[1], r2 = sz[2], h2 = sz[3];
  int n = 0;
  if (fn >= PAIR_SPHERE_SPHERE) {
    // bounding spheres (radius + half-length, MuJoCo's geom_rbound) apart: no contact.  Exact (a
    // contact needs dist <= 0 between the geoms, inside both bounds), so only a shortcut -- and when
    // no lane of the wave holds a near pair, the wave skips the capsule-capsule branch altogether
    const T d[3] = {p1[0] - p2[0], p1[1] - p2[1], p1[2] - p2[2]};
    const T R = r1 + h1 + r2 + h2;
    if (dot3(d, d) > R * R) return 0;
  }
  if (fn == PAIR_PLANE_SPHERE) {
    n = plane_sphere(p1, a1, p2, r2, c0) ? 1 : 0;
  } else if (fn == PAIR_PLANE_CAPSULE) {
    T e[3];
    for (int k = 0; k < 3; k++) e[k] = p2[k] + h2 * a2[k];
    Con<T> t;
    if (plane_sphere(p1, a1, e, r2, t)) { for (int k = 0; k < 3; k++) t.t1[k] = a2[k]; c0 = t; n = 1; }
    for (int k = 0; k < 3; k++) e[k] = p2[k] - h2 * a2[k];
    if (plane_sphere(p1, a1, e, r2, t)) {
      for (int k = 0; k < 3; k++) t.t1[k] = a2[k];
      if (n == 0) c0 = t; else c1 = t;
      n++;
    }
  } else if (fn == PAIR_SPHERE_SPHERE) {
    n = sphere_sphere(p1, r1, p2, r2, c0) ? 1 : 0;
  } else if (fn == PAIR_SPHERE_CAPSULE) {
    T d[3] = {p1[0] - p2[0], p1[1] - p2[1], p1[2] - p2[2]};
    T x = dot3(a2, d);
    x = x > h2 ? h2 : (x < -h2 ? -h2 : x);
    T v[3] = {p2[0] + x * a2[0], p2[1] + x * a2[1], p2[2] + x * a2[2]};
    n = sphere_sphere(p1, r1, v, r2, c0) ? 1 : 0;
  } else {   // capsule-capsule (mjc_CapsuleCapsule)
    T ax1[3] = {a1[0] * h1, a1[1] * h1, a1[2] * h1}, ax2[3] = {a2[0] * h2, a2[1] * h2, a2[2] * h2};
    T dif[3] = {p1[0] - p2[0], p1[1] - p2[1], p1[2] - p2[2]};
    T ma = dot3(ax1, ax1), mb = -dot3(ax1, ax2), mc = dot3(ax2, ax2), u = -dot3(ax1, dif), v = dot3(ax2, dif);
    T det = ma * mc - mb * mb;
    T v1[3], v2[3];
    if (fabs(det) >= T(1e-15)) {
      T x1 = (mc * u - mb * v) / det, x2 = (ma * v - mb * u) / det;
      if (x1 > 1) { x1 = 1; x2 = (v - mb) / mc; }
      else if (x1 < -1) { x1 = -1; x2 = (v + mb) / mc; }
      if (x2 > 1) { x2 = 1; x1 = (u - mb) / ma; x1 = x1 > 1 ? 1 : (x1 < -1 ? -1 : x1); }
      else if (x2 < -1) { x2 = -1; x1 = (u + mb) / ma; x1 = x1 > 1 ? 1 : (x1 < -1 ? -1 : x1); }
      for (int k = 0; k < 3; k++) { v1[k] = p1[k] + x1 * ax1[k]; v2[k] = p2[k] + x2 * ax2[k]; }
      n = sphere_sphere(v1, r1, v2, r2, c0) ? 1 : 0;
    } else {
      for (int side = 1; side >= -1; side -= 2) {
        T x2 = (v - side * mb) / mc;
        x2 = x2 > 1 ? 1 : (x2 < -1 ? -1 : x2);
        for (int k = 0; k < 3; k++) { v1[k] = p1[k] + side * ax1[k]; v2[k] = p2[k] + x2 * ax2[k]; }
        Con<T> t;
        if (sphere_sphere(v1, r1, v2, r2, t)) { if (n == 0) c0 = t; else c1 = t; n++; }
      }
    }
  }
  if (n > 0) make_frame(c0);
  if (n > 1) make_frame(c1);
  return n;
}

template <typename T, typename C>
__device__ __forceinline__ void store_contact(MPtr<T> m, Scratch<T, C>& s, int slot, const Con<T>& c, int p) {
  if (slot >= C::CON) return;
  for (int k = 0; k < 3; k++) { s.con_pos[slot][k] = c.pos[k]; s.con_n[slot][k] = c.n[k]; s.con_t1[slot][k] = c.t1[k]; }
  s.con_dist[slot] = c.dist;
  s.con_pair[slot] = p;
  const int b1 = m->pair_b1[p], b2 = m->pair_b2[p];
  s.con_bb[slot] = (uint32_t)b1 | (uint32_t)b2 << 8 | (uint32_t)m->pair_dim[p] << 16;
  s.con_m1[slot] = b1 ? m->body_chainmask[b1] : 0u;
  s.con_m2[slot] = m->body_chainmask[b2];
  s.con_mu[slot] = m->pair_mu[p];
}

// impedance (mj_makeImpedance getimpedance), MuJoCo clamps d0/dmax to [1e-4, 0.9999].  The sigmoid
// y = x^p / mid^(p-1) (x <= mid) or 1 - (1-x)^p / (1-mid)^(p-1) takes its constant denominators from
// the model (si[5..7], fill_solimp) and one pow, skipped for the default power 2.
template <typename T>
__device__ __forceinline__ T impedance(CPtr<T> si, T pos, T margin) {
  T s0 = fmin(T(0.9999), fmax(T(0.0001), si[0])), s1 = fmin(T(0.9999), fmax(T(0.0001), si[1]));
  if (s0 == s1 || si[2] <= T(1e-15)) return T(0.5) * (s0 + s1);
  T x = (pos - margin) * si[5];
  if (x < 0) x = -x;
  if (x >= 1 || x <= 0) return x >= 1 ? s1 : s0;
  const T p = si[4];
  T y = x;
  if (p != T(1)) {
    const bool lo = x <= si[3];
    const T base = lo ? x : 1 - x;
    T pw = base * base;
    if (p != T(2)) pw = pow(base, p);
    y = lo ? pw * si[6] : 1 - pw * si[7];
  }
  return s0 + y * (s1 - s0);
}

// ------------------------------------------------------------------ J x for all rows
// s.vx (generalized vector) -> body spatial velocities -> contact frame velocities
// ch: this body lane's dof chain mask (body_chainmask, 0 for the world), loaded by the caller
template <typename T>
__device__ __forceinline__ uint32_t chain_mask(MPtr<T> m, int sl, int nb) {
  return (sl > 0 && sl < nb) ? m->body_chainmask[sl] : 0u;
}
template <int NV, typename T, typename C>
__device__ __forceinline__ void map_vx(Scratch<T, C>& s, int sl, int nb, uint32_t ch) {
  if (sl < nb) {   // body spatial velocity = sum over the body's dof chain of cdof_j x_j
    T v[6] = {0, 0, 0, 0, 0, 0};
    // the chain's dofs only, ascending: the same sum as over all dofs (the skipped terms are exact
    // zeros), ~half the fp64 FMAs (fp64 0.866 -> 0.812 ms per launch)
    for_bits<T>(ch, [&](int j) { ValsX<T, 6> r; r.x = s.vx[j]; for (int k = 0; k < 6; k++) r.v[k] = s.cdof[j][k]; return r; },
                [&](int, const ValsX<T, 6>& r) {
#pragma unroll
                  for (int k = 0; k < 6; k++) v[k] = fma(r.v[k], r.x, v[k]);
                });
    for (int k = 0; k < 6; k++) s.u.n.bvel[sl][k] = v[k];
  }
  WSYNC();
#pragma unroll
  for (int cs = 0; cs < C::CON; cs += HL) {   // contact slots of this lane (one per lane in the resident tier)
    const int c = cs + sl;
    if (c < s.ncon) {
      const uint32_t bb = s.con_bb[c];
      const int b1 = bb & 0xff, b2 = (bb >> 8) & 0xff;
      T r[3] = {s.con_pos[c][0] - s.com[0], s.con_pos[c][1] - s.com[1], s.con_pos[c][2] - s.com[2]};
      T w[3], v1[3], v2[3];
      cross3(s.u.n.bvel[b2], r, w);
      for (int k = 0; k < 3; k++) v2[k] = s.u.n.bvel[b2][3 + k] + w[k];
      cross3(s.u.n.bvel[b1], r, w);
      for (int k = 0; k < 3; k++) v1[k] = s.u.n.bvel[b1][3 + k] + w[k];
      T dv[3] = {v2[0] - v1[0], v2[1] - v1[1], v2[2] - v1[2]};
      T t2[3];
      cross3(s.con_n[c], s.con_t1[c], t2);
      s.con_v[c][0] = dot3(s.con_n[c], dv);
      s.con_v[c][1] = dot3(s.con_t1[c], dv);
      s.con_v[c][2] = dot3(t2, dv);
    }
  }
  WSYNC();
}

// Row descriptor kept in registers by the row's lane for the whole solve (no LDS / model
// lookups per use): desc = kind << 16 | j with j = dof (joint limits), tendon id or contact id;
// coef = +-1 (limits), +-mu (pyramid rows), 0 (frictionless contact normal).
template <typename T, typename C>
__device__ __forceinline__ T row_Jx(MPtr<T> m, const Scratch<T, C>& s, int desc, T coef) {
  int kind = rk_kind(desc), j = rk_id(desc);
  if (kind <= RK_JHI) return coef * s.vx[j];
  if (kind <= RK_THI) {
    T v = 0;
    for (int w = 0; w < m->ten_nwrap[j]; w++) v += m->ten_wrapcoef[j][w] * s.vx[m->ten_wrapdof[j][w]];
    return coef * v;
  }
  int comp = kind == RK_CN ? 1 : 1 + ((kind - RK_P0) >> 1);
  return s.con_v[j][0] + coef * s.con_v[j][comp];
}

// world-frame force direction u of a contact row
template <typename T, typename C>
__device__ __forceinline__ void row_u(MPtr<T> m, const Scratch<T, C>& s, int kind, int c, T* u) {
  if (kind == RK_CN) { for (int k = 0; k < 3; k++) u[k] = s.con_n[c][k]; return; }
  int sub = kind - RK_P0;
  T mu = s.con_mu[c];
  T sg = (sub & 1) ? -mu : mu;
  T t[3];
  if (sub >> 1) cross3(s.con_n[c], s.con_t1[c], t);
  else { t[0] = s.con_t1[c][0]; t[1] = s.con_t1[c][1]; t[2] = s.con_t1[c][2]; }
  for (int k = 0; k < 3; k++) u[k] = s.con_n[c][k] + sg * t[k];
}

// per-contact aggregates from current row forces: U = sum D u u' (active rows), F = sum f u
// and the mask of contacts whose force is nonzero (the others add exact zeros to J'f and the Newton
// Hessian, so those loops skip them)
template <typename T, typename C>
__device__ __forceinline__ void contact_aggregates(MPtr<T> m, Scratch<T, C>& s, int sl) {
  const bool up = threadIdx.x >= HL;
#pragma unroll
  for (int cs = 0; cs < C::CON; cs += HL) {
    const int c = cs + sl;
    bool act = false;
    if (c < s.ncon) {
      int adr = s.con_adr[c];
      int nr = (s.con_bb[c] >> 16) == 1 ? 1 : 4;
      T U[6] = {0, 0, 0, 0, 0, 0}, F[3] = {0, 0, 0};
      // straight-line over the (at most 4) rows: every LDS operand is read up front (one round trip),
      // then the same sums in the same order as the row loop below
      const bool pyr = nr == 4;
      T f4[4], D4[4], nn[3], t1[3], t2[3];
#pragma unroll
      for (int q = 0; q < 4; q++) {
        const bool on = q == 0 || pyr;
        f4[q] = on ? s.row_f[adr + q] : T(0);
        D4[q] = on ? s.row_D[adr + q] : T(0);
      }
      for (int k = 0; k < 3; k++) { nn[k] = s.con_n[c][k]; t1[k] = s.con_t1[c][k]; }
      const T mu = s.con_mu[c];
      cross3(nn, t1, t2);
#pragma unroll
      for (int q = 0; q < 4; q++) {
        const T f = f4[q];
        if (f != T(0)) {
          T u[3];
          if (!pyr) {
            for (int k = 0; k < 3; k++) u[k] = nn[k];
          } else {
            const T sg = (q & 1) ? -mu : mu;
            for (int k = 0; k < 3; k++) u[k] = nn[k] + sg * ((q >> 1) ? t2[k] : t1[k]);
          }
          const T D = D4[q];
          U[0] += D * u[0] * u[0]; U[1] += D * u[1] * u[1]; U[2] += D * u[2] * u[2];
          U[3] += D * u[0] * u[1]; U[4] += D * u[0] * u[2]; U[5] += D * u[1] * u[2];
          for (int k = 0; k < 3; k++) F[k] += f * u[k];
        }
      }
      for (int k = 0; k < 6; k++) s.con_U[c][k] = U[k];
      for (int k = 0; k < 3; k++) s.con_F[c][k] = F[k];
      act = F[0] != T(0) || F[1] != T(0) || F[2] != T(0) || U[0] != T(0) || U[1] != T(0) || U[2] != T(0);
    }
    const uint32_t mk = hballot(act, up);
    if (sl == 0) s.con_act[cs / HL] = mk;
  }
  WSYNC();
}
// for each contact c with a nonzero force, in contact order: f(c)
template <typename C, typename F>
__device__ __forceinline__ void for_active_contacts(const uint32_t* act, F&& f) {
#pragma unroll
  for (int w = 0; w < (C::CON + HL - 1) / HL; w++)
    for (uint32_t mk = act[w]; mk; mk &= mk - 1u) f(w * HL + __builtin_ctz(mk));
}

// the same with every per-contact LDS operand read by ld(c) in one batch (one round trip per
// contact instead of a read, a branch on it and dependent reads; HS_CONTACT_FLAT) and the next
// contact's reads issued before the current contact's arithmetic (HS_CONTACT_AHEAD): J'f and the
// Hessian's contact terms.  A/B, fp64 ms per configs[1] launch: 0.635 -> flat 0.634 -> + ahead 0.632.
template <typename T, typename C, typename LD, typename F>
__device__ __forceinline__ void for_active_contacts_ld(const uint32_t* act, LD&& ld, F&& f) {
#pragma unroll
  for (int w = 0; w < (C::CON + HL - 1) / HL; w++)
    for_bits<T, true>(
        act[w], [&](int j) { return ld(w * HL + j); }, [&](int j, const auto& v) { f(w * HL + j, v); });
}

// (J' f)_i for dof sub-lane i (contacts via point Jacobians, joint limits via the dof's
// limit-row slots, tendon limits via rows [njl, nlim))
template <typename T, typename C>
__device__ __forceinline__ T jtf_lane(MPtr<T> m, const Scratch<T, C>& s, int sl, const T* cd) {
  T acc = 0;
  struct CV { uint32_t m1, m2; T p[3], f[3]; };
  for_active_contacts_ld<T, C>(s.con_act, [&](int c) {
    CV v;
    v.m1 = s.con_m1[c]; v.m2 = s.con_m2[c];
    for (int k = 0; k < 3; k++) { v.p[k] = s.con_pos[c][k]; v.f[k] = s.con_F[c][k]; }
    return v;
  }, [&](int, const CV& v) {
    const int in2 = bit(v.m2, sl), in1 = bit(v.m1, sl);
    if (in1 != in2) {
      T r[3] = {v.p[0] - s.com[0], v.p[1] - s.com[1], v.p[2] - s.com[2]};
      T w[3];
      cross3(cd, r, w);
      T jp[3] = {cd[3] + w[0], cd[4] + w[1], cd[5] + w[2]};
      T x = dot3(jp, v.f);
      acc += in2 ? x : -x;
    }
  });
  if (sl < MAXDOF) {
    int lr = s.lim_row[sl];
    int lo = (lr & 0xff) - 1, hi = (lr >> 8) - 1;
    if (lo >= 0) acc += s.row_f[lo];
    if (hi >= 0) acc -= s.row_f[hi];
  }
  for (int r = s.njl; r < s.nlim; r++) {
    int id = rk_id(s.row_kid[r]);
    T f = rk_kind(s.row_kid[r]) == RK_TLO ? s.row_f[r] : -s.row_f[r];
    for (int w = 0; w < m->ten_nwrap[id]; w++)
      if (m->ten_wrapdof[id][w] == sl) acc += f * m->ten_wrapcoef[id][w];
  }
  return acc;
}

// ------------------------------------------------------------------ diagnostic phase timing
// Built only with -DHS_TIMING (libhsim_timing.so): s_memtime stamps accumulated per phase,
// summed over waves into dbg[8000 + slot].  The product build compiles them out.
#ifdef HS_TIMING
constexpr int NSLOT = 29;
struct PhaseClock {
  uint64_t acc[NSLOT] = {0};
  uint64_t prev = 0, t0 = 0, rt0 = 0;   // rt0: s_memrealtime (100 MHz, one clock for all XCDs)
  __device__ __forceinline__ void start() { prev = t0 = __builtin_amdgcn_s_memtime(); rt0 = __builtin_amdgcn_s_memrealtime(); }
  __device__ __forceinline__ void stamp(int slot) {
    uint64_t now = __builtin_amdgcn_s_memtime();
    uint64_t d = now - prev;
    asm volatile("" : "+v"(d));   // accumulate in VGPRs (stamps sit in divergent regions too)
    acc[slot] += d;
    prev = now;
  }
};
#define HS_STAMP(clk, slot) (clk).stamp(slot)
// flushed once, inside the substep loop at its exits: a per-lane accumulator live past the loop
// trips an isel bug ("illegal VGPR to SGPR copy") in this compiler
#define HS_FLUSH()                                                                              \
  do {                                                                                           \
    T* dbg_ = opaque(ka)->b.dbg;                                                                 \
    if (dbg_ && !WIDE) {                                                                         \
      if (sl == 0)                                                                               \
        for (int q = 0; q < NSLOT; q++) { atomicAdd(&dbg_[8000 + q], (T)st.clk.acc[q]); st.clk.acc[q] = 0; } \
      if (sl == 0) atomicAdd(&dbg_[8030], (T)tot_iter);                                          \
      if (lane == 0 && blockIdx.x < 2048) dbg_[9000 + blockIdx.x] = (T)(st.clk.prev - st.clk.t0);  \
      if (lane == 0 && blockIdx.x < 2048) {                                                      \
        dbg_[16384 + blockIdx.x] = (T)(uint32_t)(st.clk.rt0 & 0xFFFFFFu);                          \
        dbg_[18432 + blockIdx.x] = (T)(uint32_t)(__builtin_amdgcn_s_memrealtime() & 0xFFFFFFu);    \
      }                                                                                          \
      if (sl == 0 && blockIdx.x < 2048) dbg_[11100 + 2 * blockIdx.x + (up ? 1 : 0)] = (T)tot_iter;  \
      if (lane == 0 && titem >= 0 && titem < 4096) {   /* queued items: realtime start / end */  \
        dbg_[20480 + 2 * titem] = (T)(uint32_t)(st.clk.rt0 & 0xFFFFFFu);                            \
        dbg_[20480 + 2 * titem + 1] = (T)(uint32_t)(__builtin_amdgcn_s_memrealtime() & 0xFFFFFFu);  \
      }                                                                                          \
      tot_iter = 0;                                                                              \
    }                                                                                            \
  } while (0)
#else
#define HS_FLUSH() ((void)0)
struct PhaseClock {
  __device__ __forceinline__ void start() {}
  __device__ __forceinline__ void stamp(int) {}
};
#define HS_STAMP(clk, slot) ((void)0)
#endif

// ------------------------------------------------------------------ one mj_step (per half-wave)
template <typename T, int NV, typename C>
struct Stepper {
  PhaseClock clk;
  MPtr<T> m;
  Scratch<T, C>& s;
  int sl, nb;
  bool up;        // upper half-wave (second env of the wave)
  T cd[6];        // cdof of this sub-lane's dof (registers)
  T Mr[NV];       // mass-matrix row of this sub-lane's dof
  T fsmooth;      // qfrc_smooth_i
  T fcon;         // qfrc_constraint_i
  T qacc;         // solver output qacc_i
  T qfa;          // qfrc_actuator_i (obs / kneeling reward)
  T damp;         // dof_damping_i, loaded with the constraint rows (Euler reads it)
  int niter;
  T* dbg = nullptr;   // stage-dump target (env 0 in debug mode only)

  __device__ Stepper(MPtr<T> mm, Scratch<T, C>& ss, int lane)
      : m(mm), s(ss), sl(lane & (HL - 1)), nb(mm->nbody), up(lane >= HL) {}

  // The Newton iterations rebuild H and factor it every time.  MuJoCo's rank-1 updates of the factor
  // (mju_cholUpdate) were built and measured slower on MI355X (DESIGN.md 3.1 "Incremental factor"):
  // each update is a serial 27-column chain, and the extra live state costs the queue kernel its last
  // registers.
  // the Newton factor as L D L' in the fp64 engine (unit lower L): the same elimination, but the
  // triangular solves lose one dependent multiply per column (fp64 0.740 -> 0.731 ms per configs[1]
  // launch; the Euler factorization and the fp32 engine measured the same either way and stay L L').
  static constexpr bool LDLF = sizeof(T) == 8;
  static constexpr bool LDLE = false;
  // the launch arguments (every step-kernel instance takes its KArgs at kernarg offset 0)
  __device__ __forceinline__ static KPtr<T> kargs() { return (KPtr<T>)__builtin_amdgcn_kernarg_segment_ptr(); }

  // start of a pipeline phase: nothing lane-invariant is carried over from the previous phase
  __device__ __forceinline__ void phase_begin() {
    m = opaque(m);
    sl = opaque_v(sl);
  }

  // mj_kinematics + mj_comPos
  __device__ __forceinline__ void kinematics() {
    phase_begin();
    if (sl == 0) {
      for (int k = 0; k < 3; k++) s.u.k.xpos[0][k] = 0;
      s.u.k.xquat[0][0] = 1; s.u.k.xquat[0][1] = s.u.k.xquat[0][2] = s.u.k.xquat[0][3] = 0;
      for (int k = 0; k < 9; k++) s.u.k.xmat[0][k] = (k % 4 == 0) ? T(1) : T(0);
    }
    // mj_kinematics, split so the serial level loop carries one frame composition per level:
    // (1) in parallel over bodies, the body's transform RELATIVE TO ITS PARENT (body_pos/quat
    //     followed by its hinges, each rotating about jnt_pos: p' = a - R(q qloc) jpos with the
    //     anchor a = p + R(q) jpos) and each hinge's anchor/axis in the parent frame;
    // (2) level by level: xquat = normalize(xquat_par * q_loc), xpos = xpos_par + xmat_par p_loc;
    // (3) in parallel again: xanchor = xpos_par + xmat_par a_loc, xaxis = xmat_par ax_loc.
    // Mathematically identical to MuJoCo's per-joint world-frame recursion (rounding differs).
    const int b = sl;
    const bool isb = b > 0 && b < nb;
    int depth = -1, par = 0, ja = 0, jn = 0, fqa = 0;
    bool isfree = false;
    T pl[3] = {0, 0, 0}, ql[4] = {1, 0, 0, 0};
    T anl[MAXJPB][3], axl[MAXJPB][3];
    if (isb) {
      depth = m->body_depth[b];
      par = m->body_parentid[b];
      ja = m->body_jntadr[b];
      jn = m->body_jntnum[b];
      isfree = jn == 1 && m->jnt_type[ja] == JNT_FREE;
      fqa = m->jnt_qposadr[ja];
      for (int k = 0; k < 3; k++) pl[k] = m->body_pos[b][k];
      for (int k = 0; k < 4; k++) ql[k] = m->body_quat[b][k];
    }
    if (isfree) {
      for (int k = 0; k < 3; k++) pl[k] = s.qpos[fqa + k];
      for (int k = 0; k < 4; k++) ql[k] = s.qpos[fqa + 3 + k];
    }
#pragma unroll
    for (int jj = 0; jj < MAXJPB; jj++) {
      const bool use = isb && !isfree && jj < jn;
      const int j = use ? ja + jj : 0;
      T jp[3], jx[3], ang = 0;
      for (int k = 0; k < 3; k++) { jp[k] = use ? m->jnt_pos[j][k] : T(0); jx[k] = use ? m->jnt_axis[j][k] : T(0); }
      if (use) {
        int qa = m->jnt_qposadr[j];
        ang = s.qpos[qa] - m->qpos0[qa];
      }
      T sn, cs;
      sincos_t(T(0.5) * ang, sn, cs);
      const T jr[4] = {cs, jx[0] * sn, jx[1] * sn, jx[2] * sn};
      T R[9];
      quat2mat(ql, R);
      mv3(R, jx, axl[jj]);
      mv3(R, jp, anl[jj]);
      for (int k = 0; k < 3; k++) anl[jj][k] += pl[k];
      if (use) {
        mulq(ql, jr, ql);
        quat2mat(ql, R);
        T v[3];
        mv3(R, jp, v);
        for (int k = 0; k < 3; k++) pl[k] = anl[jj][k] - v[k];
      }
    }
    WSYNC();
    for (int L = 1; L <= m->nlevel; L++) {
      if (depth == L) {
        T pos[3], q[4];
        if (isfree) {   // parent is the world: the free joint's qpos is the world frame
          for (int k = 0; k < 3; k++) pos[k] = pl[k];
          for (int k = 0; k < 4; k++) q[k] = ql[k];
        } else {
          mv3(s.u.k.xmat[par], pl, pos);
          for (int k = 0; k < 3; k++) pos[k] += s.u.k.xpos[par][k];
          T pq[4] = {s.u.k.xquat[par][0], s.u.k.xquat[par][1], s.u.k.xquat[par][2], s.u.k.xquat[par][3]};
          mulq(pq, ql, q);
        }
        normalize4(q);
        for (int k = 0; k < 4; k++) s.u.k.xquat[b][k] = q[k];
        for (int k = 0; k < 3; k++) s.u.k.xpos[b][k] = pos[k];
        quat2mat(q, s.u.k.xmat[b]);
      }
      WSYNC();
    }
    if (isb) {
      if (isfree) {
        for (int k = 0; k < 3; k++) { s.u.k.xanchor[ja][k] = s.u.k.xpos[b][k]; s.u.k.xaxis[ja][k] = m->jnt_axis[ja][k]; }
      } else {
        const T* Rp = s.u.k.xmat[par];
        const T* xp = s.u.k.xpos[par];
#pragma unroll
        for (int jj = 0; jj < MAXJPB; jj++) {
          if (jj < jn) {
            T an[3], ax[3];
            mv3(Rp, anl[jj], an);
            mv3(Rp, axl[jj], ax);
            for (int k = 0; k < 3; k++) { s.u.k.xanchor[ja + jj][k] = xp[k] + an[k]; s.u.k.xaxis[ja + jj][k] = ax[k]; }
          }
        }
      }
    }
    if (sl < m->ngeom) {
      int g = sl, gb = m->geom_bodyid[g];
      T gp[3] = {m->geom_pos[g][0], m->geom_pos[g][1], m->geom_pos[g][2]};
      T gz[3] = {m->geom_zaxis[g][0], m->geom_zaxis[g][1], m->geom_zaxis[g][2]};
      T w[3];
      mv3(s.u.k.xmat[gb], gp, w);
      for (int k = 0; k < 3; k++) s.u.k.gpos[g][k] = s.u.k.xpos[gb][k] + w[k];
      mv3(s.u.k.xmat[gb], gz, s.u.k.gax[g]);
    }
    T mx = 0, my = 0, mz = 0, xi[3] = {0, 0, 0};
    if (b > 0 && b < nb) {
      T ip[3] = {m->body_ipos[b][0], m->body_ipos[b][1], m->body_ipos[b][2]}, w[3];
      mv3(s.u.k.xmat[b], ip, w);
      for (int k = 0; k < 3; k++) xi[k] = s.u.k.xpos[b][k] + w[k];
      T mb = m->body_mass[b];
      mx = mb * xi[0]; my = mb * xi[1]; mz = mb * xi[2];
    }
    // mj_comPos: single kinematic tree -> subtree_com[root] == subtree_com[0] == whole-model COM
    T inv = T(1) / m->total_mass;
    T c0 = hsum(mx) * inv, c1 = hsum(my) * inv, c2 = hsum(mz) * inv;
    if (sl == 0) { s.com[0] = c0; s.com[1] = c1; s.com[2] = c2; }
    if (b > 0 && b < nb) {   // cinert (mju_inertCom)
      const T* R = s.u.k.xmat[b];
      CPtr<T> I6 = m->body_inert[b];
      T I[9] = {I6[0], I6[3], I6[4], I6[3], I6[1], I6[5], I6[4], I6[5], I6[2]};
      T A[9];
      for (int r = 0; r < 3; r++)
        for (int c = 0; c < 3; c++) A[3 * r + c] = R[3 * r] * I[c] + R[3 * r + 1] * I[3 + c] + R[3 * r + 2] * I[6 + c];
      T Ic[6];
      Ic[0] = A[0] * R[0] + A[1] * R[1] + A[2] * R[2];
      Ic[1] = A[3] * R[3] + A[4] * R[4] + A[5] * R[5];
      Ic[2] = A[6] * R[6] + A[7] * R[7] + A[8] * R[8];
      Ic[3] = A[0] * R[3] + A[1] * R[4] + A[2] * R[5];
      Ic[4] = A[0] * R[6] + A[1] * R[7] + A[2] * R[8];
      Ic[5] = A[3] * R[6] + A[4] * R[7] + A[5] * R[8];
      T d[3] = {xi[0] - c0, xi[1] - c1, xi[2] - c2};
      T mass = m->body_mass[b];
      T* ci = s.cinert[b];
      ci[0] = Ic[0] + mass * (d[1] * d[1] + d[2] * d[2]);
      ci[1] = Ic[1] + mass * (d[0] * d[0] + d[2] * d[2]);
      ci[2] = Ic[2] + mass * (d[0] * d[0] + d[1] * d[1]);
      ci[3] = Ic[3] - mass * d[0] * d[1];
      ci[4] = Ic[4] - mass * d[0] * d[2];
      ci[5] = Ic[5] - mass * d[1] * d[2];
      ci[6] = mass * d[0]; ci[7] = mass * d[1]; ci[8] = mass * d[2]; ci[9] = mass;
    }
    if (sl == 0)
      for (int k = 0; k < 10; k++) s.cinert[0][k] = 0;
    for (int k = 0; k < 6; k++) cd[k] = 0;
    if (sl < NV) {   // cdof (mju_dofCom)
      int j = m->dof_jntid[sl], db = m->dof_bodyid[sl];
      T off[3] = {c0 - s.u.k.xanchor[j][0], c1 - s.u.k.xanchor[j][1], c2 - s.u.k.xanchor[j][2]};
      T ax[3];
      bool lin = false;
      if (m->jnt_type[j] == JNT_FREE) {
        int k = sl - m->jnt_dofadr[j];
        if (k < 3) {   // no dynamic indexing of register arrays (it would demote the Stepper to scratch)
          lin = true;
          cd[3] = k == 0 ? T(1) : T(0); cd[4] = k == 1 ? T(1) : T(0); cd[5] = k == 2 ? T(1) : T(0);
        } else {
          int c = k - 3;
          ax[0] = s.u.k.xmat[db][c]; ax[1] = s.u.k.xmat[db][3 + c]; ax[2] = s.u.k.xmat[db][6 + c];
        }
      } else {
        ax[0] = s.u.k.xaxis[j][0]; ax[1] = s.u.k.xaxis[j][1]; ax[2] = s.u.k.xaxis[j][2];
      }
      if (!lin) {
        cd[0] = ax[0]; cd[1] = ax[1]; cd[2] = ax[2];
        cross3(ax, off, cd + 3);
      }
      for (int k = 0; k < 6; k++) s.cdof[sl][k] = cd[k];
    }
    WSYNC();
    if (dbg)    // stage dump (env 0, debug mode): xpos is phase-local, so dump it here
      for (int k = sl; k < MAXBODY * 3; k += HL) dbg[k] = s.u.k.xpos[k / 3][k % 3];
  }

  // mj_collision: one static pair per sub-lane per pass, ordered compaction into contacts
  __device__ __forceinline__ int collision() {
    phase_begin();
    int ncon = 0;
    const int npair = m->npair;
    // the next pass's pair records are loaded while this pass runs (their L1/L2 latency is otherwise
    // exposed at the top of every pass: one wave per SIMD in fp64)
    int4 info_n = make_int4(0, 0, 0, 0);
    T sz_n[4] = {0, 0, 0, 0};
    if (sl < npair) {
      info_n = make_int4(m->pair_info[sl][0], m->pair_info[sl][1], m->pair_info[sl][2], m->pair_info[sl][3]);
      for (int k = 0; k < 4; k++) sz_n[k] = m->pair_size[sl][k];
    }
    for (int base = 0; base < npair; base += HL) {
      int p = base + sl;
      Con<T> c0, c1;
      int n = 0;
      const int4 info = info_n;
      T sz[4] = {sz_n[0], sz_n[1], sz_n[2], sz_n[3]};
      if (p + HL < npair) {
        info_n = make_int4(m->pair_info[p + HL][0], m->pair_info[p + HL][1], m->pair_info[p + HL][2],
                           m->pair_info[p + HL][3]);
        for (int k = 0; k < 4; k++) sz_n[k] = m->pair_size[p + HL][k];
      }
      if (p < npair) n = collide_pair(s, info, sz, c0, c1);
      uint32_t m1 = hballot(n >= 1, up), m2 = hballot(n >= 2, up);
      int pre = below(m1, sl) + below(m2, sl);
      if (n >= 1) store_contact(m, s, ncon + pre, c0, p);
      if (n >= 2) store_contact(m, s, ncon + pre + 1, c1, p);
      ncon += __popc(m1) + __popc(m2);
    }
    int overflow = ncon > C::CON;
    if (overflow) ncon = C::CON;
    if (sl == 0) s.ncon = ncon;
    WSYNC();
    return overflow;
  }

  // mj_crb -> Mr rows (registers)
  __device__ __forceinline__ void mass_matrix() {
    phase_begin();
    if (sl > 0 && sl < nb) {
      const uint32_t dm = m->body_descmask[sl] & ~1u & ((nb < 32 ? (1u << nb) : 0u) - 1u);
      T a[10] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0};
      for_bits<T>(dm, [&](int c) { Vals<T, 10> r; for (int k = 0; k < 10; k++) r.v[k] = s.cinert[c][k]; return r; },
                  [&](int, const Vals<T, 10>& r) { for (int k = 0; k < 10; k++) a[k] += r.v[k]; });   // the subtree's bodies, ascending
      for (int k = 0; k < 10; k++) s.u.c.crb[sl][k] = a[k];
    }
    WSYNC();
    T bf[6] = {0, 0, 0, 0, 0, 0};
    uint32_t anci = 0;
    T arm = 0;
    if (sl < NV) {
      mul_inert(s.u.c.crb[m->dof_bodyid[sl]], cd, bf);
      for (int k = 0; k < 6; k++) s.u.c.buf[sl][k] = bf[k];
      anci = m->dof_ancmask[sl];
      arm = m->dof_armature[sl];
    }
    WSYNC();
    // one column per scheduling group (2 or 3 measured the same)
    {
      // software-pipelined: column j+1's cdof / buf rows are read before column j's arithmetic
      T cb2[2][12];
      auto load = [&](auto jc, T (&dst)[12]) {
        constexpr int j = decltype(jc)::value;
        for (int k = 0; k < 6; k++) { dst[k] = s.cdof[j][k]; dst[6 + k] = s.u.c.buf[j][k]; }
      };
      load(std::integral_constant<int, 0>{}, cb2[0]);
      static_for<0, NV>([&](auto jc) {
        constexpr int j = decltype(jc)::value;
        if constexpr (j + 1 < NV) load(std::integral_constant<int, j + 1>{}, cb2[(j + 1) & 1]);
        SCHED_FENCE();
        const uint32_t ancj = m->dof_ancmask[j];
        const bool rel = (sl < NV) && (bit(anci, j) || bit(ancj, sl));
        const T* cj = cb2[j & 1];
        const T v = (j <= sl) ? dot6(cj, bf) : dot6(cd, cj + 6);
        Mr[j] = rel ? v + ((j == sl) ? arm : T(0)) : T(0);
      });
    }
    WSYNC();
  }

  // mj_comVel (cvel, cdof_dot), mj_passive, mj_fwdActuation, mj_rne -> fsmooth
  __device__ __forceinline__ void velocity_forces() {
    phase_begin();
    if (sl < nb) {
      T v[6] = {0, 0, 0, 0, 0, 0};
      if (sl > 0) {
        const uint32_t ch = m->body_chainmask[sl];
        for_bits<T>(ch, [&](int j) { ValsX<T, 6> r; r.x = s.qvel[j]; for (int k = 0; k < 6; k++) r.v[k] = s.cdof[j][k]; return r; },
                    [&](int, const ValsX<T, 6>& r) { for (int k = 0; k < 6; k++) v[k] = fma(r.v[k], r.x, v[k]); });   // the chain's dofs, ascending
      }
      for (int k = 0; k < 6; k++) s.cvel[sl][k] = v[k];
    }
    if (sl < NV) {
      const uint32_t dm = m->dof_dotmask[sl];
      T v[6] = {0, 0, 0, 0, 0, 0}, cdd[6];
      for_bits<T>(dm, [&](int j) { ValsX<T, 6> r; r.x = s.qvel[j]; for (int k = 0; k < 6; k++) r.v[k] = s.cdof[j][k]; return r; },
                  [&](int, const ValsX<T, 6>& r) { for (int k = 0; k < 6; k++) v[k] = fma(r.v[k], r.x, v[k]); });   // ascending, set bits only
      cross_motion(v, cd, cdd);
      for (int k = 0; k < 6; k++) s.u.r.cdofdot[sl][k] = cdd[k];
    }
    WSYNC();
    if (sl > 0 && sl < nb) {   // RNE: cacc, cfrc_body
      const uint32_t ch = m->body_chainmask[sl];
      T a[6] = {0, 0, 0, -m->gravity[0], -m->gravity[1], -m->gravity[2]};
      for_bits<T>(ch, [&](int j) { ValsX<T, 6> r; r.x = s.qvel[j]; for (int k = 0; k < 6; k++) r.v[k] = s.u.r.cdofdot[j][k]; return r; },
                  [&](int, const ValsX<T, 6>& r) { for (int k = 0; k < 6; k++) a[k] = fma(r.v[k], r.x, a[k]); });   // the chain's dofs, ascending
      T f[6], t[6], t2[6];
      mul_inert(s.cinert[sl], a, f);
      mul_inert(s.cinert[sl], s.cvel[sl], t);
      cross_force(s.cvel[sl], t, t2);
      for (int k = 0; k < 6; k++) s.u.r.cfrc[sl][k] = f[k] + t2[k];
    }
    WSYNC();
    if (sl > 0 && sl < nb) {   // subtree sums of cfrc_body
      const uint32_t dm = m->body_descmask[sl] & ~1u & ((nb < 32 ? (1u << nb) : 0u) - 1u);
      T a[6] = {0, 0, 0, 0, 0, 0};
      for_bits<T>(dm, [&](int c) { Vals<T, 6> r; for (int k = 0; k < 6; k++) r.v[k] = s.u.r.cfrc[c][k]; return r; },
                  [&](int, const Vals<T, 6>& r) { for (int k = 0; k < 6; k++) a[k] += r.v[k]; });   // the subtree's bodies, ascending
      for (int k = 0; k < 6; k++) s.u.r.csub[sl][k] = a[k];
    }
    WSYNC();
    fsmooth = 0;
    qfa = 0;
    if (sl < NV) {
      T bias = dot6(cd, s.u.r.csub[m->dof_bodyid[sl]]);
      int qa = m->dof_qposadr[sl];
      T pas = -m->dof_damping[sl] * s.qvel[sl];
      if (qa >= 0) pas -= m->dof_stiffness[sl] * (s.qpos[qa] - m->dof_springref[sl]);
      int u = m->dof_actuator[sl];
      if (u >= 0) {
        T c = s.ctrl[u];
        if (m->act_ctrllimited[u]) c = fmin(m->act_ctrlrange[u][1], fmax(m->act_ctrlrange[u][0], c));
        qfa = m->act_gear[u] * c;
      }
      fsmooth = pas - bias + qfa;
    }
    WSYNC();
  }

  // mj_makeConstraint + mj_makeImpedance + reference (aref); row q of this lane: r = sl + 32 q
  __device__ __forceinline__ int rows(T (&D)[C::RPL], T (&ar)[C::RPL], int (&rd)[C::RPL], T (&rc)[C::RPL]) {
    phase_begin();
    damp = sl < NV ? m->dof_damping[sl] : T(0);
    int overflow = 0;
    int ncon = s.ncon;
    int nrow = 0;
    {   // joint limits (lower side first, MuJoCo side = -1 then +1)
      bool lo = false, hi = false;
      if (sl < m->njnt && m->jnt_limited[sl]) {
        T q = s.qpos[m->jnt_qposadr[sl]];
        lo = (q - m->jnt_range[sl][0]) < m->jnt_margin[sl];
        hi = (m->jnt_range[sl][1] - q) < m->jnt_margin[sl];
      }
      uint32_t ml = hballot(lo, up), mh = hballot(hi, up);
      int pre = below(ml, sl) + below(mh, sl);
      if (lo) s.row_kid[pre] = (RK_JLO << 16) | sl;
      if (hi) s.row_kid[pre + lo] = (RK_JHI << 16) | sl;
      nrow = __popc(ml) + __popc(mh);
      s.lim_row[sl] = 0;                       // MAXDOF == HL: one slot per sub-lane
      if (lo || hi)
        s.lim_row[m->jnt_dofadr[sl]] = (uint16_t)((lo ? pre + 1 : 0) | (hi ? (pre + lo + 1) << 8 : 0));
    }
    const int njl = nrow;
    {   // tendon limits
      bool lo = false, hi = false;
      if (sl < m->ntendon && m->ten_limited[sl]) {
        T L = 0;
        for (int w = 0; w < m->ten_nwrap[sl]; w++) L += m->ten_wrapcoef[sl][w] * s.qpos[m->ten_wrapqadr[sl][w]];
        lo = (L - m->ten_range[sl][0]) < m->ten_margin[sl];
        hi = (m->ten_range[sl][1] - L) < m->ten_margin[sl];
      }
      uint32_t ml = hballot(lo, up), mh = hballot(hi, up);
      int pre = nrow + below(ml, sl) + below(mh, sl);
      if (lo) s.row_kid[pre] = (RK_TLO << 16) | sl;
      if (hi) s.row_kid[pre + lo] = (RK_THI << 16) | sl;
      nrow += __popc(ml) + __popc(mh);
    }
    int nlim = nrow;
    {   // contacts: 1 row (condim 1) or 4 pyramid rows (condim 3), in contact order
      int tot = 0;
#pragma unroll
      for (int cs = 0; cs < C::CON; cs += HL) {
        const int c = cs + sl;
        const bool isc = c < ncon;
        const bool pyr = isc && (s.con_bb[c] >> 16) == 3;
        tot += __popc(hballot(isc, up)) + 3 * __popc(hballot(pyr, up));
      }
      if (nrow + tot > C::EFC) {   // drop whole contacts that do not fit (counted as overflow)
        overflow = 1;
        int fit = 0, nr = nrow;
        for (int c = 0; c < ncon; c++) {
          int need = (s.con_bb[c] >> 16) == 3 ? 4 : 1;
          if (nr + need > C::EFC) break;
          nr += need;
          fit++;
        }
        ncon = fit;
      }
#pragma unroll
      for (int cs = 0; cs < C::CON; cs += HL) {
        const int c = cs + sl;
        const bool isc = c < ncon;
        const bool pyr = isc && (s.con_bb[c] >> 16) == 3;
        const uint32_t mc = hballot(isc, up), mp = hballot(pyr, up);
        const int pre = nrow + below(mc, sl) + 3 * below(mp, sl);
        if (isc) {
          s.con_adr[c] = pre;
          if (!pyr) s.row_kid[pre] = (RK_CN << 16) | c;
          else for (int q = 0; q < 4; q++) s.row_kid[pre + q] = ((RK_P0 + q) << 16) | c;
        }
        nrow += __popc(mc) + 3 * __popc(mp);
      }
    }
    if (sl == 0) { s.ncon = ncon; s.nefc = nrow; s.nlim = nlim; s.njl = njl; }
    if (sl < NV) s.vx[sl] = s.qvel[sl];
    WSYNC();
    map_vx<NV>(s, sl, nb, chain_mask(m, sl, nb));     // row velocities J qvel for aref
#pragma unroll
    for (int q = 0; q < C::RPL; q++) {
      int r = sl + HL * q;
      D[q] = 0;
      ar[q] = 0;
      rd[q] = 0;
      rc[q] = 0;
      bool dense = false;
      if (r < nrow) {
        int kid = s.row_kid[r];
        int kind = rk_kind(kid), id = rk_id(kid);
        T pos, margin, dA, rscale = 1;
        CPtr<T> sr;
        CPtr<T> si;
        if (kind <= RK_JHI) {
          T qv = s.qpos[m->jnt_qposadr[id]];
          pos = kind == RK_JLO ? qv - m->jnt_range[id][0] : m->jnt_range[id][1] - qv;
          margin = m->jnt_margin[id];
          sr = m->jnt_solref[id]; si = m->jnt_solimp[id];
          int dof = m->jnt_dofadr[id];
          dA = m->dof_invweight0[dof];
          rd[q] = (kind << 16) | dof;
          rc[q] = kind == RK_JLO ? T(1) : T(-1);
        } else if (kind <= RK_THI) {
          T L = 0;
          for (int w = 0; w < m->ten_nwrap[id]; w++) L += m->ten_wrapcoef[id][w] * s.qpos[m->ten_wrapqadr[id][w]];
          pos = kind == RK_TLO ? L - m->ten_range[id][0] : m->ten_range[id][1] - L;
          margin = m->ten_margin[id];
          sr = m->ten_solref[id]; si = m->ten_solimp[id];
          dA = m->ten_invweight0[id];
          rd[q] = kid;
          rc[q] = kind == RK_TLO ? T(1) : T(-1);
          dense = true;
        } else {
          int p = s.con_pair[id];
          pos = s.con_dist[id];
          margin = m->pair_margin[p];
          sr = m->pair_solref[p]; si = m->pair_solimp[p];
          const uint32_t bb = s.con_bb[id];
          T tran = m->body_invweight_tran[bb & 0xff] + m->body_invweight_tran[(bb >> 8) & 0xff];
          T mu = s.con_mu[id];
          dA = kind == RK_CN ? tran : tran + mu * mu * tran;
          // pyramidal edges share one R: Rpy = 2 mu^2 R_edge / impratio (impratio = 1, enforced by the
          // compiler); pinned by the reference's recorded MuJoCo state, tests/test_reference_pin.py
          if (kind != RK_CN) rscale = 2 * mu * mu;
          rd[q] = kid;
          rc[q] = kind == RK_CN ? T(0) : (((kind - RK_P0) & 1) ? -mu : mu);
          dense = s.con_m1[id] != 0u;
        }
        T imp = impedance(si, pos, margin);
        T dmax = fmin(T(0.9999), fmax(T(0.0001), si[1]));
        T K, B;
        if (sr[0] > 0) {   // (reciprocals, not IEEE divides: ~1 ulp, and a shorter fp64 chain)
          T tc = fmax(sr[0], 2 * m->timestep), dr = sr[1];
          const T u = recip(dmax * tc), ud = u * recip(dr);
          K = ud * ud;
          B = 2 * u;
        } else {
          const T v = recip(dmax);
          K = -sr[0] * v * v;
          B = -sr[1] * v;
        }
        T R = rscale * fmax(T(1e-15), (1 - imp) * dA * recip(imp));
        D[q] = recip(R);
        s.row_D[r] = D[q];
        ar[q] = -B * row_Jx(m, s, rd[q], rc[q]) - K * imp * (pos - margin);
      }
      uint32_t dm = hballot(dense, up);
      if (sl == 0) s.dense_mask[q] = dm;
    }
    WSYNC();
    return overflow;
  }

  // primal Newton (mj_solNewton semantics), warm-started; x = qacc
  __device__ __forceinline__ void solve(T xws, int maxit, T tol, const T (&D)[C::RPL], const T (&ar)[C::RPL],
                                        const int (&rd)[C::RPL], const T (&rc)[C::RPL]) {
    phase_begin();
    const int nefc = s.nefc;
    T x = sl < NV ? xws : T(0);
    bool vr[C::RPL];
#pragma unroll
    for (int q = 0; q < C::RPL; q++) vr[q] = sl + HL * q < nefc;
    const uint32_t anci = sl < NV ? m->dof_ancmask[sl] : 0u;
    const uint32_t bch = chain_mask(m, sl, nb);     // loaded once per solve (map_vx per iteration)
    const T scale = m->newton_scale;
    if (sl < NV) s.vx[sl] = x;
    WSYNC();
    T Mx = matvec_lds(Mr, s.vx);     // kept current below (Mx += alpha M s)
    map_vx<NV>(s, sl, nb, bch);
    T jar[C::RPL], Js[C::RPL];
#pragma unroll
    for (int q = 0; q < C::RPL; q++) jar[q] = vr[q] ? row_Jx(m, s, rd[q], rc[q]) - ar[q] : T(0);
    HS_STAMP(clk, 6);
    bool done = false;      // this half-wave's solver has converged
    int it = 0;
    if (sl == 0) s.niter = maxit;   // per env: the iteration at which this half converged
    for (; it < maxit; it++) {
      m = opaque(m);
      sl = opaque_v(sl);
      bool act[C::RPL];
#pragma unroll
      for (int q = 0; q < C::RPL; q++) {
        act[q] = vr[q] && jar[q] < 0;
        if (vr[q]) s.row_f[sl + HL * q] = act[q] ? -D[q] * jar[q] : T(0);
      }
      WSYNC();
      contact_aggregates(m, s, sl);
      HS_STAMP(clk, 7);
      T jtf = jtf_lane(m, s, sl, cd);
      T g = sl < NV ? Mx - fsmooth - jtf : T(0);
      const T gn2 = hsum(g * g);                 // |g| scale < tol, squared (no sqrt on the chain)
      const bool conv = scale * scale * gn2 < tol * tol;
      if (conv && !done && sl == 0) s.niter = it;
      done = done || conv;
      HS_STAMP(clk, 8);
      if (__ballot(!done) == 0) break;       // both envs of the wave converged
      T H[NV];
#ifndef HS_NEWTON_GJ
      T hdinv = 0, hdiag = 0;
#endif
      // Hessian lower rows: M + contact (tree form) + joint limits (diag) + dense rank-1 rows
      {
        T aug[6] = {0, 0, 0, 0, 0, 0};
        T dadd = 0;
        struct CU { uint32_t m1, m2; T p[3], U[6]; };
        for_active_contacts_ld<T, C>(s.con_act, [&](int c) {
          CU v;
          v.m1 = s.con_m1[c]; v.m2 = s.con_m2[c];
          for (int k = 0; k < 3; k++) v.p[k] = s.con_pos[c][k];
          for (int k = 0; k < 6; k++) v.U[k] = s.con_U[c][k];
          return v;
        }, [&](int, const CU& v) {   // (contacts with U = 0 add exact zeros)
          if (v.m1 != 0u || !bit(v.m2, sl)) return;   // body-body: dense rank-1 rows below
          T r[3] = {v.p[0] - s.com[0], v.p[1] - s.com[1], v.p[2] - s.com[2]};
          T w[3];
          cross3(cd, r, w);
          T jp[3] = {cd[3] + w[0], cd[4] + w[1], cd[5] + w[2]};
          const T* U = v.U;
          T z[3] = {U[0] * jp[0] + U[3] * jp[1] + U[4] * jp[2], U[3] * jp[0] + U[1] * jp[1] + U[5] * jp[2],
                    U[4] * jp[0] + U[5] * jp[1] + U[2] * jp[2]};
          T rz[3];
          cross3(r, z, rz);
          for (int k = 0; k < 3; k++) { aug[k] += rz[k]; aug[3 + k] += z[k]; }
        });
        {   // active joint-limit rows of this dof (diagonal)
          int lr = s.lim_row[sl];
          int lo = (lr & 0xff) - 1, hi = (lr >> 8) - 1;
          if (lo >= 0 && s.row_f[lo] != T(0)) dadd += s.row_D[lo];
          if (hi >= 0 && s.row_f[hi] != T(0)) dadd += s.row_D[hi];
        }
        HS_STAMP(clk, 27);
#ifdef HS_NEWTON_GJ
        // the full symmetric rows (gj_solve2 needs the upper triangle too): H_ij = cdof_j . aug_i for an
        // ancestor j of dof i, = cdof_i . aug_j for a descendant j (H_ji, with lane j's aggregate read
        // from LDS), as mass_matrix() builds M's full rows
        if (sl < NV)
          for (int k = 0; k < 6; k++) s.u.n.aug[sl][k] = aug[k];
        WSYNC();
        {
          // software-pipelined like the lower-only rows: column j + 1's cdof and aug rows are read
          // before column j's arithmetic (fenced), so each LDS round trip overlaps the FMAs
          const uint32_t relm = sl < NV ? m->dof_relmask[sl] : 0u;
          T cbuf[2][12];
          auto load = [&](auto jc, T (&dst)[12]) {
            constexpr int j = decltype(jc)::value;
            for (int k = 0; k < 6; k++) { dst[k] = s.cdof[j][k]; dst[6 + k] = s.u.n.aug[j][k]; }
          };
          load(std::integral_constant<int, 0>{}, cbuf[0]);
          static_for<0, NV>([&](auto jc) {
            constexpr int j = decltype(jc)::value;
            if constexpr (j + 1 < NV) load(std::integral_constant<int, j + 1>{}, cbuf[(j + 1) & 1]);
            SCHED_FENCE();
            const T* cj = cbuf[j & 1];
            const T v = (j <= sl) ? dot6(cj, aug) : dot6(cd, cj + 6);
            H[j] = Mr[j] + (bit(relm, j) ? v : T(0)) + ((j == sl) ? dadd : T(0));
          });
        }
#else
        // HESS_G columns per scheduling group: their cdof rows are read from LDS together, so one
        // LDS round trip is exposed per group instead of per column
        constexpr int HESS_G = sizeof(T) == 8 ? 2 : 1;
        if constexpr (HESS_G == 1) {
#pragma unroll
          for (int j = 0; j < NV; j++) {
            T cj[6];
            for (int k = 0; k < 6; k++) cj[k] = s.cdof[j][k];
            H[j] = Mr[j] + (bit(anci, j) ? dot6(cj, aug) : T(0)) + ((j == sl) ? dadd : T(0));
            SCHED_FENCE();
          }
        } else {
          // software-pipelined: group g+1's cdof rows are read before group g's arithmetic (fenced),
          // so each group's LDS round trip overlaps the previous group's FMAs
          constexpr int NG = (NV + HESS_G - 1) / HESS_G;
          T cbuf[2][HESS_G][6];
          auto load = [&](auto gc, T (&dst)[HESS_G][6]) {
            constexpr int j0 = decltype(gc)::value * HESS_G;
            static_for<0, HESS_G>([&](auto tc) {
              constexpr int t = decltype(tc)::value;
              if constexpr (j0 + t < NV)
                for (int k = 0; k < 6; k++) dst[t][k] = s.cdof[j0 + t][k];
            });
          };
          load(std::integral_constant<int, 0>{}, cbuf[0]);
          static_for<0, NG>([&](auto gc) {
            constexpr int g = decltype(gc)::value, j0 = g * HESS_G;
            if constexpr (g + 1 < NG) load(std::integral_constant<int, g + 1>{}, cbuf[(g + 1) & 1]);
            SCHED_FENCE();
            static_for<0, HESS_G>([&](auto tc) {
              constexpr int t = decltype(tc)::value, j = j0 + t;
              if constexpr (j < NV)
                H[j] = Mr[j] + (bit(anci, j) ? dot6(cbuf[g & 1][t], aug) : T(0)) + ((j == sl) ? dadd : T(0));
            });
          });
        }
#endif
        HS_STAMP(clk, 28);
        // dense rank-1 rows (tendon limits, body-body contacts): only the rows flagged in
        // dense_mask; the loop runs max(#rows of either half) times (wave-uniform control)
        uint32_t dm[C::RPL];
#pragma unroll
        for (int q = 0; q < C::RPL; q++) dm[q] = s.dense_mask[q] & hballot(act[q], up);   // active ones only
        for (;;) {
          int r = -1;
#pragma unroll
          for (int q = C::RPL - 1; q >= 0; q--)
            if (dm[q]) r = HL * q + __builtin_ctz(dm[q]);
          if (__ballot(r >= 0) == 0) break;
          T jr = 0, Dr = 0;
          if (r >= 0) {
            dm[r / HL] &= dm[r / HL] - 1u;           // consume the row
            if (s.row_f[r] != T(0)) {
              int kid = s.row_kid[r];
              int kind = rk_kind(kid), id = rk_id(kid);
              Dr = s.row_D[r];
              if (kind == RK_TLO || kind == RK_THI) {
                for (int w = 0; w < m->ten_nwrap[id]; w++)
                  if (m->ten_wrapdof[id][w] == sl) jr += m->ten_wrapcoef[id][w];
                if (kind == RK_THI) jr = -jr;
              } else {
                int in2 = bit(s.con_m2[id], sl), in1 = bit(s.con_m1[id], sl);
                if (in1 != in2) {
                  T rr[3] = {s.con_pos[id][0] - s.com[0], s.con_pos[id][1] - s.com[1], s.con_pos[id][2] - s.com[2]};
                  T w[3], u[3];
                  cross3(cd, rr, w);
                  T jp[3] = {cd[3] + w[0], cd[4] + w[1], cd[5] + w[2]};
                  row_u(m, s, kind, id, u);
                  jr = in2 ? dot3(u, jp) : -dot3(u, jp);
                }
              }
            }
          }
          if (sl >= NV) jr = 0;
          T dj = Dr * jr;
          static_for<0, NV>([&](auto jc) {
            constexpr int j = decltype(jc)::value;
            H[j] += dj * bcast<j>(jr);
          });
        }
      }
      HS_STAMP(clk, 9);
#ifndef HS_NEWTON_GJ   // the factor + substitutions (HS_NEWTON_GJ: the Gauss-Jordan A/B build)
      chol_rows<NV, T, LDLF>(H, hdinv, sl, s.u.n.cb, &hdiag);   // (LDLF: as L D L')
      HS_STAMP(clk, 15);
      T sdir = -chol_solve<NV, T, LDLF>(H, hdinv, g, sl);
#else
      T sdir = -gj_solve2<NV>(H, g, sl, &s.u.n.cb[0][0]);
      HS_STAMP(clk, 15);
#endif
      if (sl >= NV) sdir = 0;
      HS_STAMP(clk, 10);
      // exact line search along sdir (piecewise-quadratic cost)
      if (sl < NV) s.vx[sl] = sdir;
      WSYNC();
      T Ms = matvec_lds(Mr, s.vx);
      T A0 = hsum(sl < NV ? sdir * Ms : T(0));
      T B0 = hsum(sl < NV ? sdir * (Mx - fsmooth) : T(0));
      HS_STAMP(clk, 18);
      map_vx<NV>(s, sl, nb, bch);
      HS_STAMP(clk, 19);
#pragma unroll
      for (int q = 0; q < C::RPL; q++) Js[q] = vr[q] ? row_Jx(m, s, rd[q], rc[q]) : T(0);
      HS_STAMP(clk, 16);
      // alpha = 1 is exact when no row changes state on [0, 1] (jar is linear in alpha)
      bool same1 = true;
#pragma unroll
      for (int q = 0; q < C::RPL; q++) same1 = same1 && (!vr[q] || ((jar[q] + Js[q] < 0) == act[q]));
      bool lsdone = done || (hballot(!same1, up) == 0);
      T alpha = 1, lo = 0, hi = T(1e30);
      T d0 = 0;
      {
        T c = 0;
#pragma unroll
        for (int q = 0; q < C::RPL; q++) c += act[q] ? D[q] * jar[q] * Js[q] : T(0);
        d0 = B0 + hsum(c);
      }
      const T ltol = (sizeof(T) == 8 ? T(1e-10) : T(1e-5)) * fabs(d0);
      for (int ls = 0; ls < 30; ls++) {
        if (__ballot(!lsdone) == 0) break;
        T c1 = 0, c2 = 0;
#pragma unroll
        for (int q = 0; q < C::RPL; q++) {
          T jq = jar[q] + alpha * Js[q];
          bool a = vr[q] && jq < 0;
          c1 += a ? D[q] * jq * Js[q] : T(0);
          c2 += a ? D[q] * Js[q] * Js[q] : T(0);
        }
        T d1 = B0 + alpha * A0 + hsum(c1);
        T d2 = A0 + hsum(c2);
        if (!lsdone) {
          if (fabs(d1) <= ltol) {
            lsdone = true;
          } else {
            if (d1 < 0) lo = alpha; else hi = alpha;
            T an = d2 > 0 ? alpha - d1 * recip(d2) : T(-1);
            if (!(an > lo && an < hi)) an = hi < T(1e29) ? T(0.5) * (lo + hi) : T(2) * alpha;
            if (hi - lo <= (sizeof(T) == 8 ? T(1e-14) : T(1e-6)) * hi) lsdone = true;
            else alpha = an;
          }
        }
      }
      HS_STAMP(clk, 11);
      if (!done) {
        x += alpha * sdir;
        Mx += alpha * Ms;
        bool changed = false;
#pragma unroll
        for (int q = 0; q < C::RPL; q++) {
          T nj = jar[q] + alpha * Js[q];
          changed = changed || (vr[q] && ((nj < 0) != act[q]));
          jar[q] = nj;
        }
        if (hballot(changed, up) == 0 && fabs(alpha - T(1)) < T(1e-3)) {
          done = true;
          if (sl == 0) s.niter = it + 1;
        }
      }
      if (__ballot(!done) == 0) { it++; break; }
    }
    WSYNC();
    niter = s.niter;
    // final forces -> qfrc_constraint
#pragma unroll
    for (int q = 0; q < C::RPL; q++)
      if (vr[q]) s.row_f[sl + HL * q] = jar[q] < 0 ? -D[q] * jar[q] : T(0);
    WSYNC();
    contact_aggregates(m, s, sl);
    fcon = sl < NV ? jtf_lane(m, s, sl, cd) : T(0);
    qacc = x;
    WSYNC();
    HS_STAMP(clk, 12);
  }


  // lane (dof) j's entry of constraint row r's Jacobian (the same per-row Jacobians row_Jx applies
  // through body velocities and the Newton Hessian's dense rank-1 terms use)
  __device__ __forceinline__ T row_J_lane(int r) {
    if (sl >= NV) return T(0);
    const int kid = s.row_kid[r];
    const int kind = rk_kind(kid), id = rk_id(kid);
    if (kind <= RK_JHI) return m->jnt_dofadr[id] == sl ? (kind == RK_JLO ? T(1) : T(-1)) : T(0);
    if (kind <= RK_THI) {
      T v = 0;
      for (int w = 0; w < m->ten_nwrap[id]; w++)
        if (m->ten_wrapdof[id][w] == sl) v += m->ten_wrapcoef[id][w];
      return kind == RK_TLO ? v : -v;
    }
    const int in2 = bit(s.con_m2[id], sl), in1 = bit(s.con_m1[id], sl);
    if (in1 == in2) return T(0);
    T rr[3] = {s.con_pos[id][0] - s.com[0], s.con_pos[id][1] - s.com[1], s.con_pos[id][2] - s.com[2]};
    T w[3], u[3];
    cross3(cd, rr, w);
    T jp[3] = {cd[3] + w[0], cd[4] + w[1], cd[5] + w[2]};
    row_u(m, s, kind, id, u);
    const T v = dot3(u, jp);
    return in2 ? v : -v;
  }

  // mj_solPGS (<option solver="PGS">), restating oracle/hsim_oracle.c solve_pgs: projected
  // Gauss-Seidel on the dual  min 0.5 f'AR f + f'b, f >= 0  (AR = J M^-1 J' + R, b = J qacc_smooth -
  // aref), rows swept in efc order, MuJoCo's stopping rule (a sweep's improvement * scale <
  // tolerance, or maxit sweeps).  Without forming AR (see PgsCache): with z = L' qacc = L^-1
  // (qfrc_smooth + J'f) kept per dof lane, row r's dual residual is  u_r . z + R_r f_r - aref_r  (z is
  // the NET acceleration in the factor's basis, so fp32 sums do not cancel two large terms) and its
  // update adds delta u_r to z.  The half-wave sum u_r . z runs PGS_LA rows ahead (see PGS_LA).
  // u_r = L^-1 J_r' of the cached rows comes from one multi-right-hand-side forward substitution per
  // substep.  Warm start: the forces of qacc_warmstart under the primal map, kept if their dual cost
  // is not positive.  z is re-anchored on the forces every 8 sweeps (fp32 rounding drift); the final
  // qacc = M^-1 (qfrc_smooth + J'f) comes from the final forces.
  __device__ __forceinline__ void solve_pgs(T xws, int maxit, const T (&D)[C::RPL], const T (&ar)[C::RPL],
                                            const int (&rd)[C::RPL], const T (&rc)[C::RPL], PgsCache<T, C>& pc) {
    phase_begin();
    const int nefc = s.nefc;
    const uint32_t bch = chain_mask(m, sl, nb);
    const T fs = sl < NV ? fsmooth : T(0);
    constexpr int NC = PgsCache<T, C>::NC;
    constexpr int LA = PGS_LA;
    bool vr[C::RPL];
#pragma unroll
    for (int q = 0; q < C::RPL; q++) vr[q] = sl + HL * q < nefc;
    T L[NV];
#pragma unroll
    for (int j = 0; j < NV; j++) L[j] = Mr[j];
    T dinv = 0;
    chol_rows<NV>(L, dinv, sl, s.u.n.cb);
    // warm start: f = -D (J xws - aref)_-;  per-row b_r = -aref_r, R_r
    if (sl < NV) s.vx[sl] = xws;
    WSYNC();
    map_vx<NV>(s, sl, nb, bch);
    T wc = 0;     // this lane's rows' part of the warm start's dual cost: sum f (0.5 R f - aref)
#pragma unroll
    for (int q = 0; q < C::RPL; q++) {
      const int r = sl + HL * q;
      if (vr[q]) {
        const T jar = row_Jx(m, s, rd[q], rc[q]) - ar[q];
        const T f = jar < 0 ? -D[q] * jar : T(0);
        const T R = recip(D[q]);
        s.row_f[r] = f;
        pc.row[r].b = -ar[q];
        pc.row[r].R = R;
        wc += f * (T(0.5) * R * f - ar[q]);
      }
    }
    WSYNC();
    // rows that exist in either half of the wave (wave-uniform loop bounds)
    int maxr = nefc;
    maxr = max(maxr, __shfl_xor(maxr, HL));
    // u_r of the cached rows (G right-hand sides per forward substitution)
    constexpr int G = sizeof(T) == 8 ? 4 : 8;
    const int ncache = maxr < NC ? maxr : NC;
    for (int r0 = 0; r0 < ncache; r0 += G) {
      T y[G];
      static_for<0, G>([&](auto gc) {
        constexpr int g = decltype(gc)::value;
        y[g] = r0 + g < nefc ? row_J_lane(r0 + g) : T(0);
      });
      chol_fwd_multi<NV, G>(L, dinv, y, sl);
      static_for<0, G>([&](auto gc) {
        constexpr int g = decltype(gc)::value;
        if (r0 + g < NC) pc.u[r0 + g][sl] = sl < NV ? y[g] : T(0);   // MAXDOF == HL: a slot per sub-lane
      });
    }
    WSYNC();
    // u_r of any row (LDS cache, or rebuilt for rows past it; 0 past the half's rows)
    auto urow = [&](int r) -> T {
      if (r < NC) return pc.u[r][sl];
      T y = chol_fwd<NV>(L, dinv, r < nefc ? row_J_lane(r) : T(0), sl);
      return sl < NV ? y : T(0);
    };
    // AR_rr = |u_r|^2 + R_r and the lookahead Gram terms of every row
    {
      T uw[LA + 1];     // u_{r-LA} .. u_r
#pragma unroll
      for (int j = 0; j < LA; j++) uw[j] = 0;
      for (int r = 0; r < maxr; r++) {
        uw[LA] = urow(r);
        const T a = hsum(uw[LA] * uw[LA]);
        T gr[LA];
#pragma unroll
        for (int j = 1; j <= LA; j++) gr[j - 1] = hsum(uw[LA] * uw[LA - j]);
        if (r < nefc && sl == 0) {
          const T arr = a + pc.row[r].R;
          pc.row[r].ar = arr;
          pc.row[r].ai = recip(arr < T(1e-15) ? T(1e-15) : arr);
#pragma unroll
          for (int j = 0; j < LA; j++) pc.row[r].g[j] = gr[j];
        }
#pragma unroll
        for (int j = 0; j < LA; j++) uw[j] = uw[j + 1];
      }
    }
    WSYNC();
    // y0 = L^-1 qfrc_smooth and z = L^-1 (qfrc_smooth + J'f) of the warm-start forces
    contact_aggregates(m, s, sl);
    T z, y0;
    {
      T y2[2] = {fs, fs + (sl < NV ? jtf_lane(m, s, sl, cd) : T(0))};
      chol_fwd_multi<NV, 2>(L, dinv, y2, sl);
      y0 = sl < NV ? y2[0] : T(0);
      z = sl < NV ? y2[1] : T(0);
    }
    // keep the warm start only if its dual cost 0.5 f'AR f + f'b = 0.5 |z|^2 - 0.5 |y0|^2 +
    // sum f (0.5 R f - aref) is not positive
    if (hsum(wc + T(0.5) * (z * z - y0 * y0)) > T(0)) {
#pragma unroll
      for (int q = 0; q < C::RPL; q++)
        if (vr[q]) s.row_f[sl + HL * q] = 0;
      z = y0;
    }
    WSYNC();
    const T scale = m->newton_scale, tol = m->pgs_tol;
    bool done = false;
    int it = 0;
    for (int sweep = 0; sweep < maxit; sweep++) {
      m = opaque(m);
      sl = opaque_v(sl);
      T improvement = 0;
      // ring registers (slot = row mod RING, RING = LA + 1; the row loop is unrolled by RING so every
      // slot index is a compile-time constant and the pipeline shifts no registers):
      // U[slot] = u_row, S[slot] = u_row . z_{row-LA-1} (z with rows < row-LA applied),
      // Dl[slot] = delta_row.  At row r, z still lacks row r-1's update.  Positions past maxr are
      // phantom rows (u = 0, delta = 0).
      // LDS operands are loaded one row before their use (P/F: row r+1's scalars and force, un: u of
      // row r+LA+1), so no row waits on an LDS round trip (a wave issues in order: a load consumed
      // in the same row would stall it for the full LDS latency); loads are unconditional (clamped
      // index, masked value) so the row step has no divergent branch.
      // FAST: every row of both halves is in the u cache (the common case), no rebuild path.
      auto sweep_rows = [&](auto fastc) {
        constexpr bool FAST = decltype(fastc)::value;
        auto uget = [&](int r) -> T {
          if constexpr (FAST) return pc.u[r][sl];
          else return urow(r);
        };
        constexpr int RING = LA + 1;
        static_assert(RING % 2 == 0, "P/F double buffer alternates with the row parity");
        T U[RING], S[RING], Dl[RING];
#pragma unroll
        for (int i = 0; i < RING; i++) {
          U[i] = (i < LA && i < maxr) ? uget(i) : T(0);
          S[i] = i < LA ? hsum(U[i] * z) : T(0);
          Dl[i] = 0;
        }
        PgsRow<T> P[2];
        T F[2];
        P[0] = pc.row[0];
        F[0] = nefc > 0 ? s.row_f[0] : T(0);
        T unext = LA < maxr ? uget(LA) : T(0);
        for (int r0 = 0; r0 < maxr; r0 += RING) {
          static_for<0, RING>([&](auto ic) {
            constexpr int i = decltype(ic)::value;
            constexpr int prev = (i + RING - 1) % RING;   // slot of row r-1 (and of row r+LA)
            constexpr int cur = i & 1, nxt = cur ^ 1;
            const int r = r0 + i;
            {   // next row's operands
              const int rn = r + 1 < C::EFC ? r + 1 : C::EFC - 1;
              P[nxt] = pc.row[rn];
              const T fl = s.row_f[rn];
              F[nxt] = r + 1 < nefc ? fl : T(0);
            }
            const T un = unext;                          // u_{r+LA}
            unext = r + LA + 1 < maxr ? uget(r + LA + 1) : T(0);
            z = fma(Dl[prev], U[prev], z);               // z_{r-1}: rows < r applied
            const T Sn = hsum(un * z);                   // start row r+LA's sum on z_{r-1}
            const bool row = r < nefc;
            const bool live = row && !done;
            const PgsRow<T>& pr = P[cur];
            const T fr = F[cur];
            T dot = S[i];
            static_for<1, LA + 1>([&](auto jc) {         // corrections for rows r-1 .. r-LA
              constexpr int j = decltype(jc)::value;
              dot = fma(Dl[(i + RING - j) % RING], pr.g[j - 1], dot);
            });
            const T res = dot + (pr.b + pr.R * fr);
            T nf = fr - res * pr.ai;
            nf = nf < T(0) ? T(0) : nf;
            const T delta = live ? nf - fr : T(0);
            const T di = delta * res + T(0.5) * pr.ar * delta * delta;
            improvement -= row ? di : T(0);
            if (live && sl == 0) s.row_f[r] = nf;
            U[prev] = un;                                // row r+LA takes row r-1's slot
            S[prev] = Sn;
            Dl[i] = delta;
          });
        }
        z = fma(Dl[RING - 1], U[RING - 1], z);           // the last position's update (0 if phantom)
      };
      if (maxr <= NC) sweep_rows(std::true_type{});
      else sweep_rows(std::false_type{});
      if (!done) it++;
      done = done || (improvement * scale < tol);
      if (__ballot(!done) == 0) break;
      // re-anchor z on the current forces (fp32: every 8 sweeps; fp64 drifts ~1e-16 per update)
      if ((sweep & (sizeof(T) == 8 ? 31 : 7)) == (sizeof(T) == 8 ? 31 : 7)) {
        WSYNC();
        contact_aggregates(m, s, sl);
        const T zz = chol_fwd<NV>(L, dinv, fs + (sl < NV ? jtf_lane(m, s, sl, cd) : T(0)), sl);
        z = sl < NV ? zz : T(0);
      }
    }
    niter = it;
    WSYNC();
    contact_aggregates(m, s, sl);
    fcon = sl < NV ? jtf_lane(m, s, sl, cd) : T(0);
    const T qa = chol_solve<NV>(L, dinv, fs + fcon, sl);     // M^-1 (qfrc_smooth + J'f)
    qacc = sl < NV ? qa : T(0);
    WSYNC();
  }

  // full_state: contact part of mj_rnePostConstraint (cfrc_ext, at the root subtree com: body 2 of a
  // contact gets +[(p - com) x F, F], body 1 the opposite, world skipped) and mj_subtreeVel's linear
  // part (m v_com of every body = m lin + ang x (m d) from cvel / cinert, summed over subtrees).
  // Results stay in the Newton union (free after the solve) until obs / reward / commit read them.
  __device__ __forceinline__ void post_constraint() {
    phase_begin();
    const int b = sl;
    T cf[6] = {0, 0, 0, 0, 0, 0}, mv[3] = {0, 0, 0};
    if (b > 0 && b < nb) {
      for (int c = 0; c < s.ncon; c++) {
        const uint32_t bb = s.con_bb[c];
        const int b1 = bb & 0xff, b2 = (bb >> 8) & 0xff;
        if (b != b1 && b != b2) continue;
        const T sg = b == b2 ? T(1) : T(-1);
        T r[3] = {s.con_pos[c][0] - s.com[0], s.con_pos[c][1] - s.com[1], s.con_pos[c][2] - s.com[2]}, t[3];
        cross3(r, s.con_F[c], t);
        for (int k = 0; k < 3; k++) { cf[k] += sg * t[k]; cf[3 + k] += sg * s.con_F[c][k]; }
      }
      const T* ci = s.cinert[b];
      const T* cv = s.cvel[b];
      T w[3];
      cross3(cv, ci + 6, w);
      for (int k = 0; k < 3; k++) mv[k] = ci[9] * cv[3 + k] + w[k];
    }
    if (b < nb) {
      for (int k = 0; k < 6; k++) s.u.n.cfrc[b][k] = cf[k];
      for (int k = 0; k < 3; k++) s.u.n.mv[b][k] = mv[k];
    }
    WSYNC();
    if (b < nb) {
      const uint32_t dm = b == 0 ? ((1u << nb) - 2u) : m->body_descmask[b];
      T a[3] = {0, 0, 0}, ms = 0;
      for (int c = 1; c < nb; c++)
        if (bit(dm, c)) {
          for (int k = 0; k < 3; k++) a[k] += s.u.n.mv[c][k];
          ms += s.cinert[c][9];
        }
      const T inv = T(1) / (ms > T(1e-15) ? ms : T(1e-15));
      for (int k = 0; k < 3; k++) s.u.n.linv[b][k] = a[k] * inv;
    }
    WSYNC();
  }

  // mj_Euler with implicit damping, mj_integratePos
  __device__ __forceinline__ void euler(T& time) {
    phase_begin();
    T h = m->timestep;
    T He[NV];
#pragma unroll
    for (int j = 0; j < NV; j++) He[j] = Mr[j] + ((j == sl) ? h * damp : T(0));
    HS_STAMP(clk, 20);
    T edinv = 0, ediag = 0;
    chol_rows<NV, T, LDLE>(He, edinv, sl, s.u.n.cb, &ediag);
    HS_STAMP(clk, 21);
    T a = chol_solve<NV, T, LDLE>(He, edinv, fsmooth + fcon, sl);
    HS_STAMP(clk, 17);
    if (sl < NV) s.qvel[sl] += h * a;
    WSYNC();
    if (sl < m->njnt) {
      int qa = m->jnt_qposadr[sl], da = m->jnt_dofadr[sl];
      if (m->jnt_type[sl] == JNT_FREE) {
        for (int k = 0; k < 3; k++) s.qpos[qa + k] += h * s.qvel[da + k];
        T w[3] = {s.qvel[da + 3], s.qvel[da + 4], s.qvel[da + 5]};
        T ang = h * normalize3(w);
        T sn, cs;
        sincos_t(T(0.5) * ang, sn, cs);
        T qr[4] = {cs, w[0] * sn, w[1] * sn, w[2] * sn};
        T q[4] = {s.qpos[qa + 3], s.qpos[qa + 4], s.qpos[qa + 5], s.qpos[qa + 6]};
        normalize4(q);
        mulq(q, qr, q);
        for (int k = 0; k < 4; k++) s.qpos[qa + 3 + k] = q[k];
      } else {
        s.qpos[qa] += h * s.qvel[da];
      }
    }
    time += h;
    WSYNC();
  }
};

// ------------------------------------------------------------------ state helpers
__device__ __forceinline__ uint64_t splitmix(uint64_t x) {
  x += 0x9E3779B97F4A7C15ull;
  x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
  x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
  return x ^ (x >> 31);
}
template <typename T>
__device__ __forceinline__ T uniform_pm(uint64_t seed, int env, uint32_t episode, int k, T scale) {
  uint64_t h = splitmix(seed ^ splitmix(((uint64_t)env << 32) ^ ((uint64_t)episode << 8) ^ (uint64_t)k));
  double u = (double)(h >> 11) * (1.0 / 9007199254740992.0);   // [0, 1)
  return (T)(-scale + 2.0 * scale * u);
}

template <typename T, typename C>
__device__ __forceinline__ void reset_state(MPtr<T> m, Scratch<T, C>& s, int sl, T& time, T& xws) {
  if (sl < m->nq) s.qpos[sl] = m->qpos0[sl];
  if (sl + HL < m->nq) s.qpos[sl + HL] = m->qpos0[sl + HL];
  if (sl < m->nv) s.qvel[sl] = 0;
  if (sl < m->nu) s.ctrl[sl] = 0;
  xws = 0;
  time = 0;
  WSYNC();
}

template <typename T, int NV, bool PGS, typename C>
__device__ __forceinline__ void physics_step(Stepper<T, NV, C>& st, KPtr<T> k, T& time, T& xws, int* warn,
                                             PgsCache<T, C>* pc) {
  MPtr<T> m = st.m;
  Scratch<T, C>& s = st.s;
  const int sl = st.sl;
  const bool up = st.up;
  // mj_checkPos / mj_checkVel (auto-reset to qpos0, time 0)
  bool bq = (sl < m->nq && isbad(s.qpos[sl])) || (sl + HL < m->nq && isbad(s.qpos[sl + HL]));
  bool bv = sl < m->nv && isbad(s.qvel[sl]);
  if (hballot(bq, up)) { warn[WARN_BADQPOS]++; reset_state(m, s, sl, time, xws); }
  else if (hballot(bv, up)) { warn[WARN_BADQVEL]++; reset_state(m, s, sl, time, xws); }
  T D[C::RPL], ar[C::RPL], rc[C::RPL];
  int rd[C::RPL];
  for (int attempt = 0; attempt < 2; attempt++) {
    HS_STAMP(st.clk, 0);
    st.kinematics();
    HS_STAMP(st.clk, 1);
    if (st.collision()) warn[WARN_OVERFLOW]++;
    HS_STAMP(st.clk, 4);
    st.mass_matrix();
    HS_STAMP(st.clk, 2);
    st.velocity_forces();
    HS_STAMP(st.clk, 3);
    if (st.rows(D, ar, rd, rc)) warn[WARN_OVERFLOW]++;
    HS_STAMP(st.clk, 5);
    if constexpr (PGS)
      st.solve_pgs(xws, opaque(k)->p.max_newton, D, ar, rd, rc, *pc);
    else
      st.solve(xws, opaque(k)->p.max_newton, sizeof(T) == 8 ? T(1e-13) : T(1e-7), D, ar, rd, rc);
    bool ba = sl < m->nv && isbad(st.qacc);
    bool redo = hballot(ba, up) != 0 && attempt == 0;
    if (__ballot(redo) == 0) break;          // wave-uniform loop control
    if (redo) {                               // mj_checkAcc: reset and redo mj_forward
      warn[WARN_BADQACC]++;
      reset_state(m, s, sl, time, xws);
    }
  }
  if (opaque(k)->p.full_state) st.post_constraint();   // pre-integration state, like cinert / cvel in the obs
  st.euler(time);
  HS_STAMP(st.clk, 13);
  xws = st.qacc;
}

// sum |cfrc_ext| of the last two bodies ("feet", reward_functions.py:121-122,176-177)
template <typename T, typename C>
__device__ __forceinline__ void foot_forces(MPtr<T> m, const Scratch<T, C>& s, T& lf, T& rf) {
  const int nb = m->nbody;
  lf = 0;
  rf = 0;
  for (int k = 0; k < 6; k++) { lf += fabs(s.u.n.cfrc[nb - 2][k]); rf += fabs(s.u.n.cfrc[nb - 1][k]); }
}

// The reward plug-ins' inputs, gathered per env.  The step kernel fills them from its scratch
// (compute_reward below); hs_reward_eval (reward_eval_kernel) from caller-supplied fields.  Both run
// the same reward_formula, so the device formulas are pinned directly by the reference's golden vectors.
template <typename T>
struct RewardIn {
  T h, qw, qx, qy, qz;   // qpos[2], qpos[3:7]
  T vx;                  // qvel[0]
  T time;
  T com0, com1;          // subtree_com[0][0:2]
  T comv;                // sum(subtree_linvel[0]^2), numpy order (sequential: 3 < 8 terms)
  T lf, rf;              // sum |cfrc_ext[-2]|, sum |cfrc_ext[-1]| (numpy order: sequential over 6)
  T energy;              // sum((qfrc_actuator[-nj:] * qvel[6:])^2), numpy's pairwise order (np_sum_half)
  T ctrl_sq;             // sum(ctrl^2), numpy's pairwise order
};

// reward_functions.py:66-261 + utils.py:3-21, each expression in the reference's own association
// and without FMA contraction, so the only difference to numpy is the device libm (exp / atan2 / asin).
// The reference's Python min(a, b) is `b if b < a else a` (a NaN first operand is returned as is).
template <typename T, typename KP>
__device__ __forceinline__ T reward_formula(int reward_id, KP kn, const RewardIn<T>& in) {
#pragma clang fp contract(off)
  const T w = in.qw, x = in.qx, y = in.qy, z = in.qz;
  const T roll = atan2(T(2) * (w * x + y * z), T(1) - T(2) * (x * x + y * y));
  const T pitch = asin(T(2) * (w * y - z * x));   // not clamped: |sinp| > 1 -> NaN, as np.arcsin
  const T h = in.h;
  auto pymin = [](T a, T b) { return b < a ? b : a; };
  if (reward_id == REWARD_STAND || reward_id == REWARD_WALK) {
    const T hd = h - T(1.282);
    const T height_reward = exp(T(-2.0) * (hd * hd));
    const T orientation_reward = exp(T(-3.0) * (roll * roll + pitch * pitch));
    const T posture = T(0.5) * height_reward + T(0.5) * orientation_reward;
    const T torque = exp(T(-0.05) * in.ctrl_sq);
    if (reward_id == REWARD_STAND) {                       // :156-211
      if (h < T(0.8)) return T(0);
      const T vd = in.vx - T(1.0);
      const T vr = exp(T(-2.0) * (vd * vd));
      const T total = in.lf + in.rf + T(1e-8);
      const T foot = T(1.0) - pymin(in.lf, in.rf) / total;
      return T(0.4) * vr + T(0.3) * posture + T(0.2) * foot + T(0.1) * torque;
    }
    if (h < T(0.8)) return T(0.1) * h / T(0.8);           // :213-261
    const T vd = in.vx - T(10.0);
    const T vr = exp(T(-0.5) * (vd * vd));
    return vr + posture * torque;
  }
  if (reward_id == REWARD_KNEELING) {                      // :66-154
    // kn: target_height, min_height, max_roll_pitch, com_radius, energy_w, posture_w, com_w, foot_w, alive_w
    if (h < T(kn[1])) return h * h;
    const T mrp = T(kn[2]);
    const T orientation_error = (roll * roll + pitch * pitch) / (mrp * mrp);
    const T posture_reward = exp(T(-5.0) * orientation_error);
    const T hd = h - T(kn[0]);
    const T height_reward = exp(T(-5.0) * (hd * hd));
    const T posture = T(0.7) * posture_reward + T(0.3) * height_reward;
    const T dist = sqrt(in.com0 * in.com0 + in.com1 * in.com1);
    const T com = T(0.7) * exp(T(-10.0) * (dist / T(kn[3]))) + T(0.3) * exp(T(-0.1) * in.comv);
    const T total = in.lf + in.rf + T(1e-8);
    const T foot = pymin(in.lf, in.rf) / total;
    const T energy = exp(T(-0.01) * in.energy);
    const T alive = T(1.0) - exp(T(-0.5) * in.time);
    return T(kn[5]) * posture + T(kn[6]) * com + T(kn[7]) * foot + T(kn[4]) * energy + T(kn[8]) * alive;
  }
  return T(0);
}

// the step kernel's reward: inputs from the env's scratch.  cfrc_ext and subtree_linvel are never
// computed by mj_step without sensors (lazy), so the reference's reward reads zeros for them; with
// full_state, the real wrenches / velocity of post_constraint.
template <typename T, typename C>
__device__ __forceinline__ T compute_reward(MPtr<T> m, const Scratch<T, C>& s, KPtr<T> k, T time,
                                            T energy_sum, T ctrl_sq) {
  RewardIn<T> in;
  in.h = s.qpos[2];
  in.qw = s.qpos[3];
  in.qx = s.qpos[4];
  in.qy = s.qpos[5];
  in.qz = s.qpos[6];
  in.vx = s.qvel[0];
  in.time = time;
  in.com0 = s.com[0];
  in.com1 = s.com[1];
  in.comv = T(0);
  in.lf = T(0);
  in.rf = T(0);
  if (k->p.full_state) {
#pragma clang fp contract(off)
    for (int q = 0; q < 3; q++) in.comv += s.u.n.linv[0][q] * s.u.n.linv[0][q];
    foot_forces(m, s, in.lf, in.rf);
  }
  in.energy = energy_sum;
  in.ctrl_sq = ctrl_sq;
  return reward_formula(k->p.reward_id, k->p.kneel, in);
}

// np.sum's order (numpy pairwise_sum, n <= 128) over the values x_i held by sub-lanes off + i,
// i < n, of each 32-lane half: n < 8 -> ((0 + x0) + x1) + ...; else eight accumulators r_j = x_j +
// x_{j+8} + ... over the whole blocks of 8, combined ((r0 + r1) + (r2 + r3)) + ((r4 + r5) + (r6 + r7)),
// then the rest added in order.  The block stage and the tree are DPP (row_ror:8, permlane16 swap,
// the quad / half-mirror steps of hsum); the tail is a few lane reads.  off + n <= 32; the result is
// in every lane of the half.  (hsum's butterfly order differs from numpy's by an ulp of the sum,
// which the exp() of a reward term can amplify to several ulp of the reward.)
template <typename T>
__device__ __forceinline__ T np_sum_half(T v, int off, int n, int lane) {
#pragma clang fp contract(off)
  const int base = (lane & HL) + off;
  auto at = [&](int i) { return __shfl(v, base + i, WAVE); };
  T res;
  int i;
  if (n < 8) {
    res = T(0);
    i = 0;
  } else {
    T x = off == 0 ? v : __shfl(v, base + (lane & (HL - 1)), WAVE);   // x_j on sub-lane j
    const int nb = n - n % 8;
    T r = x;
    const T x8 = dpp<0x128>(x);                           // row_ror:8 -> x_{j+8} on sub-lanes 0..7
    if (nb >= 16) r += x8;
    if (nb >= 24) { const T t = x; r += up_row(t); }       // x_{j+16}
    if (nb >= 32) r += up_row(x8);                         // x_{j+24}
    r += dpp<0xB1>(r);                                     // r0 + r1, r2 + r3, ...
    r += dpp<0x4E>(r);                                     // (r0 + r1) + (r2 + r3), ...
    r += dpp<0x141>(r);                                    // ... + ((r4 + r5) + (r6 + r7)) on sub-lane 0
    res = bcast<0>(r);
    i = nb;
  }
  for (; i < n; i++) res += at(i);
  return res;
}

// custom_env.py:232-261 layout; qfrc_actuator comes from registers (sub-lane i holds dof i)
template <typename T, typename C, typename O>
__device__ __forceinline__ void write_obs(MPtr<T> m, const Scratch<T, C>& s, int sl, T qfa, O* out,
                          int obs_dim) {
  int nq = m->nq, nv = m->nv;
  int o1 = nq - 2, o2 = o1 + nv, o3 = o2 + 10 * m->nbody, o4 = o3 + 6 * m->nbody;
  for (int k = sl; k < o4; k += HL) {
    T v;
    if (k < o1) v = s.qpos[2 + k];
    else if (k < o2) v = s.qvel[k - o1];
    else if (k < o3) { int q = k - o2; v = s.cinert[q / 10][q % 10]; }
    else { int q = k - o3; v = s.cvel[q / 6][q % 6]; }
    out[k] = (O)v;
  }
  if (sl < nv && o4 + sl < obs_dim) out[o4 + sl] = (O)qfa;
  const int o5 = o4 + nv, nf = 6 * (m->nbody - 1);
  if (obs_dim >= o5 + nf)    // full_state: + cfrc_ext[1:] (custom_env.py:247,255, commented out there)
    for (int k = sl; k < nf; k += HL) out[o5 + k] = (O)s.u.n.cfrc[1 + k / 6][k % 6];
}

// Fused rollout: the SB3 MlpPolicy's pi net (mlp_extractor.policy_net + action_net, fp32 as SB3's
// policy) on the wave's two envs at once (the lower half-wave's env and the upper's; a ghost half
// mirrors its partner).  Hidden layers of 256: lane L (of 64) owns outputs 4L .. 4L + 3 for BOTH envs,
// so each input costs one 16-B weight load per lane (coalesced: the wave reads each weight row once)
// and two LDS broadcasts (the two envs' inputs).  The head: sub-lane sl < A of each half owns action
// sl of its half's env.  The obs rows and hidden activations are staged in each half's scratch union
// (free after the env step).  Returns the action mean of (this half's env, sub-lane sl), 0 for sl >= A.
// unroll of the hidden layers' loads (groups of 4 rows) and of the head's: measured 1 / 2 / 4 / 8 in
// profiles/ab/ab_r4u_policy_unroll.log (4 and 8 tie), a rolling 16-row ring in ab_r4ae_policy_ring.log
constexpr int kPolUnroll = 4, kPolHeadUnroll = 16;
template <typename T, typename C>
__device__ __forceinline__ float policy_mean(KPtr<T> k, const float* obs, Scratch<T, C>* smem, int lane) {
  const bool up = lane >= HL;
  const int sl = lane & (HL - 1);
  float* xa = smem[0].u.pol.x;   // lower half's env
  float* xb = smem[1].u.pol.x;   // upper half's env
  float* ha = smem[0].u.pol.h;
  float* hb = smem[1].u.pol.h;
  const int D = k->ro.D, A = k->ro.A, ld1 = k->ro.ld1;
  float* xo = up ? xb : xa;
  for (int i = sl; i < D; i += HL) xo[i] = obs[i];
  WSYNC();
  auto layer = [&](const float* w, int ld, const float* b, const float* ina, const float* inb, int n, float* outa,
                   float* outb) {
    const float4 bb = reinterpret_cast<const float4*>(b + 4 * lane)[0];
    float a[4] = {bb.x, bb.y, bb.z, bb.w}, c[4] = {bb.x, bb.y, bb.z, bb.w};
    const float* wl = w + 4 * lane;
#pragma unroll kPolUnroll
    for (int i = 0; i < n; i += 4) {
      const float4 va = *reinterpret_cast<const float4*>(ina + i);
      const float4 vb = *reinterpret_cast<const float4*>(inb + i);
      const float xs[4] = {va.x, va.y, va.z, va.w}, ys[4] = {vb.x, vb.y, vb.z, vb.w};
#pragma unroll
      for (int ii = 0; ii < 4; ii++) {
        const float4 u = *reinterpret_cast<const float4*>(wl + (size_t)(i + ii) * ld);
        a[0] += xs[ii] * u.x; a[1] += xs[ii] * u.y; a[2] += xs[ii] * u.z; a[3] += xs[ii] * u.w;
        c[0] += ys[ii] * u.x; c[1] += ys[ii] * u.y; c[2] += ys[ii] * u.z; c[3] += ys[ii] * u.w;
      }
    }
    WSYNC();   // every lane has read the inputs (the outputs may alias them)
#pragma unroll
    for (int j = 0; j < 4; j++) {
      outa[4 * lane + j] = fmaxf(a[j], 0.f);
      outb[4 * lane + j] = fmaxf(c[j], 0.f);
    }
    WSYNC();
  };
  layer(k->ro.w1, ld1, k->ro.b1, xa, xb, D, ha, hb);        // obs -> h1
  layer(k->ro.w2, 256, k->ro.b2, ha, hb, 256, xa, xb);      // h1 -> h2 (into the obs slots)
  float mean = 0.f;
  if (sl < A) {
    mean = k->ro.b3[sl];
    const float* w3 = k->ro.w3 + sl;
#pragma unroll kPolHeadUnroll
    for (int i = 0; i < 256; i++) mean += xo[i] * w3[(size_t)i * A];
  }
  return mean;
}

template <typename T, int NV, typename C>
__device__ __forceinline__ void dump_debug(const Stepper<T, NV, C>& st, T* dbg) {
  const Scratch<T, C>& s = st.s;
  int sl = st.sl;
  for (int k = sl; k < MAXBODY * 10; k += HL) dbg[200 + k] = s.cinert[k / 10][k % 10];
  for (int k = sl; k < MAXDOF * 6; k += HL) dbg[500 + k] = s.cdof[k / 6][k % 6];
  if (sl < NV)
    for (int j = 0; j < NV; j++) dbg[700 + sl * MAXDOF + j] = st.Mr[j];
  for (int k = sl; k < MAXBODY * 6; k += HL) dbg[1800 + k] = s.cvel[k / 6][k % 6];
  if (sl < NV) {
    dbg[2280 + sl] = st.qfa;
    dbg[2320 + sl] = st.fsmooth;
    dbg[2360 + sl] = st.fcon;
    dbg[2400 + sl] = st.qacc;
  }
  if (sl == 0) {
    dbg[2500] = s.com[0]; dbg[2501] = s.com[1]; dbg[2502] = s.com[2];
    dbg[2503] = s.ncon; dbg[2504] = s.nefc; dbg[2505] = st.niter; dbg[2506] = s.nlim;
  }
  for (int c = sl; c < s.ncon; c += HL) {
    T* o = dbg + 2600 + 11 * c;
    for (int k = 0; k < 3; k++) { o[k] = s.con_pos[c][k]; o[3 + k] = s.con_n[c][k]; o[6 + k] = s.con_t1[c][k]; }
    o[9] = s.con_dist[c];
    o[10] = s.con_pair[c];
  }
  for (int r = sl; r < s.nefc; r += HL) {
    T* o = dbg + 4000 + 6 * r;     // contacts above end at 2600 + 11 * 64
    o[0] = rk_kind(s.row_kid[r]); o[1] = rk_id(s.row_kid[r]); o[2] = s.row_D[r]; o[4] = s.row_f[r];
  }
}

// per-env commit of state (+ the optional aux row / ctrl copy) for one half-wave
template <typename T, int NV, typename C>
__device__ __forceinline__ void commit(MPtr<T> m, KPtr<T> k, const Stepper<T, NV, C>& st,
                       int env, T time, T xws, int step_count, uint32_t episode, T total, const int* warn,
                       bool full) {
  const Scratch<T, C>& s = st.s;
  const int sl = st.sl, nq = m->nq, nv = m->nv, nu = m->nu;
  const int outputs = k->p.outputs;
  if (sl < nq) k->b.qpos[(size_t)env * nq + sl] = s.qpos[sl];
  if (sl + HL < nq) k->b.qpos[(size_t)env * nq + sl + HL] = s.qpos[sl + HL];
  if (sl < nv) {
    k->b.qvel[(size_t)env * nv + sl] = s.qvel[sl];
    k->b.qacc_ws[(size_t)env * nv + sl] = xws;
    if (outputs & OUT_AUX) k->b.aux[(size_t)env * AUXDIM + sl] = st.qacc;
  }
  // data.ctrl: always for resets and raw physics calls (rare); for env steps only with OUT_CTRL
  // (the host marks the buffer stale otherwise, hs_api.cpp)
  if (sl < nu && ((outputs & OUT_CTRL) || k->p.mode != MODE_ENV_STEP)) k->b.ctrl[(size_t)env * nu + sl] = s.ctrl[sl];
  if (sl == 0) {
    k->b.time[env] = time;
    k->b.step_count[env] = step_count;
    k->b.episode[env] = episode;
    k->b.total_reward[env] = total;
    if (outputs & OUT_AUX) {
      T* a = k->b.aux + (size_t)env * AUXDIM;
      a[MAXDOF + 0] = s.com[0]; a[MAXDOF + 1] = s.com[1]; a[MAXDOF + 2] = s.com[2];
      a[MAXDOF + 3] = (T)s.ncon; a[MAXDOF + 4] = (T)s.nefc; a[MAXDOF + 5] = (T)st.niter;
    }
    for (int w = 0; w < NWARN; w++)   // read-modify-write only when set (a load here would wait for
      if (warn[w]) k->b.warning[(size_t)env * NWARN + w] += warn[w];   // every store issued above)
  }
  if (full) {   // data.cfrc_ext / data.subtree_linvel of the last substep (pre-integration)
    const int nb = m->nbody;
    for (int q = sl; q < 6 * nb; q += HL) k->b.cfrc_ext[(size_t)env * 6 * nb + q] = s.u.n.cfrc[q / 6][q % 6];
    for (int q = sl; q < 3 * nb; q += HL) k->b.subtree_linvel[(size_t)env * 3 * nb + q] = s.u.n.linv[q / 3][q % 3];
  }
}

// ------------------------------------------------------------------ the kernel
// One env step (or reset / raw physics call) of the env pair (index, index + 1) of one wave.
// `list` (wide tier): indices map to env ids through it; resident tier: indices are env ids.
// In the resident tier an env whose contacts / rows overflowed the resident capacity in any
// substep is NOT committed: it is appended to the wide tier's work list instead, and the wide
// launch that follows re-runs its whole step from the same (untouched) inputs.
// Queued schedule (launch_step sets p.queue when the pairs outnumber the resident waves): the
// pair's substeps [s0, s1) only.  A chunk that ends before the last substep hands the state over
// through b.mid and sets the pair's flag := this launch's tag; the last-substep chunk waits for the
// tag and starts from that row.  b.mid and the flags live in UNCACHED device memory (hs_api.cpp; its
// blocks are recycled only as uncached memory), so the stores are in memory once `s_waitcnt
// vmcnt(0)` returns and the consumer's loads cannot hit a stale L1 / L2 line: no cache invalidate or
// write-back on either side.  Every chunk recomputes the whole mj_step pipeline from (qpos, qvel,
// qacc_warmstart, time), so the hand-off is exact: results are bitwise those of one wave running all
// substeps.
// ghost: this half-wave mirrors env idx (the single-env schedule's upper half) and commits nothing.
template <typename T, int NV, bool PGS, typename C, bool ROLL = false>
__device__ __forceinline__ void step_pair(KPtr<T> ka, Scratch<T, C>* smem, PgsCache<T, C>* pcache, int idx,
                                          int nidx, const int* list, int s0, int s1, int pair, bool ghost = false,
                                          int wait_tag = 0, int set_tag = 0, int tstep = 0, bool tape_launch = false) {
  constexpr bool WIDE = C::WIDE;
  const int lane = opaque_v(threadIdx.x);   // (no lane-derived value hoisted out of the chunk-queue loop)
  const bool up = lane >= HL;
  const int sl = lane & (HL - 1);
  bool active = idx < nidx && !ghost;                 // ghost half: odd count, or the single-env schedule
  const int ei = idx < nidx ? idx : nidx - 1;
  const int env_id = list ? list[ei] : ei;
  const int mode = ka->p.mode;
  if (mode == MODE_RESET && ka->reset_mask && !ka->reset_mask[env_id]) active = false;
  if (__ballot(active) == 0) return;                  // wave-uniform exit
  const bool real = active;                           // this half steps (and commits) a real env
  // fused rollout (fp64 engine): the episode return so far and the step's done flag, carried to the
  // policy forward after the step; the action of steps after the launch's first comes in the row
  const bool rollout = ROLL && ka->ro.obs != nullptr;
  double epacc = 0.0;
  bool rdone = false;
  T act_row = T(0);
  Scratch<T, C>& s = smem[up ? 1 : 0];
  MPtr<T> m = ka->m;
  const int nq = m->nq, nv = m->nv, nu = m->nu;
  Stepper<T, NV, C> st(m, s, lane);
  if (ka->b.dbg && env_id == 0 && active) st.dbg = ka->b.dbg;
  int warn[NWARN] = {0, 0, 0, 0, 0};
  T time, xws;
  int step_count;
  uint32_t episode;
  T total, act;
  {
    if (wait_tag != 0) {   // queued: wait for the pair's previous chunk (or tape step) to hand the state over
      int* flag = ka->b.qsync + QS_FLAG + pair;
      int seen = 0, abort = 0;
      if (lane == 0) {   // bounded (~0.5 s): a broken hand-off must not hang the GPU
        int w = 0;
        if (pair + 1 != ka->p.dbg_lose_pair1)   // test hook: treat this unit's hand-off as lost
          while ((seen = __hip_atomic_load(flag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) != wait_tag &&
                 ++w < (1 << 22)) {
            // a tape launch that aborted (overflow) never hands this pair over: leave at once
            if (tstep > 0 && (abort = __hip_atomic_load(ka->b.qsync + QS_ABORT, __ATOMIC_RELAXED,
                                                        __HIP_MEMORY_SCOPE_AGENT)) != 0)
              break;
            __builtin_amdgcn_s_sleep(2);
          }
      }
      if (__builtin_amdgcn_readfirstlane(abort) != 0) return;   // results discarded: the host replays
      const bool lost = __builtin_amdgcn_readfirstlane(seen) != wait_tag;
      WSYNC();   // (compiler order: the row loads stay behind the poll)
      const T* r = ka->b.mid + (size_t)env_id * MIDDIM;
      time = row_ld(r + MID_TIME);
      xws = (sl < nv) ? row_ld(r + MID_WS + sl) : T(0);
      if (sl < nq) s.qpos[sl] = row_ld(r + MID_Q + sl);
      if (sl + HL < nq) s.qpos[sl + HL] = row_ld(r + MID_Q + sl + HL);
      if (sl < nv) s.qvel[sl] = row_ld(r + MID_V + sl);
#pragma unroll
      for (int w = 0; w < NWARN; w++) warn[w] = (int)row_ld(r + MID_W + w);
      step_count = (int)row_ld(r + MID_SC);
      episode = (uint32_t)row_ld(r + MID_EP);
      total = row_ld(r + MID_TOT);
      if (rollout) {
        if (sl < nu) act_row = row_ld(r + MID_ACT + sl);
        epacc = (double)row_ld(r + MID_EPACC);
      }
      // never seen in practice; if it were, the state is poisoned so that the substep's mj_checkPos
      // resets the env (mj_resetData, ctrl 0 for that substep) -- counted in its own slot,
      // HS_WARN_HANDOFF, not as a bad state (the -1 cancels the HS_WARN_BADQPOS count the poisoned
      // qpos draws); the trainer raises on it: loud, never silent
      if (lost) {
        warn[WARN_HANDOFF]++;
        warn[WARN_BADQPOS]--;
        if (sl == 2) s.qpos[2] = T(NAN);
      }
    } else {
      time = ka->b.time[env_id];
      xws = (sl < nv) ? ka->b.qacc_ws[(size_t)env_id * nv + sl] : T(0);
      if (sl < nq) s.qpos[sl] = ka->b.qpos[(size_t)env_id * nq + sl];
      if (sl + HL < nq) s.qpos[sl + HL] = ka->b.qpos[(size_t)env_id * nq + sl + HL];
      if (sl < nv) s.qvel[sl] = ka->b.qvel[(size_t)env_id * nv + sl];
      step_count = ka->b.step_count[env_id];
      episode = ka->b.episode[env_id];
      total = ka->b.total_reward[env_id];
      if (rollout) epacc = ka->ro.ep_acc[env_id];
    }
    // data.ctrl is an input only to a raw physics call that keeps the current ctrl; env steps set
    // it from the action, resets zero it
    const float* actions = ka->actions;
    if (sl < nu) s.ctrl[sl] = (mode == MODE_PHYSICS && !actions) ? ka->b.ctrl[(size_t)env_id * nu + sl] : T(0);
    // the action is the same for all substeps: one load, issued with the state loads (a tape
    // launch's step tstep reads its own [N][nu] slice)
    // (a rollout's `actions` is its first step's, ro.act_clip; later steps' come in the row)
    act = (rollout && tstep > 0) ? act_row
        : (actions && sl < nu) ? (T)actions[((size_t)tstep * ka->nenv + env_id) * nu + sl] : T(0);
  }
  WSYNC();
  st.clk.start();
  st.qfa = 0;
  st.qacc = 0;
  st.niter = 0;
  // resident tier: an overflowing env is deferred to the wide tier instead of committed
  auto defer = [&](KPtr<T> k) -> bool {
    if constexpr (WIDE) {
      return false;
    } else {
      if (!k->b.redo || warn[WARN_OVERFLOW] == 0) return false;
      if (sl == 0) {
        const int slot = atomicAdd(&k->b.redo[0], 1);
        k->b.redo[2 + slot] = env_id;
        atomicAdd(k->b.redo_total, 1ull);
      }
      return true;
    }
  };
  // Tape launch (set_tag on a whole-step item): the state goes on to the pair's next env step only
  // through its hand-off row (uncached), together with the warning counters accumulated so far.
  // Only the tape's LAST step commits to the batch buffers: consecutive steps of one env may run on
  // different XCDs, whose L2s are not coherent with each other, so two steps writing the same
  // batch address would leave whichever dirty line is written back last.  For the same reason the
  // batch's obs / reward / done rows are written by the last step only when the tape has no
  // per-step outputs, and the host keeps each env to at most one finished episode per tape launch
  // (hs_step_tape), so its terminal obs / info rows are written once.
  const bool tape_handoff = set_tag != 0 && s1 == ka->p.nsub;
  const bool tape_final = !(ka->p.nsteps > 1 && tstep < ka->p.nsteps - 1);
  bool deferred = false;
  auto handoff = [&](KPtr<T> k, int env, T time_, T xws_, int sc, uint32_t ep, T tot) {
    T* r = k->b.mid + (size_t)env * MIDDIM;
    if (sl < nq) row_st(r + MID_Q + sl, s.qpos[sl]);
    if (sl + HL < nq) row_st(r + MID_Q + sl + HL, s.qpos[sl + HL]);
    if (sl < nv) { row_st(r + MID_V + sl, s.qvel[sl]); row_st(r + MID_WS + sl, xws_); }
    if (sl == 0) {
      row_st(r + MID_TIME, time_);
#pragma unroll
      for (int w = 0; w < NWARN; w++) row_st(r + MID_W + w, (T)warn[w]);
      row_st(r + MID_SC, (T)sc);
      row_st(r + MID_EP, (T)ep);
      row_st(r + MID_TOT, tot);
    }
  };
  // this env step's output rows: the tape's slice tstep, or the batch's own buffers (null: an
  // intermediate step of a tape launch without per-step outputs writes none)
  auto obs_row = [&](KPtr<T> k, int env, int obs_dim) -> T* {
    if (k->tape.obs) return k->tape.obs + ((size_t)tstep * k->nenv + env) * obs_dim;
    return tape_final ? k->b.obs + (size_t)env * obs_dim : nullptr;
  };
  // fused rollout: the rollout buffer's obs row of step g + 1 (the obs this step returns)
  auto ro_next_obs = [&](KPtr<T> k, int env) -> float* {
    const int g = k->ro.t_begin + tstep;
    return g + 1 < k->ro.t_total ? k->ro.obs + ((size_t)(g + 1) * k->nenv + env) * k->ro.D
                                 : k->ro.obs_last + (size_t)env * k->ro.D;
  };

  // Both halves always run the same instruction stream; a half that is inactive (ghost env,
  // masked reset) or not resetting while its partner resets computes on scratch but commits
  // nothing (its real state was committed before the shared reset pass).
  bool do_reset = mode == MODE_RESET && active;
  const int nsub = (mode == MODE_RESET) ? 0 : ka->p.nsub;
  bool in_reset = false;
#ifdef HS_TIMING
  int tot_iter = 0;
  const int titem = (ka->p.queue ? (s0 > 0 ? (nidx + 1) / 2 : 0) + pair : -1);
#endif
  // One loop, ONE inlined physics_step call site: substeps 0..nsub-1 apply the action; after the
  // last one the env bookkeeping runs; if any half of the wave must reset, one more substep
  // runs with the reset state (a half that is not resetting has already committed and computes
  // on scratch only).  Launch arguments are re-read through k = opaque(ka) at each use.
  for (int sub = s0;; sub++) {
    st.m = opaque(st.m);
    st.sl = opaque_v(st.sl);
    const int env = opaque_v(env_id);   // per-env addresses recomputed at each use, not kept live
    if (sub == s1 && s1 < nsub) {         // queued chunk ends before the last substep: hand over
      KPtr<T> k = opaque(ka);
      if (active) {
        T* r = k->b.mid + (size_t)env * MIDDIM;
        if (sl < nq) row_st(r + MID_Q + sl, s.qpos[sl]);
        if (sl + HL < nq) row_st(r + MID_Q + sl + HL, s.qpos[sl + HL]);
        if (sl < nv) { row_st(r + MID_V + sl, s.qvel[sl]); row_st(r + MID_WS + sl, xws); }
        if (sl == 0) {
          row_st(r + MID_TIME, time);
#pragma unroll
          for (int w = 0; w < NWARN; w++) row_st(r + MID_W + w, (T)warn[w]);
          row_st(r + MID_SC, (T)step_count);
          row_st(r + MID_EP, (T)episode);
          row_st(r + MID_TOT, total);
        }
      }
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // the row is in memory before the flag is
      if (lane == 0) __hip_atomic_store(k->b.qsync + QS_FLAG + pair, set_tag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      HS_FLUSH();
      break;
    }
    if (sub == nsub && !in_reset) {
      if (nsub > 0) {
        KPtr<T> k = opaque(ka);
        const int obs_dim = k->p.obs_dim;
        HS_STAMP(st.clk, 22);
        T* orow = obs_row(k, env, obs_dim);
        if (active && orow) write_obs(st.m, s, sl, st.qfa, orow, obs_dim);
        HS_STAMP(st.clk, 23);
        if (k->p.mode == MODE_ENV_STEP) {
          step_count += 1;
          bool trunc = step_count >= k->p.max_steps;
          // np.sum(np.square(qfrc_actuator[-nj:] * qvel[6:])) and np.sum(np.square(ctrl)) in numpy's order
          // (each sum only for the reward that reads it: kneeling the energy, stand / walk the torque;
          // the launch's reward id is wave-uniform)
          const int rid = opaque(k)->p.reward_id;
          const T e = sl < nv ? st.qfa * s.qvel[sl] : T(0);
          const T esum = rid == REWARD_KNEELING ? np_sum_half(e * e, 6, nv - 6, lane) : T(0);
          const T cu = sl < st.m->nu ? s.ctrl[sl] : T(0);
          const T csum = (rid == REWARD_STAND || rid == REWARD_WALK) ? np_sum_half(cu * cu, 0, st.m->nu, lane) : T(0);
          HS_STAMP(st.clk, 24);
          T r = trunc ? T(0) : compute_reward(st.m, s, k, time, esum, csum);
          HS_STAMP(st.clk, 25);
          total += r;
          bool term = (double)time >= k->p.duration;
          if (sl == 0 && active && (k->tape.reward || tape_final)) {
            const size_t o = k->tape.reward ? (size_t)tstep * k->nenv : 0;
            (k->tape.reward ? k->tape.reward : k->b.reward)[o + env] = r;
            (k->tape.terminated ? k->tape.terminated : k->b.terminated)[o + env] = term;
            (k->tape.truncated ? k->tape.truncated : k->b.truncated)[o + env] = trunc;
          }
          // the final step's info of a finished episode (SubprocVecEnv returns its step_count /
          // total_reward before resetting, custom_env.py:216-224), with or without auto-reset
          if ((term || trunc) && active && sl == 0) {
            if (k->b.term_step_count) k->b.term_step_count[env] = step_count;
            if (k->b.term_total_reward) k->b.term_total_reward[env] = total;
          }
          // fused rollout: SB3 collect_rollouts' bookkeeping of this step (ppo_post_kernel): reward and
          // done rows, the episode return, TimeLimit.truncated envs' terminal obs for the bootstrap,
          // and the returned obs (an env that auto-resets returns its reset obs, written below)
          if (rollout && active) {
            const float rf = (float)r;
            const double acc = epacc + (double)rf;
            rdone = term || trunc;
            const size_t gi = (size_t)(k->ro.t_begin + tstep) * k->nenv + env;
            if (sl == 0) {
              k->ro.rew[gi] = rf;
              k->ro.done[gi] = rdone;
              k->ro.epret[gi] = acc;
              k->ro.boot[gi] = trunc && !term;
            }
            epacc = rdone ? 0.0 : acc;
            if (trunc && !term) write_obs(st.m, s, sl, st.qfa, k->ro.tobs + gi * obs_dim, obs_dim);
            if (!rdone) write_obs(st.m, s, sl, st.qfa, ro_next_obs(k, env), obs_dim);
          }
          if ((term || trunc) && k->p.autoreset && active) {
            write_obs(st.m, s, sl, st.qfa, k->b.terminal_obs + (size_t)env * obs_dim, obs_dim);
            do_reset = true;
          }
        }
        if (active && !do_reset) {
          if (!defer(k)) {
            if (tape_final) commit(st.m, k, st, env, time, xws, step_count, episode, total, warn, k->p.full_state != 0);
            if (tape_handoff) handoff(k, env, time, xws, step_count, episode, total);
          } else {
            deferred = true;
          }
          active = false;   // committed (or deferred); a reset pass below is scratch work for this half
        }
      }
      if (__ballot(do_reset) == 0) { HS_FLUSH(); break; }
      // custom_env.py:97-130: mj_resetData; qpos = init (z=1.282, upright); += U(+-0.01) noise
      // with z noise x0.1 and no quaternion noise; qvel = U(+-0.01); one mj_step with ctrl = 0.
      KPtr<T> k = opaque(ka);
      in_reset = true;
      st.dbg = nullptr;
      T sc = (T)k->p.noise_scale;
      const uint64_t seed = k->p.seed;
      const T* nz_q = k->nz_q;
      const T* nz_v = k->nz_v;
      uint32_t ep = episode + 1;
      for (int q = sl; q < nq; q += HL) {
        T v = m->qpos0[q];
        T nzq = nz_q ? nz_q[(size_t)env * nq + q] : uniform_pm<T>(seed, env, ep, q, sc);
        if (m->jnt_type[0] == JNT_FREE) {
          if (q == 2) { v = (T)k->p.init_height; nzq *= T(0.1); }
          if (q >= 3 && q < 7) { v = q == 3 ? T(1) : T(0); nzq = 0; }
        }
        s.qpos[q] = v + nzq;
      }
      if (sl < nv) s.qvel[sl] = nz_v ? nz_v[(size_t)env * nv + sl] : uniform_pm<T>(seed, env, ep, 64 + sl, sc);
      if (sl < nu) s.ctrl[sl] = 0;
      xws = 0;
      time = 0;
      episode = ep;
      WSYNC();
    } else if (sub > nsub) {
      if (do_reset && active) {
        KPtr<T> k = opaque(ka);
        if (k->b.dbg && env == 0) dump_debug(st, k->b.dbg);
        const int obs_dim = k->p.obs_dim;
        T* orow = obs_row(k, env, obs_dim);
        if (orow) write_obs(st.m, s, sl, st.qfa, orow, obs_dim);
        if (rollout) write_obs(st.m, s, sl, st.qfa, ro_next_obs(k, env), obs_dim);   // the reset obs
        if (!defer(k)) {
          if (tape_final) commit(st.m, k, st, env, time, xws, 0, episode, T(0), warn, k->p.full_state != 0);
          if (tape_handoff) handoff(k, env, time, xws, 0, episode, T(0));
        } else {
          deferred = true;
        }
      }
      HS_FLUSH();
      break;
    } else {
      // data.ctrl[:] = action each substep (custom_env.py:159); mj_resetData may have zeroed it
      if (sl < nu && opaque(ka)->actions) s.ctrl[sl] = act;
      WSYNC();
    }
    physics_step<T, NV, PGS>(st, ka, time, xws, warn, pcache);
#ifdef HS_TIMING
    tot_iter += st.niter;
#endif
    if (st.dbg && active && !in_reset) dump_debug(st, st.dbg);
  }
  if constexpr (ROLL) {
    if (rollout) {   // the policy acts on the step's obs: step g + 1's action, drawn as ppo_act_kernel does
      KPtr<T> k = opaque(ka);
      const int g = k->ro.t_begin + tstep, N = k->nenv, A = k->ro.A;
      const bool last_of_launch = tstep == k->p.nsteps - 1;
      T* r = k->b.mid + (size_t)env_id * MIDDIM;
      if (g + 1 < k->ro.t_total) {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // this wave's obs row is written before it is read
        const float mean = policy_mean(k, k->ro.obs + ((size_t)(g + 1) * N + env_id) * k->ro.D, smem, lane);
        const float ls = sl < A ? k->ro.log_std[sl] : 0.f;
        float z = 0.f;
        if (!k->ro.deterministic && sl < A)
          z = policy_noise((uint32_t)env_id, (uint32_t)sl, (uint64_t)(g + 1) + *k->ro.ctr_base, k->ro.k0, k->ro.k1);
        const float a = mean + __expf(ls) * z;
        const float lp = half_sum(sl < A ? -0.5f * z * z - ls - 0.91893853320467274f : 0.f);
        if (real) {
          const size_t gi = (size_t)(g + 1) * N + env_id;
          if (sl < A) {
            const float ac = fminf(fmaxf(a, -1.f), 1.f);
            k->ro.act[gi * A + sl] = a;
            if (last_of_launch) k->ro.act_clip[(size_t)env_id * A + sl] = ac;
            else row_st(r + MID_ACT + sl, (T)ac);
          }
          if (sl == 0) {
            k->ro.logp[gi] = lp;
            k->ro.start[gi] = rdone ? 1.f : 0.f;
          }
        }
      }
      // the rollout's last step: act_clip ends as the action that step ran with (as the per-step path)
      if (real && last_of_launch && g + 1 >= k->ro.t_total && sl < A) k->ro.act_clip[(size_t)env_id * A + sl] = (float)act;
      if (real && sl == 0) {
        if (last_of_launch) {
          k->ro.ep_acc[env_id] = epacc;
          k->ro.episode_start[env_id] = rdone ? 1.f : 0.f;
        } else {
          row_st(r + MID_EPACC, (T)epacc);
        }
      }
    }
  }
  // A tape launch never runs the wide tier, so an env deferred on ANY of its steps -- the last one
  // included, which hands nothing over -- stops the launch: the host restores the saved state and
  // replays the tape step by step (hs_api.cpp guarded_tape).  Otherwise the pair's next env step may
  // start: rows in memory, then the flag.
  if (tape_handoff || tape_launch) {
    KPtr<T> k = opaque(ka);
    const bool any_deferred = __ballot(deferred) != 0;
    if (tape_handoff || any_deferred) {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      if (lane == 0) {
        if (any_deferred)
          __hip_atomic_store(k->b.qsync + QS_ABORT, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        else
          __hip_atomic_store(k->b.qsync + QS_FLAG + pair, set_tag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
    }
  }
}

// Resident tier: one wave per env pair, all pairs of the batch in one grid.
// 2 waves/SIMD (the VGPR budget of 256) for the fp32 engine; the fp64 parity engine needs more
// registers and runs at 1.  PGS: the <option solver="PGS"> instance (its own LDS cache).
template <typename T, int NV, bool PGS>
__global__ __launch_bounds__(64, (sizeof(T) == 4 && !PGS) ? 2 : 1) void step_kernel(KArgs<T> /* read via kernarg ptr */) {
  __shared__ Scratch<T, Resident<T>> smem[2];
  PgsCache<T, Resident<T>>* pcache = nullptr;
  if constexpr (PGS) {
    __shared__ PgsCache<T, Resident<T>> pgs_smem[2];
    pcache = &pgs_smem[threadIdx.x >= HL ? 1 : 0];
  }
  const KPtr<T> ka = (KPtr<T>)__builtin_amdgcn_kernarg_segment_ptr();
  const bool up = threadIdx.x >= HL;
  // single-env schedule (small batches, p.single): env blockIdx.x on the lower half, its mirror on
  // the upper half (same data, so the same control flow), one env per wave
  const bool single = ka->p.single != 0;
  step_pair<T, NV, PGS, Resident<T>>(ka, smem, pcache, single ? (int)blockIdx.x : 2 * blockIdx.x + (up ? 1 : 0),
                                     ka->nenv, nullptr, 0, ka->p.nsub, blockIdx.x, single && up);
}

// Resident tier, chunk-queue schedule (launch_step picks it when the env pairs outnumber the waves
// the GPU holds at once -- the fp64 engine at 1 wave per SIMD -- for multi-substep calls).  A
// persistent grid claims items from one counter: first every pair's substeps [0, nsub - 1), then
// every pair's last substep (+ obs / reward / auto-reset), so the launch ends on short items
// instead of a second generation of whole env steps.  Pairs are taken heaviest
// first by the durations the previous queued launch measured (QNB cost buckets, hs_kernels.h), so
// the launch ends on the cheapest last substeps; the batch's first queued launch uses a fixed
// multiplicative permutation (p.qmul).  The order only decides which wave runs which pair when:
// results are bitwise the same in any order.  Items are claimed only by running waves and a
// last-substep item waits only on its own pair's first chunk, claimed npairs items earlier by a
// running wave: no residency can deadlock it.
// ROLL: the fused-rollout instance (fp64 Newton engine; launch_step picks it for hs_rollout), so the
// policy forward's code and registers stay out of the per-step kernel
template <typename T, int NV, bool PGS, bool ROLL = false>
__global__ __launch_bounds__(64, 1) void step_kernel_queue(KArgs<T> /* read via kernarg ptr */) {
  const KPtr<T> ka = (KPtr<T>)__builtin_amdgcn_kernarg_segment_ptr();
  // this launch's epoch (its hand-off tags are qtag(epoch, ...)): the epoch only changes after every
  // wave of the launch has left the claim loop (last wave out, below)
  const uint32_t epoch = __builtin_amdgcn_readfirstlane(
      __hip_atomic_load(ka->b.qsync + QS_EPOCH, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
  __shared__ Scratch<T, Resident<T>> smem[2];
  PgsCache<T, Resident<T>>* pcache = nullptr;
  if constexpr (PGS) {
    __shared__ PgsCache<T, Resident<T>> pgs_smem[2];
    pcache = &pgs_smem[threadIdx.x >= HL ? 1 : 0];
  }
  // claim order: prefix sums of the previous launch's bucket counts (qpre[QNB] == nunits: valid).
  // A unit is an env pair, or one env (upper half-wave a ghost) in the single-env mode of small
  // batches (p.single: every env gets a wave of its own)
  __shared__ int qpre[QNB + 1];
  {
    const int nunits = ka->p.single ? ka->nenv : (ka->nenv + 1) / 2, lane = threadIdx.x;
    int c = (ka->p.qorder && lane < QNB) ? ka->b.qsync[qs_cnt(nunits, epoch & 1) + lane] : 0;
#pragma unroll
    for (int d = 1; d < QNB; d <<= 1) {
      const int y = __shfl_up(c, d);
      if (lane >= d) c += y;
    }
    if (lane < QNB) qpre[lane + 1] = c;
    if (lane == 0) qpre[0] = 0;
    WSYNC();
  }
  for (;;) {
    const KPtr<T> k = opaque(ka);       // nothing uniform kept live across items
    const bool single = k->p.single != 0;
    const int nsub = k->p.nsub, npairs = single ? k->nenv : (k->nenv + 1) / 2, K = k->p.nsteps;   // (units)
    int* qs = k->b.qsync;
    int i = 0;
    if (threadIdx.x == 0) i = atomicAdd(&qs[QS_HEAD], 1);
    i = __builtin_amdgcn_readfirstlane(i);
    // tape launch: K whole env steps per pair, step-major (step t of every pair, then step t + 1);
    // one env step: every pair's first chunk, then every pair's last substep
    const bool tape = K > 1 || k->ro.obs != nullptr;   // (a fused rollout is a tape launch even for K = 1)
    if (i >= (tape ? K * npairs : 2 * npairs)) break;
    if (tape) {   // an aborted tape launch only drains its claims
      int ab = 0;
      if (threadIdx.x == 0) ab = __hip_atomic_load(qs + QS_ABORT, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      if (__builtin_amdgcn_readfirstlane(ab) != 0) continue;
    }
    const int t = tape ? i / npairs : 0;
    const bool last = !tape && i >= npairs;
    const int ii = tape ? i - t * npairs : (last ? i - npairs : i);
    int pair;
    if (qpre[QNB] == npairs) {   // bucket b holds claims [qpre[b], qpre[b + 1])
      const int lane = opaque_v(threadIdx.x);
      const bool hit = lane < QNB && qpre[lane] <= ii && ii < qpre[lane + 1];
      const int b = __builtin_ctzll(__ballot(hit) | (1ull << (QNB - 1)));
      int p = 0;
      if (lane == 0) p = qs[qs_ord(npairs, epoch & 1) + (size_t)b * npairs + (ii - qpre[b])];
      pair = min(max(__builtin_amdgcn_readfirstlane(p), 0), npairs - 1);
    } else {
      pair = (int)((uint64_t)ii * (uint32_t)k->p.qmul % (uint32_t)npairs);
    }
    const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
    const bool upper = opaque_v(threadIdx.x) >= HL;
    const int env = single ? pair : 2 * pair + (upper ? 1 : 0);
    // ONE step_pair call site (the whole pipeline is inlined): a tape item is env step t, waiting for
    // the pair's step t - 1 and handing over to its step t + 1; otherwise the first chunk hands over
    // to the last substep
    const int s0 = last ? nsub - 1 : 0, s1 = (tape || last) ? nsub : nsub - 1;
    const int wait_tag = tape ? (t > 0 ? qtag(epoch, t - 1, 1) : 0) : (last ? qtag(epoch, 0, 0) : 0);
    const int set_tag = tape ? (t < K - 1 ? qtag(epoch, t, 1) : 0) : (last ? 0 : qtag(epoch, 0, 0));
    step_pair<T, NV, PGS, Resident<T>, ROLL>(k, smem, pcache, env, k->nenv, nullptr, s0, s1, pair, single && upper,
                                             wait_tag, set_tag, t, tape);
    // the pair's duration for the next launch's order: the first chunk's is kept in qcost (its
    // store trails the hand-off, but the last substep reads it ~100 us later; a stale value only
    // makes the order less exact, never the results different); a tape launch times the pair's
    // last env step
    const uint32_t d = (uint32_t)(__builtin_amdgcn_s_memrealtime() - t0);
    if (threadIdx.x == 0) {
      qs = opaque(ka)->b.qsync;
      if (!last && !tape) {
        qs[qs_cost(npairs) + pair] = (int)d;
      } else if (!tape || t == K - 1) {
        const uint32_t tot = tape ? d : d + (uint32_t)qs[qs_cost(npairs) + pair];
        const int b = QNB - 1 - (int)min(tot / (uint32_t)QBIN, (uint32_t)(QNB - 1));
        const int slot = atomicAdd(&qs[qs_cnt(npairs, (epoch + 1) & 1) + b], 1);
        qs[qs_ord(npairs, (epoch + 1) & 1) + (size_t)b * npairs + slot] = pair;
      }
    }
  }
  // the last wave out resets the counters, clears the bucket counts this launch read, and advances
  // the epoch for the next launch (every wave has made its final claim and read this launch's tag)
  int* qs = ka->b.qsync;
  int lastout = 0;
  if (threadIdx.x == 0) lastout = atomicAdd(&qs[QS_EXIT], 1) == (int)gridDim.x - 1;
  if (__builtin_amdgcn_readfirstlane(lastout)) {
    const int nunits = ka->p.single ? ka->nenv : (ka->nenv + 1) / 2;
    if (threadIdx.x < QNB) qs[qs_cnt(nunits, epoch & 1) + threadIdx.x] = 0;
    if (threadIdx.x == 0) {
      qs[QS_HEAD] = 0;
      qs[QS_EXIT] = 0;
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    if (threadIdx.x == 0) atomicAdd(&qs[QS_EPOCH], 1);
  }
}

// Wide tier: a small grid that strides over the envs the resident launch deferred (usually none:
// every wave reads the count and leaves), then the last wave out clears the list for the next step.
template <typename T, int NV, bool PGS>
__global__ __launch_bounds__(64, 1) void step_kernel_wide(KArgs<T> /* read via kernarg ptr */) {
  __shared__ Scratch<T, Wide> smem[2];
  PgsCache<T, Wide>* pcache = nullptr;
  if constexpr (PGS) {
    __shared__ PgsCache<T, Wide> pgs_smem[2];
    pcache = &pgs_smem[threadIdx.x >= HL ? 1 : 0];
  }
  const KPtr<T> ka = (KPtr<T>)__builtin_amdgcn_kernarg_segment_ptr();
  int* redo = ka->b.redo;
  const int count = redo[0];
  // nothing deferred (the usual case): every wave reads 0 and leaves; the list and its read counter
  // are already clear, so no fence and no atomic (32 of them on one word cost ~2 us per launch)
  if (count == 0) return;
  for (int base = 2 * blockIdx.x; base < count; base += 2 * gridDim.x)
    step_pair<T, NV, PGS, Wide>(ka, smem, pcache, base + (threadIdx.x >= HL ? 1 : 0), count, redo + 2, 0,
                                ka->p.nsub, 0);
  __threadfence();
  if (threadIdx.x == 0 && atomicAdd(&redo[1], 1) == (int)gridDim.x - 1) {   // every wave has read the list
    redo[0] = 0;
    redo[1] = 0;
  }
}

// mj_kinematics + mj_comPos of ONE state (visualisation / data view, never the step path): one
// wave, the lower half-wave computes, the upper half duplicates it.  out = [xpos MAXBODY*3]
// [xmat MAXBODY*9][geom_xpos MAXGEOM*3][geom z-axis MAXGEOM*3][subtree_com[0] 3].
template <typename T, int NV>
__global__ __launch_bounds__(64) void kin_kernel(MPtr<T> m, const T* __restrict__ qpos, T* __restrict__ out) {
  __shared__ Scratch<T, Resident<T>> smem[2];
  const int lane = threadIdx.x;
  const bool up = lane >= HL;
  const int sl = lane & (HL - 1);
  Scratch<T, Resident<T>>& s = smem[up ? 1 : 0];
  for (int k = sl; k < m->nq; k += HL) s.qpos[k] = qpos[k];
  WSYNC();
  Stepper<T, NV, Resident<T>> st(m, s, lane);
  st.kinematics();
  if (up) return;
  const int nb = m->nbody, ng = m->ngeom;
  for (int k = sl; k < nb * 3; k += HL) out[k] = s.u.k.xpos[k / 3][k % 3];
  out += MAXBODY * 3;
  for (int k = sl; k < nb * 9; k += HL) out[k] = s.u.k.xmat[k / 9][k % 9];
  out += MAXBODY * 9;
  for (int k = sl; k < ng * 3; k += HL) out[k] = s.u.k.gpos[k / 3][k % 3];
  out += MAXGEOM * 3;
  for (int k = sl; k < ng * 3; k += HL) out[k] = s.u.k.gax[k / 3][k % 3];
  out += MAXGEOM * 3;
  if (sl < 3) out[sl] = s.com[sl];
}

// hs_reward_eval: the step kernel's reward code (np_sum_half + reward_formula) on caller-supplied
// fields, one env per 32-lane half as in the step kernel.  Not on the step path: it exists so the
// device formulas can be checked against the reference's own outputs on arbitrary states.
template <typename T>
__global__ __launch_bounds__(256) void reward_eval_kernel(RewardEvalArgs<T> a) {
  const int lane = threadIdx.x & (WAVE - 1);
  const int sl = lane & (HL - 1);
  const long long env = ((long long)blockIdx.x * blockDim.x + threadIdx.x) / HL;
  const bool ok = env < a.n;
  const int nv = a.nv, nu = a.nu;
  const long long ldc = a.ld_com ? a.ld_com : 3, ldl = a.ld_linv ? a.ld_linv : 3, ldq = a.ld_qfrc ? a.ld_qfrc : nv;
  T e = T(0), cu = T(0);
  if (ok && sl < nv) e = a.qfrc_actuator[env * ldq + sl] * a.qvel[env * nv + sl];
  if (ok && sl < nu) cu = a.ctrl[env * nu + sl];
  const T esum = np_sum_half(e * e, 6, nv - 6, lane);   // every lane of the wave takes part
  const T csum = np_sum_half(cu * cu, 0, nu, lane);
  if (!ok || sl != 0) return;
  const T* q = a.qpos + env * a.nq;
  RewardIn<T> in;
  in.h = q[2];
  in.qw = q[3];
  in.qx = q[4];
  in.qy = q[5];
  in.qz = q[6];
  in.vx = a.qvel[env * nv];
  in.time = a.time[env];
  in.com0 = a.subtree_com0[env * ldc];
  in.com1 = a.subtree_com0[env * ldc + 1];
  {
#pragma clang fp contract(off)
    in.comv = T(0);
    for (int d = 0; d < 3; d++) in.comv += a.subtree_linvel0[env * ldl + d] * a.subtree_linvel0[env * ldl + d];
  }
  const T* cf = a.cfrc_ext + (env * a.nbody + a.nbody - 2) * 6;
  in.lf = T(0);
  in.rf = T(0);
  for (int d = 0; d < 6; d++) { in.lf += fabs(cf[d]); in.rf += fabs(cf[6 + d]); }
  in.energy = esum;
  in.ctrl_sq = csum;
  a.out[env] = reward_formula(a.reward_id, a.kneel, in);
}

// hs_pack_outputs: one step's host-bound outputs as ONE float64 buffer in one launch (the drop-in's
// single device-to-host copy): obs rows, then ncols columns of N values, then the warning rows
// (column-major: kind k of env i at k * N + i).  Grid-stride over the whole buffer: coalesced writes.
template <typename T>
__global__ __launch_bounds__(256) void pack_kernel(PackArgs<T> a) {
  const size_t nobs = (size_t)a.n * a.obs_dim, ncol = (size_t)a.ncols * a.n, nw = (size_t)a.nwarn * a.n;
  const size_t total = nobs + ncol + nw;
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += (size_t)gridDim.x * blockDim.x) {
    double v;
    if (i < nobs) {
      v = (double)a.obs[i];
    } else if (i < nobs + ncol) {
      const size_t j = i - nobs;
      const int c = (int)(j / a.n);
      const size_t e = j - (size_t)c * a.n;
      switch (c) {
        case 0: v = (double)a.reward[e]; break;
        case 1: v = (double)a.terminated[e]; break;
        case 2: v = (double)a.truncated[e]; break;
        case 3: v = (double)a.total_reward[e]; break;
        case 4: v = (double)a.step_count[e]; break;
        case 5: v = a.term_step_count ? (double)a.term_step_count[e] : 0.0; break;
        default: v = a.term_total_reward ? (double)a.term_total_reward[e] : 0.0; break;
      }
    } else {
      const size_t j = i - nobs - ncol;
      const int kind = (int)(j / a.n);
      const size_t e = j - (size_t)kind * a.n;
      v = (double)a.warning[e * a.nwarn_stride + kind];
    }
    a.out[i] = v;
  }
}

}  // namespace

template <typename T>
hipError_t launch_pack(const PackArgs<T>& a, hipStream_t stream) {
  const size_t total = (size_t)a.n * (a.obs_dim + a.ncols + a.nwarn);
  if (total == 0) return hipSuccess;
  const unsigned blocks = (unsigned)std::min<size_t>((total + 255) / 256, 2048);
  hipLaunchKernelGGL((pack_kernel<T>), dim3(blocks), dim3(256), 0, stream, a);
  return hipGetLastError();
}

template <typename T>
hipError_t launch_reward_eval(const RewardEvalArgs<T>& a, hipStream_t stream) {
  if (a.n <= 0) return hipSuccess;
  if (a.nv < 6 || a.nv > HL || a.nu < 0 || a.nu > HL || a.nbody < 2 || a.nq < 7) return hipErrorInvalidValue;
  const long long threads = (long long)a.n * HL;
  const unsigned blocks = (unsigned)((threads + 255) / 256);
  hipLaunchKernelGGL((reward_eval_kernel<T>), dim3(blocks), dim3(256), 0, stream, a);
  return hipGetLastError();
}

// waves of the resident step-kernel instance the current device holds at once (occupancy x CUs),
// cached per device (a racing first call computes the same value twice: benign)
template <typename T>
int resident_waves(bool pgs) {
  constexpr int MAXDEV = 64;
  static int cache[2][MAXDEV] = {};   // 0: not yet computed
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0) return 0;
  int* c = dev < MAXDEV ? &cache[pgs ? 1 : 0][dev] : nullptr;
  if (c && *c != 0) return *c > 0 ? *c : 0;
  int per_cu = 0, v = -1;
  hipDeviceProp_t prop;
  hipError_t e = hipGetDeviceProperties(&prop, dev);
  if (e == hipSuccess)
    e = pgs ? hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, step_kernel<T, 27, true>, WAVE, 0)
            : hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, step_kernel<T, 27, false>, WAVE, 0);
  if (e == hipSuccess && per_cu > 0) v = per_cu * prop.multiProcessorCount;
  if (c) *c = v;
  return v > 0 ? v : 0;
}

template <typename T>
hipError_t launch_step(const DevModel<T>* dmodel, int nv, const EnvBuffers<T>& b, const float* actions,
                       const uint8_t* reset_mask, const T* noise_qpos, const T* noise_qvel,
                       const StepParams& p, int nenv, hipStream_t stream, const TapeOut<T>* tape,
                       const RolloutArgs* ro) {
  if (nenv <= 0) return hipSuccess;
  if (nv != 27) return hipErrorInvalidValue;
  KArgs<T> args{(MPtr<T>)dmodel, b, actions, reset_mask, noise_qpos, noise_qvel, p, nenv,
                tape ? *tape : TapeOut<T>{nullptr, nullptr, nullptr, nullptr}, ro ? *ro : RolloutArgs{}};
  // fused rollouts: the fp64 Newton engine
  if (ro && (sizeof(T) != 8 || !ro->obs || p.solver == SOLVER_PGS)) return hipErrorInvalidValue;
  if (args.p.nsteps < 1) args.p.nsteps = 1;
  // chunk-queue schedule when the env pairs outnumber the waves the GPU holds at once (the fp64
  // engine: 1 wave per SIMD), for multi-substep calls (HS_SCHED_DIRECT: never)
  const int npairs = (nenv + 1) / 2;
  const int resident = resident_waves<T>(p.solver == SOLVER_PGS);
  const bool may_queue = p.schedule == SCHED_AUTO || p.schedule == SCHED_FIXED_ORDER;
  args.p.queue = (may_queue && b.mid && b.qsync && p.mode != MODE_RESET && p.nsub >= 2 && resident > 0 &&
                  npairs > resident) ? 1 : 0;
  // tape launch (several env steps of an action tape): always the chunk queue, with whole env steps
  // as items, whatever the batch size -- a pair's next env step starts as soon as its own previous
  // one is committed, so the steps of different pairs overlap instead of each step ending on its
  // slowest pair
  const bool tape_launch = args.p.nsteps > 1 || ro != nullptr;
  if (tape_launch) {
    if (p.mode != MODE_ENV_STEP || !b.mid || !b.qsync || resident <= 0 || args.p.nsteps > QTAG_STEPS)
      return hipErrorInvalidValue;
    args.p.queue = 1;
  }
  // a tape launch of a small batch (every env fits a resident wave of its own) queues single envs,
  // not pairs: twice the waves, each env's steps back to back (configs[4]'s 1024 envs would otherwise
  // leave half of the resident wave slots idle)
  const bool qsingle = tape_launch && may_queue && nenv <= resident;
  const int nunits = qsingle ? nenv : npairs;
  args.p.qorder = p.schedule == SCHED_AUTO ? 1 : 0;
  // fallback claim order (first queued launch, SCHED_FIXED_ORDER): a fixed multiplicative
  // permutation of the pairs (the same for both chunk kinds, so a pair's last substep is still
  // claimed npairs items after its first chunk).  Items whose cost is correlated with the env index
  // -- e.g. env clocks staggered by index, bench.py's window -- are spread over the launch instead
  // of arriving together at its end.
  args.p.qmul = 1;
  if (args.p.queue) {
    auto gcd = [](uint32_t a, uint32_t b) { while (b) { uint32_t t = a % b; a = b; b = t; } return a; };
    uint32_t q = (uint32_t)(0.6180339887 * nunits) | 1u;
    while (gcd(q, (uint32_t)nunits) != 1u) q += 2;
    args.p.qmul = (int)(q % (uint32_t)nunits == 0 ? 1 : q);
  }
  // single-env schedule: one wave per env (the upper half-wave a ghost of the lower) when every
  // env gets a resident wave of its own -- small batches (configs[4]'s 1024 envs per GPU) would
  // otherwise leave SIMDs idle with one wave per env pair
  args.p.single = qsingle || (!args.p.queue && (p.schedule == SCHED_SINGLE ||
                                                (p.schedule == 0 && resident > 0 && nenv <= resident))) ? 1 : 0;
  // the lost-hand-off test hook names an env (+ 1); the kernel compares it with its queue unit
  if (args.p.dbg_lose_pair1 > 0 && !qsingle) args.p.dbg_lose_pair1 = (args.p.dbg_lose_pair1 - 1) / 2 + 1;
  const dim3 grid(args.p.queue ? (tape_launch ? std::min(resident, nunits) : resident) : (args.p.single ? nenv : npairs)),
      block(WAVE);
  // the wide tier's grid: enough waves for a few deferred envs at once, few enough that the
  // common no-overflow launch (every wave reads the count and exits) costs a few microseconds
  const dim3 wgrid(std::min((nenv + 1) / 2, 32));
#ifndef HS_DEV_NEWTON_ONLY   // development builds: resource-usage checks of the Newton instances only
  if (p.solver == SOLVER_PGS) {
    if (args.p.queue) hipLaunchKernelGGL((step_kernel_queue<T, 27, true>), grid, block, 0, stream, args);
    else hipLaunchKernelGGL((step_kernel<T, 27, true>), grid, block, 0, stream, args);
    if (b.redo && !tape_launch) hipLaunchKernelGGL((step_kernel_wide<T, 27, true>), wgrid, block, 0, stream, args);
    return hipGetLastError();
  }
#endif
  if (ro) {
    if constexpr (sizeof(T) == 8) hipLaunchKernelGGL((step_kernel_queue<T, 27, false, true>), grid, block, 0, stream, args);
    return hipGetLastError();
  }
  if (args.p.queue) hipLaunchKernelGGL((step_kernel_queue<T, 27, false>), grid, block, 0, stream, args);
  else hipLaunchKernelGGL((step_kernel<T, 27, false>), grid, block, 0, stream, args);
  if (b.redo && !tape_launch) hipLaunchKernelGGL((step_kernel_wide<T, 27, false>), wgrid, block, 0, stream, args);
  return hipGetLastError();
}

template <typename T>
hipError_t launch_kinematics(const DevModel<T>* dmodel, int nv, const T* qpos, T* out, hipStream_t stream) {
  if (nv != 27) return hipErrorInvalidValue;
  hipLaunchKernelGGL((kin_kernel<T, 27>), dim3(1), dim3(WAVE), 0, stream, (MPtr<T>)dmodel, qpos, out);
  return hipGetLastError();
}
// The Makefile compiles this file once per precision (HS_ONLY_F32 / HS_ONLY_F64), so each engine
// gets its own code-generation flags (the fp64 one without MachineLICM).
#ifndef HS_ONLY_F64
template hipError_t launch_step<float>(const DevModel<float>*, int, const EnvBuffers<float>&, const float*,
                                       const uint8_t*, const float*, const float*, const StepParams&, int,
                                       hipStream_t, const TapeOut<float>*, const RolloutArgs*);
template int resident_waves<float>(bool);
template hipError_t launch_kinematics<float>(const DevModel<float>*, int, const float*, float*, hipStream_t);
template hipError_t launch_reward_eval<float>(const RewardEvalArgs<float>&, hipStream_t);
template hipError_t launch_pack<float>(const PackArgs<float>&, hipStream_t);
#endif
#if !defined(HS_DEV_F32_ONLY) && !defined(HS_ONLY_F32)
template hipError_t launch_step<double>(const DevModel<double>*, int, const EnvBuffers<double>&, const float*,
                                        const uint8_t*, const double*, const double*, const StepParams&, int,
                                        hipStream_t, const TapeOut<double>*, const RolloutArgs*);
#endif

#if !defined(HS_DEV_F32_ONLY) && !defined(HS_ONLY_F32)
template int resident_waves<double>(bool);
template hipError_t launch_kinematics<double>(const DevModel<double>*, int, const double*, double*, hipStream_t);
template hipError_t launch_reward_eval<double>(const RewardEvalArgs<double>&, hipStream_t);
template hipError_t launch_pack<double>(const PackArgs<double>&, hipStream_t);
#endif

}  // namespace hs

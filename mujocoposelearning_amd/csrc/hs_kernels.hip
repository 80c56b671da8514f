// hsim step kernel for gfx950 (MI355X).  PRODUCT CODE.
//
// Replaces, for a whole batch of envs at once:
//   custom_env.py:152-230  HumanoidEnv.step   (frame_skip x {ctrl = a; mj_step}, obs, reward, done)
//   custom_env.py:97-150   HumanoidEnv.reset  (mj_resetData, noise, one ctrl=0 mj_step, obs)
//   custom_env.py:232-261  _get_state         (352-dim obs, stale derived fields)
//   reward_functions.py:66-261 stand / kneeling / walk rewards (device plug-ins)
//   SB3 SubprocVecEnv auto-reset semantics (train_sb3.py:203)
// and MuJoCo 3.2.5's mj_step pipeline (custom_env.py:121,160): kinematics, com, CRB, collision,
// constraint assembly, RNE, actuation, primal Newton solver (pyramidal cones), Euler with
// implicit joint damping.
//
// Execution model: ONE WAVEFRONT (64 lanes) PER ENV.  All per-env state lives in LDS; lanes map
// to bodies / dofs / geom pairs / contacts / constraint rows stage by stage; dense nv x nv
// matrices (M, Newton Hessian, M + h*B) live row-per-lane in VGPRs and are factored with
// v_readlane broadcasts (no LDS traffic, no barriers).  The contact part of the Newton
// Hessian is assembled with the tree-structured "composite" form  H_ij += jp_j' U jp_i, which
// costs O(nv * ncon) instead of O(nv^2 * nefc).  HBM traffic is only the per-env state in/out.
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdint>

#include "hs_kernels.h"
#include "hs_model.h"

namespace hs {
namespace {

constexpr int WAVE = 64;

// ------------------------------------------------------------------ cross-lane helpers
__device__ __forceinline__ float rl(float v, int l) {
  return __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), l));
}
__device__ __forceinline__ double rl(double v, int l) {
  long long x = __double_as_longlong(v);
  int lo = __builtin_amdgcn_readlane((int)(x & 0xffffffffll), l);
  int hi = __builtin_amdgcn_readlane((int)(x >> 32), l);
  return __longlong_as_double(((long long)hi << 32) | (unsigned)lo);
}
template <int CTRL>
__device__ __forceinline__ float dpp(float v) {
  return __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), CTRL, 0xF, 0xF, false));
}
template <int CTRL>
__device__ __forceinline__ double dpp(double v) {
  long long x = __double_as_longlong(v);
  int lo = __builtin_amdgcn_mov_dpp((int)(x & 0xffffffffll), CTRL, 0xF, 0xF, false);
  int hi = __builtin_amdgcn_mov_dpp((int)(x >> 32), CTRL, 0xF, 0xF, false);
  return __longlong_as_double(((long long)hi << 32) | (unsigned)lo);
}
// sum over each 32-lane half (result in every lane of the half)
template <typename T>
__device__ __forceinline__ T hsum32(T v) {
  v += dpp<0xB1>(v);    // quad_perm [1,0,3,2]
  v += dpp<0x4E>(v);    // quad_perm [2,3,0,1]
  v += dpp<0x141>(v);   // row_half_mirror
  v += dpp<0x140>(v);   // row_mirror
  v += __shfl_xor(v, 16);
  return v;
}
template <typename T>
__device__ __forceinline__ T wsum(T v) {
  v = hsum32(v);
  return rl(v, 0) + rl(v, 32);
}
__device__ __forceinline__ bool bit(uint32_t mask, int i) { return i < 32 && ((mask >> i) & 1u); }
__device__ __forceinline__ int lanes_below(uint64_t mask, int lane) {
  return __popcll(mask & ((1ull << lane) - 1ull));
}
template <typename T>
__device__ __forceinline__ bool isbad(T x) {
  return !(x <= T(1e10) && x >= T(-1e10));   // NaN or |x| > mjMAXVAL
}

// ------------------------------------------------------------------ small algebra
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
__device__ __forceinline__ T normalize3(T* v) {
  T n = sqrt(dot3(v, v));
  if (n < T(1e-15)) { v[0] = 1; v[1] = 0; v[2] = 0; }
  else { T i = T(1) / n; v[0] *= i; v[1] *= i; v[2] *= i; }
  return n;
}
template <typename T>
__device__ __forceinline__ void normalize4(T* q) {
  T n = sqrt(q[0] * q[0] + q[1] * q[1] + q[2] * q[2] + q[3] * q[3]);
  if (n < T(1e-15)) { q[0] = 1; q[1] = q[2] = q[3] = 0; }
  else { T i = T(1) / n; q[0] *= i; q[1] *= i; q[2] *= i; q[3] *= i; }
}
// spatial inertia (10-param cinert layout) times motion vector
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
// Cholesky A = L L' of an NV x NV SPD matrix held row-per-lane (lane i: A[i][0..NV)); lower part
// is replaced by L.  Upper part of each row becomes scratch.
template <int NV, typename T>
__device__ __forceinline__ void chol_rows(T (&A)[NV], int lane) {
#pragma unroll
  for (int k = 0; k < NV; k++) {
    T akk = rl(A[k], k);
    T lkk = sqrt(akk > T(1e-30) ? akk : T(1e-30));
    T inv = T(1) / lkk;
    T lik = (lane == k) ? lkk : A[k] * inv;
    A[k] = lik;
#pragma unroll
    for (int j = k + 1; j < NV; j++) A[j] -= lik * rl(lik, j);
  }
}
// solve (L L') x = b; lane i holds b_i; returns x_i
template <int NV, typename T>
__device__ __forceinline__ T chol_solve(const T (&L)[NV], T b, int lane) {
#pragma unroll
  for (int k = 0; k < NV; k++) {
    T yk = rl(b, k) / rl(L[k], k);
    b = (lane == k) ? yk : ((lane > k) ? b - L[k] * yk : b);
  }
  T x = 0;
#pragma unroll
  for (int k = NV - 1; k >= 0; k--) {
    T part = (lane > k && lane < NV) ? L[k] * x : T(0);
    T ssum = rl(hsum32(part), 0);
    T xk = (rl(b, k) - ssum) / rl(L[k], k);
    x = (lane == k) ? xk : x;
  }
  return x;
}
// y = A x for A row-per-lane (full rows)
template <int NV, typename T>
__device__ __forceinline__ T matvec_rows(const T (&A)[NV], T x) {
  T acc = 0;
#pragma unroll
  for (int j = 0; j < NV; j++) acc += A[j] * rl(x, j);
  return acc;
}

// ------------------------------------------------------------------ per-env LDS scratch
enum RowKind { RK_JLO = 0, RK_JHI = 1, RK_TLO = 2, RK_THI = 3, RK_CN = 4, RK_P0 = 5 };   // P0..P0+3: pyramid

template <typename T>
struct Scratch {
  T qpos[MAXQ];
  T qvel[MAXDOF];
  T ctrl[MAXU];
  T vx[MAXDOF];
  T qfrc_act[MAXDOF];
  T xpos[MAXBODY][3];
  T xquat[MAXBODY][4];
  T xmat[MAXBODY][9];
  T xipos[MAXBODY][3];
  T xanchor[MAXJNT][3];
  T xaxis[MAXJNT][3];
  T gpos[MAXGEOM][3];
  T gax[MAXGEOM][3];
  T cinert[MAXBODY][10];
  T crb[MAXBODY][10];
  T cdof[MAXDOF][6];
  T cdofdot[MAXDOF][6];
  T buf[MAXDOF][6];
  T cvel[MAXBODY][6];
  T bvel[MAXBODY][6];
  T cfrc[MAXBODY][6];
  T con_pos[MAXCON][3];
  T con_n[MAXCON][3];
  T con_t1[MAXCON][3];
  T con_t2[MAXCON][3];
  T con_dist[MAXCON];
  T con_v[MAXCON][3];
  T con_U[MAXCON][6];
  T con_F[MAXCON][3];
  int con_pair[MAXCON];
  int con_adr[MAXCON];
  int row_kind[MAXEFC];
  int row_id[MAXEFC];
  T row_D[MAXEFC];
  T row_aref[MAXEFC];
  T row_f[MAXEFC];
  T com[4];
  int ncon, nefc, nlim, niter;
};

template <typename T>
struct Env {
  const DevModel<T>* __restrict__ m;
  Scratch<T>& s;
  int lane;
  int nv, nb;
};

// ------------------------------------------------------------------ kinematics (mj_kinematics)
template <typename T>
__device__ void body_pose(const DevModel<T>* __restrict__ m, Scratch<T>& s, int b) {
  T pos[3], q[4];
  int ja = m->body_jntadr[b], jn = m->body_jntnum[b];
  if (jn == 1 && m->jnt_type[ja] == JNT_FREE) {
    int qa = m->jnt_qposadr[ja];
    for (int k = 0; k < 3; k++) pos[k] = s.qpos[qa + k];
    for (int k = 0; k < 4; k++) q[k] = s.qpos[qa + 3 + k];
    normalize4(q);
    for (int k = 0; k < 3; k++) { s.xanchor[ja][k] = pos[k]; s.xaxis[ja][k] = m->jnt_axis[ja][k]; }
  } else {
    int p = m->body_parentid[b];
    T bp[3] = {m->body_pos[b][0], m->body_pos[b][1], m->body_pos[b][2]};
    T bq[4] = {m->body_quat[b][0], m->body_quat[b][1], m->body_quat[b][2], m->body_quat[b][3]};
    mv3(s.xmat[p], bp, pos);
    for (int k = 0; k < 3; k++) pos[k] += s.xpos[p][k];
    T pq[4] = {s.xquat[p][0], s.xquat[p][1], s.xquat[p][2], s.xquat[p][3]};
    mulq(pq, bq, q);
    for (int j = ja; j < ja + jn; j++) {
      T R[9], ax[3], an[3], jp[3] = {m->jnt_pos[j][0], m->jnt_pos[j][1], m->jnt_pos[j][2]};
      T la[3] = {m->jnt_axis[j][0], m->jnt_axis[j][1], m->jnt_axis[j][2]};
      quat2mat(q, R);
      mv3(R, la, ax);
      mv3(R, jp, an);
      for (int k = 0; k < 3; k++) an[k] += pos[k];
      int qa = m->jnt_qposadr[j];
      T ang = s.qpos[qa] - m->qpos0[qa];
      T sn = sin(T(0.5) * ang), cs = cos(T(0.5) * ang);
      T ql[4] = {cs, la[0] * sn, la[1] * sn, la[2] * sn};
      mulq(q, ql, q);
      quat2mat(q, R);
      T v[3];
      mv3(R, jp, v);
      for (int k = 0; k < 3; k++) pos[k] = an[k] - v[k];
      for (int k = 0; k < 3; k++) { s.xanchor[j][k] = an[k]; s.xaxis[j][k] = ax[k]; }
    }
  }
  normalize4(q);
  for (int k = 0; k < 4; k++) s.xquat[b][k] = q[k];
  for (int k = 0; k < 3; k++) s.xpos[b][k] = pos[k];
  quat2mat(q, s.xmat[b]);
}

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
  else { T i = T(1) / len; for (int k = 0; k < 3; k++) o.n[k] = d[k] * i; }
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

// returns number of contacts (0..2) for static pair p
template <typename T>
__device__ int collide_pair(const DevModel<T>* __restrict__ m, const Scratch<T>& s, int p, Con<T>& c0, Con<T>& c1) {
  int g1 = m->pair_g1[p], g2 = m->pair_g2[p], fn = m->pair_fn[p];
  const T* p1 = s.gpos[g1];
  const T* p2 = s.gpos[g2];
  const T* a1 = s.gax[g1];
  const T* a2 = s.gax[g2];
  T r1 = m->geom_size[g1][0], r2 = m->geom_size[g2][0], h1 = m->geom_size[g1][1], h2 = m->geom_size[g2][1];
  int n = 0;
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

template <typename T>
__device__ __forceinline__ void store_contact(Scratch<T>& s, int slot, const Con<T>& c, int p) {
  if (slot >= MAXCON) return;
  for (int k = 0; k < 3; k++) { s.con_pos[slot][k] = c.pos[k]; s.con_n[slot][k] = c.n[k]; s.con_t1[slot][k] = c.t1[k]; }
  T t2[3];
  cross3(c.n, c.t1, t2);
  for (int k = 0; k < 3; k++) s.con_t2[slot][k] = t2[k];
  s.con_dist[slot] = c.dist;
  s.con_pair[slot] = p;
}

// impedance (mj_makeImpedance getimpedance), MuJoCo clamps d0/dmax to [1e-4, 0.9999]
template <typename T>
__device__ __forceinline__ T impedance(const T* si, T pos, T margin) {
  T s0 = fmin(T(0.9999), fmax(T(0.0001), si[0])), s1 = fmin(T(0.9999), fmax(T(0.0001), si[1]));
  if (s0 == s1 || si[2] <= T(1e-15)) return T(0.5) * (s0 + s1);
  T x = (pos - margin) / si[2];
  if (x < 0) x = -x;
  if (x >= 1 || x <= 0) return x >= 1 ? s1 : s0;
  T y;
  if (si[4] == 1) y = x;
  else if (x <= si[3]) y = pow(x, si[4]) / pow(si[3], si[4] - 1);
  else y = 1 - pow(1 - x, si[4]) / pow(1 - si[3], si[4] - 1);
  return s0 + y * (s1 - s0);
}

// ------------------------------------------------------------------ J x for all rows
// maps s.vx (generalized vector) -> body spatial velocities -> contact frame velocities
template <typename T>
__device__ void map_vx(const DevModel<T>* __restrict__ m, Scratch<T>& s, int lane, int nv, int nb) {
  if (lane > 0 && lane < nb) {
    uint32_t ch = m->body_chainmask[lane];
    T v[6] = {0, 0, 0, 0, 0, 0};
    for (int j = 0; j < nv; j++) {
      if ((ch >> j) & 1u) {
        T xj = s.vx[j];
        for (int k = 0; k < 6; k++) v[k] += s.cdof[j][k] * xj;
      }
    }
    for (int k = 0; k < 6; k++) s.bvel[lane][k] = v[k];
  }
  if (lane == 0)
    for (int k = 0; k < 6; k++) s.bvel[0][k] = 0;
  __syncthreads();
  if (lane < s.ncon) {
    int p = s.con_pair[lane];
    int b1 = m->pair_b1[p], b2 = m->pair_b2[p];
    T r[3] = {s.con_pos[lane][0] - s.com[0], s.con_pos[lane][1] - s.com[1], s.con_pos[lane][2] - s.com[2]};
    T w[3], v1[3], v2[3];
    cross3(s.bvel[b2], r, w);
    for (int k = 0; k < 3; k++) v2[k] = s.bvel[b2][3 + k] + w[k];
    cross3(s.bvel[b1], r, w);
    for (int k = 0; k < 3; k++) v1[k] = s.bvel[b1][3 + k] + w[k];
    T dv[3] = {v2[0] - v1[0], v2[1] - v1[1], v2[2] - v1[2]};
    s.con_v[lane][0] = dot3(s.con_n[lane], dv);
    s.con_v[lane][1] = dot3(s.con_t1[lane], dv);
    s.con_v[lane][2] = dot3(s.con_t2[lane], dv);
  }
  __syncthreads();
}

template <typename T>
__device__ __forceinline__ T row_Jx(const DevModel<T>* __restrict__ m, const Scratch<T>& s, int r) {
  int kind = s.row_kind[r], id = s.row_id[r];
  if (kind <= RK_JHI) {
    T v = s.vx[m->jnt_dofadr[id]];
    return kind == RK_JLO ? v : -v;
  }
  if (kind <= RK_THI) {
    T v = 0;
    for (int w = 0; w < m->ten_nwrap[id]; w++) v += m->ten_wrapcoef[id][w] * s.vx[m->ten_wrapdof[id][w]];
    return kind == RK_TLO ? v : -v;
  }
  if (kind == RK_CN) return s.con_v[id][0];
  int sub = kind - RK_P0;
  T mu = m->pair_mu[s.con_pair[id]];
  T sg = (sub & 1) ? -mu : mu;
  return s.con_v[id][0] + sg * s.con_v[id][1 + (sub >> 1)];
}

// world-frame force direction u of a contact row
template <typename T>
__device__ __forceinline__ void row_u(const DevModel<T>* __restrict__ m, const Scratch<T>& s, int kind, int c, T* u) {
  if (kind == RK_CN) { for (int k = 0; k < 3; k++) u[k] = s.con_n[c][k]; return; }
  int sub = kind - RK_P0;
  T mu = m->pair_mu[s.con_pair[c]];
  T sg = (sub & 1) ? -mu : mu;
  const T* t = (sub >> 1) ? s.con_t2[c] : s.con_t1[c];
  for (int k = 0; k < 3; k++) u[k] = s.con_n[c][k] + sg * t[k];
}

// per-contact aggregates from current row forces / activity: U = sum D u u' (active), F = sum f u
template <typename T>
__device__ void contact_aggregates(const DevModel<T>* __restrict__ m, Scratch<T>& s, int lane) {
  if (lane < s.ncon) {
    int adr = s.con_adr[lane];
    int nr = m->pair_dim[s.con_pair[lane]] == 1 ? 1 : 4;
    T U[6] = {0, 0, 0, 0, 0, 0}, F[3] = {0, 0, 0};
    for (int q = 0; q < nr; q++) {
      int r = adr + q;
      T f = s.row_f[r];
      if (f != T(0)) {
        T u[3];
        row_u(m, s, s.row_kind[r], lane, u);
        T D = s.row_D[r];
        U[0] += D * u[0] * u[0]; U[1] += D * u[1] * u[1]; U[2] += D * u[2] * u[2];
        U[3] += D * u[0] * u[1]; U[4] += D * u[0] * u[2]; U[5] += D * u[1] * u[2];
        for (int k = 0; k < 3; k++) F[k] += f * u[k];
      }
    }
    for (int k = 0; k < 6; k++) s.con_U[lane][k] = U[k];
    for (int k = 0; k < 3; k++) s.con_F[lane][k] = F[k];
  }
  __syncthreads();
}

// (J' f)_i for dof lane i (contacts via point Jacobians, limits via sparse rows)
template <typename T>
__device__ T jtf_lane(const DevModel<T>* __restrict__ m, const Scratch<T>& s, int lane, const T* cd) {
  T acc = 0;
  for (int c = 0; c < s.ncon; c++) {
    int p = s.con_pair[c];
    int b1 = m->pair_b1[p], b2 = m->pair_b2[p];
    int in2 = bit(m->body_chainmask[b2], lane), in1 = b1 ? bit(m->body_chainmask[b1], lane) : 0;
    if (in1 != in2) {
      T r[3] = {s.con_pos[c][0] - s.com[0], s.con_pos[c][1] - s.com[1], s.con_pos[c][2] - s.com[2]};
      T w[3];
      cross3(cd, r, w);
      T jp[3] = {cd[3] + w[0], cd[4] + w[1], cd[5] + w[2]};
      T v = dot3(jp, s.con_F[c]);
      acc += in2 ? v : -v;
    }
  }
  for (int r = 0; r < s.nlim; r++) {
    int kind = s.row_kind[r], id = s.row_id[r];
    T f = s.row_f[r];
    if (kind <= RK_JHI) {
      if (m->jnt_dofadr[id] == lane) acc += kind == RK_JLO ? f : -f;
    } else {
      for (int w = 0; w < m->ten_nwrap[id]; w++)
        if (m->ten_wrapdof[id][w] == lane) acc += (kind == RK_TLO ? f : -f) * m->ten_wrapcoef[id][w];
    }
  }
  return acc;
}

// ------------------------------------------------------------------ one mj_step
template <typename T, int NV>
struct Stepper {
  const DevModel<T>* __restrict__ m;
  Scratch<T>& s;
  int lane, nb;
  T cd[6];        // cdof of this lane's dof (registers)
  T Mr[NV];       // mass-matrix row of this lane's dof
  T fsmooth;      // qfrc_smooth_i
  T fcon;         // qfrc_constraint_i
  T qacc;         // solver output qacc_i
  int niter;

  __device__ Stepper(const DevModel<T>* mm, Scratch<T>& ss, int l) : m(mm), s(ss), lane(l), nb(mm->nbody) {}

  __device__ void kinematics() {
    if (lane == 0) {
      for (int k = 0; k < 3; k++) s.xpos[0][k] = 0;
      s.xquat[0][0] = 1; s.xquat[0][1] = s.xquat[0][2] = s.xquat[0][3] = 0;
      for (int k = 0; k < 9; k++) s.xmat[0][k] = (k % 4 == 0) ? T(1) : T(0);
    }
    __syncthreads();
    for (int L = 0; L < m->nlevel; L++) {
      int a0 = m->level_adr[L], n = m->level_adr[L + 1] - a0;
      if (lane < n) body_pose(m, s, m->level_body[a0 + lane]);
      __syncthreads();
    }
    if (lane < m->ngeom) {
      int b = m->geom_bodyid[lane];
      T gp[3] = {m->geom_pos[lane][0], m->geom_pos[lane][1], m->geom_pos[lane][2]};
      T gz[3] = {m->geom_zaxis[lane][0], m->geom_zaxis[lane][1], m->geom_zaxis[lane][2]};
      T w[3];
      mv3(s.xmat[b], gp, w);
      for (int k = 0; k < 3; k++) s.gpos[lane][k] = s.xpos[b][k] + w[k];
      mv3(s.xmat[b], gz, s.gax[lane]);
    }
    T mx = 0, my = 0, mz = 0;
    if (lane > 0 && lane < nb) {
      T ip[3] = {m->body_ipos[lane][0], m->body_ipos[lane][1], m->body_ipos[lane][2]}, w[3];
      mv3(s.xmat[lane], ip, w);
      for (int k = 0; k < 3; k++) s.xipos[lane][k] = s.xpos[lane][k] + w[k];
      T mb = m->body_mass[lane];
      mx = mb * s.xipos[lane][0]; my = mb * s.xipos[lane][1]; mz = mb * s.xipos[lane][2];
    }
    // mj_comPos: single kinematic tree -> subtree_com[root] == subtree_com[0] == whole-model COM
    T inv = T(1) / m->total_mass;
    T c0 = wsum(mx) * inv, c1 = wsum(my) * inv, c2 = wsum(mz) * inv;
    if (lane == 0) { s.com[0] = c0; s.com[1] = c1; s.com[2] = c2; }
    __syncthreads();
    if (lane > 0 && lane < nb) {   // cinert (mju_inertCom)
      const T* R = s.xmat[lane];
      const T* I6 = m->body_inert[lane];
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
      T d[3] = {s.xipos[lane][0] - c0, s.xipos[lane][1] - c1, s.xipos[lane][2] - c2};
      T mass = m->body_mass[lane];
      T* ci = s.cinert[lane];
      ci[0] = Ic[0] + mass * (d[1] * d[1] + d[2] * d[2]);
      ci[1] = Ic[1] + mass * (d[0] * d[0] + d[2] * d[2]);
      ci[2] = Ic[2] + mass * (d[0] * d[0] + d[1] * d[1]);
      ci[3] = Ic[3] - mass * d[0] * d[1];
      ci[4] = Ic[4] - mass * d[0] * d[2];
      ci[5] = Ic[5] - mass * d[1] * d[2];
      ci[6] = mass * d[0]; ci[7] = mass * d[1]; ci[8] = mass * d[2]; ci[9] = mass;
    }
    if (lane == 0)
      for (int k = 0; k < 10; k++) s.cinert[0][k] = 0;
    for (int k = 0; k < 6; k++) cd[k] = 0;
    if (lane < NV) {   // cdof (mju_dofCom)
      int j = m->dof_jntid[lane], b = m->dof_bodyid[lane];
      T off[3] = {c0 - s.xanchor[j][0], c1 - s.xanchor[j][1], c2 - s.xanchor[j][2]};
      T ax[3];
      bool lin = false;
      if (m->jnt_type[j] == JNT_FREE) {
        int k = lane - m->jnt_dofadr[j];
        if (k < 3) { lin = true; cd[3 + k] = 1; }
        else { int c = k - 3; ax[0] = s.xmat[b][c]; ax[1] = s.xmat[b][3 + c]; ax[2] = s.xmat[b][6 + c]; }
      } else {
        ax[0] = s.xaxis[j][0]; ax[1] = s.xaxis[j][1]; ax[2] = s.xaxis[j][2];
      }
      if (!lin) {
        cd[0] = ax[0]; cd[1] = ax[1]; cd[2] = ax[2];
        cross3(ax, off, cd + 3);
      }
      for (int k = 0; k < 6; k++) s.cdof[lane][k] = cd[k];
    }
    __syncthreads();
  }

  // mj_crb -> Mr rows (registers), buf = crb * cdof
  __device__ void mass_matrix() {
    if (lane > 0 && lane < nb) {
      uint32_t dm = m->body_descmask[lane];
      T a[10] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0};
      for (int c = 1; c < nb; c++)
        if ((dm >> c) & 1u)
          for (int k = 0; k < 10; k++) a[k] += s.cinert[c][k];
      for (int k = 0; k < 10; k++) s.crb[lane][k] = a[k];
    }
    __syncthreads();
    T bf[6] = {0, 0, 0, 0, 0, 0};
    uint32_t anci = 0;
    T arm = 0;
    if (lane < NV) {
      mul_inert(s.crb[m->dof_bodyid[lane]], cd, bf);
      for (int k = 0; k < 6; k++) s.buf[lane][k] = bf[k];
      anci = m->dof_ancmask[lane];
      arm = m->dof_armature[lane];
    }
    __syncthreads();
#pragma unroll
    for (int j = 0; j < NV; j++) {
      uint32_t ancj = m->dof_ancmask[j];
      bool rel = (lane < NV) && (bit(anci, j) || bit(ancj, lane));
      T cj[6], bj[6];
      for (int k = 0; k < 6; k++) { cj[k] = s.cdof[j][k]; bj[k] = s.buf[j][k]; }
      T v = (j <= lane) ? dot6(cj, bf) : dot6(cd, bj);
      Mr[j] = rel ? v + ((j == lane) ? arm : T(0)) : T(0);
    }
  }

  // mj_comVel (cvel, cdof_dot), mj_passive, mj_fwdActuation, mj_rne -> fsmooth
  __device__ void velocity_forces() {
    int nv = m->nv;
    if (lane > 0 && lane < nb) {
      uint32_t ch = m->body_chainmask[lane];
      T v[6] = {0, 0, 0, 0, 0, 0};
      for (int j = 0; j < nv; j++)
        if ((ch >> j) & 1u) {
          T q = s.qvel[j];
          for (int k = 0; k < 6; k++) v[k] += s.cdof[j][k] * q;
        }
      for (int k = 0; k < 6; k++) s.cvel[lane][k] = v[k];
    }
    if (lane == 0)
      for (int k = 0; k < 6; k++) s.cvel[0][k] = 0;
    T cdd[6] = {0, 0, 0, 0, 0, 0};
    if (lane < NV) {
      uint32_t dm = m->dof_dotmask[lane];
      T v[6] = {0, 0, 0, 0, 0, 0};
      for (int j = 0; j < nv; j++)
        if ((dm >> j) & 1u) {
          T q = s.qvel[j];
          for (int k = 0; k < 6; k++) v[k] += s.cdof[j][k] * q;
        }
      cross_motion(v, cd, cdd);
      for (int k = 0; k < 6; k++) s.cdofdot[lane][k] = cdd[k];
    }
    __syncthreads();
    // RNE: cacc, cfrc_body
    if (lane > 0 && lane < nb) {
      uint32_t ch = m->body_chainmask[lane];
      T a[6] = {0, 0, 0, -m->gravity[0], -m->gravity[1], -m->gravity[2]};
      for (int j = 0; j < nv; j++)
        if ((ch >> j) & 1u) {
          T q = s.qvel[j];
          for (int k = 0; k < 6; k++) a[k] += s.cdofdot[j][k] * q;
        }
      T f[6], t[6], t2[6];
      mul_inert(s.cinert[lane], a, f);
      mul_inert(s.cinert[lane], s.cvel[lane], t);
      cross_force(s.cvel[lane], t, t2);
      for (int k = 0; k < 6; k++) s.cfrc[lane][k] = f[k] + t2[k];
    }
    __syncthreads();
    if (lane > 0 && lane < nb) {   // subtree sums of cfrc_body
      uint32_t dm = m->body_descmask[lane];
      T a[6] = {0, 0, 0, 0, 0, 0};
      for (int c = 1; c < nb; c++)
        if ((dm >> c) & 1u)
          for (int k = 0; k < 6; k++) a[k] += s.cfrc[c][k];
      for (int k = 0; k < 6; k++) s.bvel[lane][k] = a[k];
    }
    __syncthreads();
    fsmooth = 0;
    if (lane < NV) {
      T bias = dot6(cd, s.bvel[m->dof_bodyid[lane]]);
      int qa = m->dof_qposadr[lane];
      T pas = -m->dof_damping[lane] * s.qvel[lane];
      if (qa >= 0) pas -= m->dof_stiffness[lane] * (s.qpos[qa] - m->dof_springref[lane]);
      T act = 0;
      int u = m->dof_actuator[lane];
      if (u >= 0) {
        T c = s.ctrl[u];
        if (m->act_ctrllimited[u]) c = fmin(m->act_ctrlrange[u][1], fmax(m->act_ctrlrange[u][0], c));
        act = m->act_gear[u] * c;
      }
      s.qfrc_act[lane] = act;
      fsmooth = pas - bias + act;
    }
    __syncthreads();
  }

  // mj_collision + mj_makeConstraint + mj_makeImpedance + reference (aref)
  __device__ int collide_and_rows() {
    int overflow = 0;
    int ncon = 0;
    for (int base = 0; base < m->npair; base += WAVE) {
      int p = base + lane;
      Con<T> c0, c1;
      int n = 0;
      if (p < m->npair) n = collide_pair(m, s, p, c0, c1);
      uint64_t m1 = __ballot(n >= 1), m2 = __ballot(n >= 2);
      int pre = lanes_below(m1, lane) + lanes_below(m2, lane);
      int tot = __popcll(m1) + __popcll(m2);
      if (n >= 1) store_contact(s, ncon + pre, c0, p);
      if (n >= 2) store_contact(s, ncon + pre + 1, c1, p);
      ncon += tot;
    }
    if (ncon > MAXCON) { overflow = 1; ncon = MAXCON; }
    // limit rows: joints (lower side first), then tendons
    int nrow = 0;
    {
      bool lo = false, hi = false;
      if (lane < m->njnt && m->jnt_limited[lane]) {
        T q = s.qpos[m->jnt_qposadr[lane]];
        lo = (q - m->jnt_range[lane][0]) < m->jnt_margin[lane];
        hi = (m->jnt_range[lane][1] - q) < m->jnt_margin[lane];
      }
      uint64_t ml = __ballot(lo), mh = __ballot(hi);
      int pre = lanes_below(ml, lane) + lanes_below(mh, lane);
      if (lo) { s.row_kind[pre] = RK_JLO; s.row_id[pre] = lane; }
      if (hi) { s.row_kind[pre + lo] = RK_JHI; s.row_id[pre + lo] = lane; }
      nrow = __popcll(ml) + __popcll(mh);
    }
    {
      bool lo = false, hi = false;
      if (lane < m->ntendon && m->ten_limited[lane]) {
        T L = 0;
        for (int w = 0; w < m->ten_nwrap[lane]; w++) L += m->ten_wrapcoef[lane][w] * s.qpos[m->ten_wrapqadr[lane][w]];
        lo = (L - m->ten_range[lane][0]) < m->ten_margin[lane];
        hi = (m->ten_range[lane][1] - L) < m->ten_margin[lane];
      }
      uint64_t ml = __ballot(lo), mh = __ballot(hi);
      int pre = nrow + lanes_below(ml, lane) + lanes_below(mh, lane);
      if (lo) { s.row_kind[pre] = RK_TLO; s.row_id[pre] = lane; }
      if (hi) { s.row_kind[pre + lo] = RK_THI; s.row_id[pre + lo] = lane; }
      nrow += __popcll(ml) + __popcll(mh);
    }
    int nlim = nrow;
    {
      bool isc = lane < ncon;
      bool pyr = isc && m->pair_dim[s.con_pair[lane]] == 3;
      uint64_t mc = __ballot(isc), mp = __ballot(pyr);
      int pre = nrow + lanes_below(mc, lane) + 3 * lanes_below(mp, lane);
      int tot = __popcll(mc) + 3 * __popcll(mp);
      if (nrow + tot > MAXEFC) {   // drop whole contacts that do not fit (counted as overflow)
        overflow = 1;
        int fit = 0;
        for (int c = 0; c < ncon; c++) {
          int need = (m->pair_dim[s.con_pair[c]] == 3) ? 4 : 1;
          if (nrow + need > MAXEFC) break;
          nrow += need;
          fit++;
        }
        ncon = fit;
        isc = lane < ncon;
        tot = nrow - nlim;
        nrow = nlim;
      }
      if (isc) {
        s.con_adr[lane] = pre;
        if (!pyr) { s.row_kind[pre] = RK_CN; s.row_id[pre] = lane; }
        else for (int q = 0; q < 4; q++) { s.row_kind[pre + q] = RK_P0 + q; s.row_id[pre + q] = lane; }
      }
      nrow += tot;
    }
    if (lane == 0) { s.ncon = ncon; s.nefc = nrow; s.nlim = nlim; }
    // velocity of rows for aref uses J qvel: map qvel through J
    if (lane < NV) s.vx[lane] = s.qvel[lane];
    __syncthreads();
    map_vx(m, s, lane, m->nv, nb);
    for (int r = lane; r < nrow; r += WAVE) {
      int kind = s.row_kind[r], id = s.row_id[r];
      T pos, margin, dA;
      const T *sr, *si;
      if (kind <= RK_JHI) {
        T q = s.qpos[m->jnt_qposadr[id]];
        pos = kind == RK_JLO ? q - m->jnt_range[id][0] : m->jnt_range[id][1] - q;
        margin = m->jnt_margin[id];
        sr = m->jnt_solref[id]; si = m->jnt_solimp[id];
        dA = m->dof_invweight0[m->jnt_dofadr[id]];
      } else if (kind <= RK_THI) {
        T L = 0;
        for (int w = 0; w < m->ten_nwrap[id]; w++) L += m->ten_wrapcoef[id][w] * s.qpos[m->ten_wrapqadr[id][w]];
        pos = kind == RK_TLO ? L - m->ten_range[id][0] : m->ten_range[id][1] - L;
        margin = m->ten_margin[id];
        sr = m->ten_solref[id]; si = m->ten_solimp[id];
        dA = m->ten_invweight0[id];
      } else {
        int p = s.con_pair[id];
        pos = s.con_dist[id];
        margin = m->pair_margin[p];
        sr = m->pair_solref[p]; si = m->pair_solimp[p];
        T tran = m->body_invweight_tran[m->pair_b1[p]] + m->body_invweight_tran[m->pair_b2[p]];
        T mu = m->pair_mu[p];
        dA = kind == RK_CN ? tran : tran + mu * mu * tran;
      }
      T imp = impedance(si, pos, margin);
      T dmax = fmin(T(0.9999), fmax(T(0.0001), si[1]));
      T K, B;
      if (sr[0] > 0) {
        T tc = fmax(sr[0], 2 * m->timestep), dr = sr[1];
        K = T(1) / (dmax * dmax * tc * tc * dr * dr);
        B = T(2) / (dmax * tc);
      } else {
        K = -sr[0] / (dmax * dmax);
        B = -sr[1] / dmax;
      }
      T R = fmax(T(1e-15), (1 - imp) * dA / imp);
      s.row_D[r] = T(1) / R;
      T vel = row_Jx(m, s, r);
      s.row_aref[r] = -B * vel - K * imp * (pos - margin);
    }
    __syncthreads();
    return overflow;
  }

  // primal Newton (mj_solNewton semantics), warm-started; x = qacc
  __device__ void solve(T xws, int maxit, T tol) {
    int nv = m->nv;
    int nefc = s.nefc;
    T x = lane < NV ? xws : T(0);
    int r0 = lane, r1 = lane + WAVE;
    bool v0 = r0 < nefc, v1 = r1 < nefc;
    T D0 = v0 ? s.row_D[r0] : T(0), D1 = v1 ? s.row_D[r1] : T(0);
    T ar0 = v0 ? s.row_aref[r0] : T(0), ar1 = v1 ? s.row_aref[r1] : T(0);
    uint32_t anci = lane < NV ? m->dof_ancmask[lane] : 0u;
    T scale = m->newton_scale;
    // jar = J x - aref
    if (lane < NV) s.vx[lane] = x;
    __syncthreads();
    map_vx(m, s, lane, nv, nb);
    T jar0 = v0 ? row_Jx(m, s, r0) - ar0 : T(0);
    T jar1 = v1 ? row_Jx(m, s, r1) - ar1 : T(0);
    int it = 0;
    bool done = false;
    for (; it < maxit && !done; it++) {
      bool a0 = v0 && jar0 < 0, a1 = v1 && jar1 < 0;
      if (v0) s.row_f[r0] = a0 ? -D0 * jar0 : T(0);
      if (v1) s.row_f[r1] = a1 ? -D1 * jar1 : T(0);
      __syncthreads();
      contact_aggregates(m, s, lane);
      T Mx = matvec_rows(Mr, x);
      T jtf = jtf_lane(m, s, lane, cd);
      T g = lane < NV ? Mx - fsmooth - jtf : T(0);
      T gn = sqrt(wsum(g * g));
      if (scale * gn < tol) break;
      // Hessian lower rows: M + contact (tree form) + limits (diag) + dense rank-1 rows
      T H[NV];
      {
        T aug[6] = {0, 0, 0, 0, 0, 0};
        T dadd = 0;
        for (int c = 0; c < s.ncon; c++) {
          int p = s.con_pair[c];
          if (m->pair_b1[p] != 0) continue;
          if (!bit(m->body_chainmask[m->pair_b2[p]], lane)) continue;
          T r[3] = {s.con_pos[c][0] - s.com[0], s.con_pos[c][1] - s.com[1], s.con_pos[c][2] - s.com[2]};
          T w[3];
          cross3(cd, r, w);
          T jp[3] = {cd[3] + w[0], cd[4] + w[1], cd[5] + w[2]};
          const T* U = s.con_U[c];
          T z[3] = {U[0] * jp[0] + U[3] * jp[1] + U[4] * jp[2], U[3] * jp[0] + U[1] * jp[1] + U[5] * jp[2],
                    U[4] * jp[0] + U[5] * jp[1] + U[2] * jp[2]};
          T rz[3];
          cross3(r, z, rz);
          for (int k = 0; k < 3; k++) { aug[k] += rz[k]; aug[3 + k] += z[k]; }
        }
        for (int r = 0; r < s.nlim; r++) {
          int kind = s.row_kind[r];
          if (kind <= RK_JHI && s.row_f[r] != T(0) && m->jnt_dofadr[s.row_id[r]] == lane) dadd += s.row_D[r];
        }
#pragma unroll
        for (int j = 0; j < NV; j++) {
          T cj[6];
          for (int k = 0; k < 6; k++) cj[k] = s.cdof[j][k];
          bool rel = bit(anci, j);
          H[j] = Mr[j] + (rel ? dot6(cj, aug) : T(0)) + ((j == lane) ? dadd : T(0));
        }
        // dense rank-1 rows: tendon limits and body-body contacts
        for (int r = 0; r < nefc; r++) {
          int kind = s.row_kind[r];
          if (s.row_f[r] == T(0) || kind <= RK_JHI) continue;
          T jr = 0;
          int id = s.row_id[r];
          if (kind <= RK_THI) {
            for (int w = 0; w < m->ten_nwrap[id]; w++)
              if (m->ten_wrapdof[id][w] == lane) jr += m->ten_wrapcoef[id][w];
            if (kind == RK_THI) jr = -jr;
          } else {
            int p = s.con_pair[id];
            int b1 = m->pair_b1[p];
            if (b1 == 0) continue;
            int in2 = bit(m->body_chainmask[m->pair_b2[p]], lane), in1 = bit(m->body_chainmask[b1], lane);
            if (in1 != in2) {
              T rr[3] = {s.con_pos[id][0] - s.com[0], s.con_pos[id][1] - s.com[1], s.con_pos[id][2] - s.com[2]};
              T w[3], u[3];
              cross3(cd, rr, w);
              T jp[3] = {cd[3] + w[0], cd[4] + w[1], cd[5] + w[2]};
              row_u(m, s, kind, id, u);
              jr = in2 ? dot3(u, jp) : -dot3(u, jp);
            }
          }
          if (lane >= NV) jr = 0;
          T dj = s.row_D[r] * jr;
#pragma unroll
          for (int j = 0; j < NV; j++) H[j] += dj * rl(jr, j);
        }
      }
      chol_rows<NV>(H, lane);
      T sdir = -chol_solve<NV>(H, g, lane);
      if (lane >= NV) sdir = 0;
      // exact line search along sdir
      T Ms = matvec_rows(Mr, sdir);
      T A0 = wsum(lane < NV ? sdir * Ms : T(0));
      T B0 = wsum(lane < NV ? sdir * (Mx - fsmooth) : T(0));
      __syncthreads();
      if (lane < NV) s.vx[lane] = sdir;
      __syncthreads();
      map_vx(m, s, lane, nv, nb);
      T Js0 = v0 ? row_Jx(m, s, r0) : T(0), Js1 = v1 ? row_Jx(m, s, r1) : T(0);
      T lo = 0, hi = T(1e30), alpha = 1;
      T d0 = B0 + wsum((a0 ? D0 * jar0 * Js0 : T(0)) + (a1 ? D1 * jar1 * Js1 : T(0)));
      T ltol = (sizeof(T) == 8 ? T(1e-12) : T(1e-6)) * fabs(d0);
      for (int ls = 0; ls < 40; ls++) {
        T j0 = jar0 + alpha * Js0, j1 = jar1 + alpha * Js1;
        bool b0 = v0 && j0 < 0, b1 = v1 && j1 < 0;
        T d1 = B0 + alpha * A0 + wsum((b0 ? D0 * j0 * Js0 : T(0)) + (b1 ? D1 * j1 * Js1 : T(0)));
        if (fabs(d1) <= ltol) break;
        T d2 = A0 + wsum((b0 ? D0 * Js0 * Js0 : T(0)) + (b1 ? D1 * Js1 * Js1 : T(0)));
        if (d1 < 0) lo = alpha; else hi = alpha;
        T an = d2 > 0 ? alpha - d1 / d2 : T(-1);
        if (!(an > lo && an < hi)) an = hi < T(1e29) ? T(0.5) * (lo + hi) : T(2) * alpha;
        if (hi - lo <= (sizeof(T) == 8 ? T(1e-15) : T(1e-7)) * hi) break;
        alpha = an;
      }
      x += alpha * sdir;
      T nj0 = jar0 + alpha * Js0, nj1 = jar1 + alpha * Js1;
      bool changed = ((v0 && ((nj0 < 0) != a0)) || (v1 && ((nj1 < 0) != a1)));
      jar0 = nj0;
      jar1 = nj1;
      uint64_t anychg = __ballot(changed);
      if (anychg == 0 && fabs(alpha - T(1)) < T(1e-3)) done = true;
      __syncthreads();
    }
    niter = it;
    // final forces -> qfrc_constraint
    if (v0) s.row_f[r0] = jar0 < 0 ? -D0 * jar0 : T(0);
    if (v1) s.row_f[r1] = jar1 < 0 ? -D1 * jar1 : T(0);
    __syncthreads();
    contact_aggregates(m, s, lane);
    fcon = lane < NV ? jtf_lane(m, s, lane, cd) : T(0);
    qacc = x;
    __syncthreads();
  }

  // mj_Euler with implicit damping, mj_integratePos
  __device__ void euler(T& time) {
    T h = m->timestep;
    T He[NV];
    T damp = lane < NV ? m->dof_damping[lane] : T(0);
#pragma unroll
    for (int j = 0; j < NV; j++) He[j] = Mr[j] + ((j == lane) ? h * damp : T(0));
    chol_rows<NV>(He, lane);
    T a = chol_solve<NV>(He, fsmooth + fcon, lane);
    if (lane < NV) s.qvel[lane] += h * a;
    __syncthreads();
    if (lane < m->njnt) {
      int qa = m->jnt_qposadr[lane], da = m->jnt_dofadr[lane];
      if (m->jnt_type[lane] == JNT_FREE) {
        for (int k = 0; k < 3; k++) s.qpos[qa + k] += h * s.qvel[da + k];
        T w[3] = {s.qvel[da + 3], s.qvel[da + 4], s.qvel[da + 5]};
        T ang = h * normalize3(w);
        T sn = sin(T(0.5) * ang), cs = cos(T(0.5) * ang);
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
    __syncthreads();
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

template <typename T>
__device__ void reset_state(const DevModel<T>* __restrict__ m, Scratch<T>& s, int lane, T& time, T& xws) {
  if (lane < m->nq) s.qpos[lane] = m->qpos0[lane];
  if (lane < m->nv) s.qvel[lane] = 0;
  if (lane < m->nu) s.ctrl[lane] = 0;
  xws = 0;
  time = 0;
  __syncthreads();
}

template <typename T, int NV>
__device__ void physics_step(Stepper<T, NV>& st, const StepParams& p, T& time, T& xws, int* warn) {
  const DevModel<T>* __restrict__ m = st.m;
  Scratch<T>& s = st.s;
  int lane = st.lane;
  // mj_checkPos / mj_checkVel (auto-reset to qpos0, time 0)
  bool bq = lane < m->nq && isbad(s.qpos[lane]);
  bool bv = lane < m->nv && isbad(s.qvel[lane]);
  if (__ballot(bq)) { warn[WARN_BADQPOS]++; reset_state(m, s, lane, time, xws); }
  else if (__ballot(bv)) { warn[WARN_BADQVEL]++; reset_state(m, s, lane, time, xws); }
  for (int attempt = 0; attempt < 2; attempt++) {
    st.kinematics();
    st.mass_matrix();
    st.velocity_forces();
    if (st.collide_and_rows()) warn[WARN_OVERFLOW]++;
    st.solve(xws, p.max_newton, sizeof(T) == 8 ? T(1e-13) : T(1e-7));
    bool ba = lane < m->nv && isbad(st.qacc);
    if (!__ballot(ba) || attempt == 1) break;
    warn[WARN_BADQACC]++;   // mj_checkAcc: reset and redo mj_forward
    reset_state(m, s, lane, time, xws);
  }
  st.euler(time);
  xws = st.qacc;
}

template <typename T>
__device__ T compute_reward(const DevModel<T>* __restrict__ m, const Scratch<T>& s, const StepParams& p, T time) {
  // quaternion_to_euler (utils.py:3-21): pitch = arcsin(2(wy - zx)), not clamped
  T w = s.qpos[3], x = s.qpos[4], y = s.qpos[5], z = s.qpos[6];
  T roll = atan2(2 * (w * x + y * z), 1 - 2 * (x * x + y * y));
  T pitch = asin(2 * (w * y - z * x));
  T h = s.qpos[2];
  int nu = m->nu;
  if (p.reward_id == REWARD_STAND || p.reward_id == REWARD_WALK) {
    T c2 = 0;
    for (int u = 0; u < nu; u++) c2 += s.ctrl[u] * s.ctrl[u];
    T torque = exp(T(-0.05) * c2);
    T post = T(0.5) * exp(T(-2) * (h - T(1.282)) * (h - T(1.282))) + T(0.5) * exp(T(-3) * (roll * roll + pitch * pitch));
    if (p.reward_id == REWARD_STAND) {
      // cfrc_ext is never computed by mj_step without sensors -> both "feet" forces are 0
      T lf = 0, rf = 0;
      T foot = 1 - fmin(lf, rf) / (lf + rf + T(1e-8));
      T vr = exp(T(-2) * (s.qvel[0] - 1) * (s.qvel[0] - 1));
      T r = T(0.4) * vr + T(0.3) * post + T(0.2) * foot + T(0.1) * torque;
      return h < T(0.8) ? T(0) : r;
    }
    T vr = exp(T(-0.5) * (s.qvel[0] - 10) * (s.qvel[0] - 10));
    return h < T(0.8) ? T(0.1) * h / T(0.8) : vr + post * torque;
  }
  if (p.reward_id == REWARD_KNEELING) {
    const double* k = p.kneel;   // target_height, min_height, max_roll_pitch, com_radius, energy_w, posture_w, com_w, foot_w, alive_w
    if (h < T(k[1])) return h * h;
    T mrp = T(k[2]);
    T posture = T(0.7) * exp(T(-5) * (roll * roll + pitch * pitch) / (mrp * mrp)) +
                T(0.3) * exp(T(-5) * (h - T(k[0])) * (h - T(k[0])));
    T dist = sqrt(s.com[0] * s.com[0] + s.com[1] * s.com[1]);
    T comv = T(0);   // subtree_linvel is lazy in MuJoCo -> 0
    T com = T(0.7) * exp(T(-10) * (dist / T(k[3]))) + T(0.3) * exp(T(-0.1) * comv);
    T foot = T(0);   // min(0,0)/(0+0+1e-8)
    T jp = 0;
    for (int i = 6; i < m->nv; i++) { T t = s.qfrc_act[i] * s.qvel[i]; jp += t * t; }
    T energy = exp(T(-0.01) * jp);
    T alive = 1 - exp(T(-0.5) * time);
    return T(k[5]) * posture + T(k[6]) * com + T(k[7]) * foot + T(k[4]) * energy + T(k[8]) * alive;
  }
  return T(0);
}

template <typename T>
__device__ void write_obs(const DevModel<T>* __restrict__ m, const Scratch<T>& s, int lane, T* out, int obs_dim) {
  int nq = m->nq, nv = m->nv, nb = m->nbody;
  int o1 = nq - 2, o2 = o1 + nv, o3 = o2 + 10 * nb, o4 = o3 + 6 * nb;
  for (int k = lane; k < obs_dim; k += WAVE) {
    T v;
    if (k < o1) v = s.qpos[2 + k];
    else if (k < o2) v = s.qvel[k - o1];
    else if (k < o3) { int q = k - o2; v = s.cinert[q / 10][q % 10]; }
    else if (k < o4) { int q = k - o3; v = s.cvel[q / 6][q % 6]; }
    else v = s.qfrc_act[k - o4];
    out[k] = v;
  }
}

template <typename T, int NV>
__device__ void dump_debug(const Stepper<T, NV>& st, T* dbg) {
  const Scratch<T>& s = st.s;
  const DevModel<T>* m = st.m;
  int lane = st.lane;
  for (int k = lane; k < MAXBODY * 3; k += WAVE) dbg[k] = s.xpos[k / 3][k % 3];
  for (int k = lane; k < MAXBODY * 4; k += WAVE) dbg[100 + k] = s.xquat[k / 4][k % 4];
  for (int k = lane; k < MAXBODY * 10; k += WAVE) dbg[200 + k] = s.cinert[k / 10][k % 10];
  for (int k = lane; k < MAXDOF * 6; k += WAVE) dbg[500 + k] = s.cdof[k / 6][k % 6];
  if (lane < NV)
    for (int j = 0; j < NV; j++) dbg[700 + lane * MAXDOF + j] = st.Mr[j];
  for (int k = lane; k < MAXBODY * 6; k += WAVE) dbg[1800 + k] = s.cvel[k / 6][k % 6];
  for (int k = lane; k < MAXDOF * 6; k += WAVE) dbg[2000 + k] = s.cdofdot[k / 6][k % 6];
  if (lane < NV) {
    dbg[2280 + lane] = s.qfrc_act[lane];
    dbg[2320 + lane] = st.fsmooth;
    dbg[2360 + lane] = st.fcon;
    dbg[2400 + lane] = st.qacc;
  }
  if (lane == 0) {
    dbg[2500] = s.com[0]; dbg[2501] = s.com[1]; dbg[2502] = s.com[2];
    dbg[2503] = s.ncon; dbg[2504] = s.nefc; dbg[2505] = st.niter; dbg[2506] = s.nlim;
  }
  for (int c = lane; c < s.ncon; c += WAVE) {
    T* o = dbg + 2600 + 11 * c;
    for (int k = 0; k < 3; k++) { o[k] = s.con_pos[c][k]; o[3 + k] = s.con_n[c][k]; o[6 + k] = s.con_t1[c][k]; }
    o[9] = s.con_dist[c];
    o[10] = s.con_pair[c];
  }
  for (int r = lane; r < s.nefc; r += WAVE) {
    T* o = dbg + 3200 + 6 * r;
    o[0] = s.row_kind[r]; o[1] = s.row_id[r]; o[2] = s.row_D[r]; o[3] = s.row_aref[r]; o[4] = s.row_f[r];
  }
  for (int k = lane; k < MAXGEOM * 3; k += WAVE) { dbg[4000 + k] = s.gpos[k / 3][k % 3]; dbg[4100 + k] = s.gax[k / 3][k % 3]; }
  for (int k = lane; k < MAXBODY * 3; k += WAVE) dbg[4200 + k] = s.xipos[k / 3][k % 3];
  (void)m;
}

// ------------------------------------------------------------------ the kernel
template <typename T, int NV>
__global__ __launch_bounds__(64) void step_kernel(const DevModel<T>* __restrict__ m, EnvBuffers<T> b,
                                                  const float* __restrict__ actions,
                                                  const uint8_t* __restrict__ reset_mask,
                                                  const T* __restrict__ nz_q, const T* __restrict__ nz_v,
                                                  StepParams p, int nenv) {
  __shared__ Scratch<T> s;
  const int env = blockIdx.x;
  const int lane = threadIdx.x;
  if (env >= nenv) return;
  if (p.mode == MODE_RESET && reset_mask && !reset_mask[env]) return;
  const int nq = m->nq, nv = m->nv, nu = m->nu;
  Stepper<T, NV> st(m, s, lane);
  int warn[NWARN] = {0, 0, 0, 0};
  T time = b.time[env];
  T xws = (lane < nv) ? b.qacc_ws[(size_t)env * nv + lane] : T(0);
  if (lane < nq) s.qpos[lane] = b.qpos[(size_t)env * nq + lane];
  if (lane < nv) s.qvel[lane] = b.qvel[(size_t)env * nv + lane];
  if (lane < nu) s.ctrl[lane] = b.ctrl[(size_t)env * nu + lane];
  __syncthreads();

  bool do_reset = p.mode == MODE_RESET;
  int step_count = b.step_count[env];
  uint32_t episode = b.episode[env];
  T total = b.total_reward[env];
  if (p.mode == MODE_ENV_STEP || p.mode == MODE_PHYSICS) {
    for (int sub = 0; sub < p.nsub; sub++) {
      // data.ctrl[:] = action each substep (custom_env.py:159); mj_resetData may have zeroed it
      if (lane < nu && actions) s.ctrl[lane] = (T)actions[(size_t)env * nu + lane];
      __syncthreads();
      physics_step(st, p, time, xws, warn);
      if (b.dbg && env == 0) dump_debug(st, b.dbg);
    }
    write_obs(m, s, lane, b.obs + (size_t)env * p.obs_dim, p.obs_dim);
    if (p.mode == MODE_ENV_STEP) {
      step_count += 1;
      bool trunc = step_count >= p.max_steps;
      T r = trunc ? T(0) : compute_reward(m, s, p, time);
      total += r;
      bool term = (double)time >= p.duration;
      if (lane == 0) {
        b.reward[env] = r;
        b.terminated[env] = term;
        b.truncated[env] = trunc;
      }
      if ((term || trunc) && p.autoreset) {
        write_obs(m, s, lane, b.terminal_obs + (size_t)env * p.obs_dim, p.obs_dim);
        do_reset = true;
      }
    }
  }
  if (do_reset) {
    // custom_env.py:97-130: mj_resetData; qpos = init (z=1.282, upright); += U(+-0.01) noise with
    // z noise x0.1 and no quaternion noise; qvel = U(+-0.01); one mj_step with ctrl = 0.
    episode += 1;
    T sc = (T)p.noise_scale;
    if (lane < nq) {
      T q = m->qpos0[lane];
      if (m->jnt_type[0] == JNT_FREE) {
        if (lane == 2) q = (T)p.init_height;
        if (lane >= 3 && lane < 7) q = lane == 3 ? T(1) : T(0);
      }
      T nzq = nz_q ? nz_q[(size_t)env * nq + lane] : uniform_pm<T>(p.seed, env, episode, lane, sc);
      if (m->jnt_type[0] == JNT_FREE) {
        if (lane == 2) nzq *= T(0.1);
        if (lane >= 3 && lane < 7) nzq = 0;
      }
      s.qpos[lane] = q + nzq;
    }
    if (lane < nv) s.qvel[lane] = nz_v ? nz_v[(size_t)env * nv + lane] : uniform_pm<T>(p.seed, env, episode, 64 + lane, sc);
    if (lane < nu) s.ctrl[lane] = 0;
    xws = 0;
    time = 0;
    __syncthreads();
    physics_step(st, p, time, xws, warn);
    if (b.dbg && env == 0) dump_debug(st, b.dbg);
    write_obs(m, s, lane, b.obs + (size_t)env * p.obs_dim, p.obs_dim);
    step_count = 0;
    total = 0;
  }
  // write back state
  if (lane < nq) b.qpos[(size_t)env * nq + lane] = s.qpos[lane];
  if (lane < nv) { b.qvel[(size_t)env * nv + lane] = s.qvel[lane]; b.qacc_ws[(size_t)env * nv + lane] = xws; }
  if (lane < nu) b.ctrl[(size_t)env * nu + lane] = s.ctrl[lane];
  if (lane < nv) b.aux[(size_t)env * AUXDIM + lane] = st.qacc;
  if (lane == 0) {
    b.time[env] = time;
    b.step_count[env] = step_count;
    b.episode[env] = episode;
    b.total_reward[env] = total;
    T* a = b.aux + (size_t)env * AUXDIM;
    a[MAXDOF + 0] = s.com[0]; a[MAXDOF + 1] = s.com[1]; a[MAXDOF + 2] = s.com[2];
    a[MAXDOF + 3] = (T)s.ncon; a[MAXDOF + 4] = (T)s.nefc; a[MAXDOF + 5] = (T)st.niter;
    for (int k = 0; k < NWARN; k++) b.warning[(size_t)env * NWARN + k] += warn[k];
  }
}

}  // namespace

template <typename T>
hipError_t launch_step(const DevModel<T>* dmodel, int nv, const EnvBuffers<T>& b, const float* actions,
                       const uint8_t* reset_mask, const T* noise_qpos, const T* noise_qvel,
                       const StepParams& p, int nenv, hipStream_t stream) {
  if (nenv <= 0) return hipSuccess;
  dim3 grid(nenv), block(WAVE);
  switch (nv) {
    case 27:
      hipLaunchKernelGGL((step_kernel<T, 27>), grid, block, 0, stream, dmodel, b, actions, reset_mask, noise_qpos,
                         noise_qvel, p, nenv);
      break;
    default:
      return hipErrorInvalidValue;
  }
  return hipGetLastError();
}

template hipError_t launch_step<float>(const DevModel<float>*, int, const EnvBuffers<float>&, const float*,
                                       const uint8_t*, const float*, const float*, const StepParams&, int,
                                       hipStream_t);
template hipError_t launch_step<double>(const DevModel<double>*, int, const EnvBuffers<double>&, const float*,
                                        const uint8_t*, const double*, const double*, const StepParams&, int,
                                        hipStream_t);

}  // namespace hs

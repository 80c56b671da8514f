// hsim C ABI implementation (product).  See include/hsim.h for the reference interfaces replaced.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <string>
#include <vector>

#include "../../include/hsim.h"
#include "hs_kernels.h"
#include "mjcf.h"

struct hs_model {
  hs::HostModel host;
};

struct hs_batch {
  const hs_model* model = nullptr;
  int n = 0, device = 0, precision = HS_FP32, obs_dim = 0;
  bool full_state = false;
  uint64_t seed = 0;
  void* dmodel = nullptr;
  hs_buffers buf{};
  bool owns = false;
  void* dbg = nullptr;
  bool debug = false;
  const void* ar_qpos_noise = nullptr;       // bound auto-reset noise [n][nq] / [n][nv] (null: device RNG)
  const void* ar_qvel_noise = nullptr;
  int* redo = nullptr;                       // wide-tier work list [2 + n] (kernel-managed)
  unsigned long long* redo_total = nullptr;  // cumulative wide-tier re-runs
  void* mid = nullptr;                       // chunk-queue hand-off rows [n][MIDDIM] (kernel-managed)
  int* qsync = nullptr;                      // chunk queue claim / exit counters, pair flags (qsync_words)
  hs_env_config cfg{};
  bool ctrl_stale = false;                   // env steps ran with HS_OUT_CTRL off: buf.ctrl is not data.ctrl
  int lose_env1 = 0;                         // hs_debug_lose_handoff test hook (env + 1; 0 = off)
  void* tape_backup = nullptr;               // hs_step_tape / hs_rollout: the state before a tape launch (replay on abort)
  size_t tape_backup_bytes = 0;
  unsigned long long tape_aborts = 0;        // tape launches replayed step by step (resident-tier overflow)
  hipStream_t last_stream = nullptr;         // stream of the batch's previous launch (order_streams)
  bool last_valid = false;
  hipEvent_t order_ev = nullptr;
  unsigned long long stream_orders = 0;      // cross-stream waits inserted (diagnostics)
  hipEvent_t tape_ev[2] = {nullptr, nullptr};   // around the last tape / rollout kernel launch
  float last_tape_ms = -1.f;                 // its duration (hs_last_tape_ms)
};

namespace {
thread_local std::string g_err;

int fail(const std::string& msg) {
  g_err = msg;
  return -1;
}
bool hip_ok(hipError_t e, const char* what) {
  if (e == hipSuccess) return true;
  g_err = std::string(what) + ": " + hipGetErrorString(e);
  return false;
}

struct DeviceGuard {
  int prev = -1;
  explicit DeviceGuard(int dev) {
    if (hipGetDevice(&prev) != hipSuccess) prev = -1;
    if (prev != dev) (void)hipSetDevice(dev);
  }
  ~DeviceGuard() {
    int cur;
    if (prev >= 0 && hipGetDevice(&cur) == hipSuccess && cur != prev) (void)hipSetDevice(prev);
  }
};

// Uncached device memory (the chunk queue's hand-off rows, claim / exit / epoch words and pair
// flags) is recycled only as uncached memory: freed blocks go to a per-device list instead of
// hipFree, for the life of the process.  Round-3 finding: after a batch was destroyed, its hipFree'd
// UNCACHED hand-off rows were handed back out as ordinary memory -- torch tensors of the next batch --
// and a few hundred obs rows of that batch intermittently read back stale values
// (tools/probes/gpu_queue_wide_probe.py: 3 of 3 runs before, none after); keeping UC memory out of the
// general pool removes that path.  Sizes are rounded up to a power of two (>= 64 KB), and a request
// takes a free block of exactly its size class, so batches of any mix of sizes reuse blocks and the
// pool holds at most the peak of concurrently live uncached memory per class -- it never has to
// give a block back (a bounded list did, round 4, and re-opened the hazard for workloads with many
// batch sizes).
struct UcBlock { int device; size_t bytes; void* ptr; };
std::mutex g_uc_mu;
std::vector<UcBlock> g_uc_free;

size_t uc_class(size_t bytes) {
  size_t c = (size_t)64 << 10;
  while (c < bytes) c <<= 1;
  return c;
}

bool uc_alloc(int device, size_t bytes, void** out) {
  const size_t cls = uc_class(bytes);
  {
    std::lock_guard<std::mutex> lk(g_uc_mu);
    for (size_t i = 0; i < g_uc_free.size(); i++)
      if (g_uc_free[i].device == device && g_uc_free[i].bytes == cls) {
        *out = g_uc_free[i].ptr;
        g_uc_free.erase(g_uc_free.begin() + (long)i);
        return true;
      }
  }
  return hipExtMallocWithFlags(out, cls, hipDeviceMallocUncached) == hipSuccess;
}

void uc_release(int device, size_t bytes, void* ptr) {
  if (!ptr) return;
  std::lock_guard<std::mutex> lk(g_uc_mu);
  g_uc_free.push_back({device, uc_class(bytes), ptr});
}

// Launches of one batch are ordered across streams (include/hsim.h): when a call comes on another
// stream than the batch's previous one, the new stream first waits for everything issued on the old
// one (an event recorded there now).  Streams in graph capture are left alone -- the capturing
// framework orders the capture against the streams it forked from, and an event recorded outside a
// capture cannot be waited on inside it.
int order_streams(hs_batch* b, hipStream_t st) {
  if (b->last_valid && st != b->last_stream) {
    hipStreamCaptureStatus cn = hipStreamCaptureStatusNone, co = hipStreamCaptureStatusNone;
    if (!hip_ok(hipStreamIsCapturing(st, &cn), "hipStreamIsCapturing") ||
        !hip_ok(hipStreamIsCapturing(b->last_stream, &co), "hipStreamIsCapturing"))
      return -1;
    if (cn == hipStreamCaptureStatusNone && co == hipStreamCaptureStatusNone) {
      if (!b->order_ev && !hip_ok(hipEventCreateWithFlags(&b->order_ev, hipEventDisableTiming), "hipEventCreate"))
        return -1;
      if (!hip_ok(hipEventRecord(b->order_ev, b->last_stream), "stream order (record)") ||
          !hip_ok(hipStreamWaitEvent(st, b->order_ev, 0), "stream order (wait)"))
        return -1;
      b->stream_orders++;
    }
  }
  b->last_stream = st;
  b->last_valid = true;
  return 0;
}

int obs_dim_of(const hs::HostModel& m) { return (m.nq - 2) + m.nv + 10 * m.nbody + 6 * m.nbody + m.nv; }

template <typename T>
hs::EnvBuffers<T> env_buffers(const hs_batch* b) {
  hs::EnvBuffers<T> e;
  e.qpos = (T*)b->buf.qpos;
  e.qvel = (T*)b->buf.qvel;
  e.qacc_ws = (T*)b->buf.qacc_warmstart;
  e.ctrl = (T*)b->buf.ctrl;
  e.time = (T*)b->buf.time;
  e.step_count = b->buf.step_count;
  e.episode = b->buf.episode;
  e.total_reward = (T*)b->buf.total_reward;
  e.warning = b->buf.warning;
  e.obs = (T*)b->buf.obs;
  e.terminal_obs = (T*)b->buf.terminal_obs;
  e.reward = (T*)b->buf.reward;
  e.terminated = b->buf.terminated;
  e.truncated = b->buf.truncated;
  e.aux = (T*)b->buf.aux;
  e.cfrc_ext = (T*)b->buf.cfrc_ext;
  e.subtree_linvel = (T*)b->buf.subtree_linvel;
  e.term_step_count = b->buf.terminal_step_count;
  e.term_total_reward = (T*)b->buf.terminal_total_reward;
  e.redo = b->redo;
  e.redo_total = b->redo_total;
  e.mid = (T*)b->mid;
  e.qsync = b->qsync;
  e.dbg = b->debug ? (T*)b->dbg : nullptr;
  return e;
}

hs::StepParams params_of(const hs_batch* b, int mode, int nsub) {
  hs::StepParams p{};
  p.mode = mode;
  p.nsub = nsub;
  p.max_steps = b->cfg.max_steps;
  p.reward_id = b->cfg.reward_id;
  p.autoreset = b->cfg.autoreset;
  p.obs_dim = b->obs_dim;
  p.max_newton = b->cfg.max_newton;
  p.full_state = b->full_state ? 1 : 0;
  p.duration = b->cfg.duration;
  p.init_height = b->cfg.init_height;
  p.noise_scale = b->cfg.noise_scale;
  p.seed = b->seed;
  for (int k = 0; k < 9; k++) p.kneel[k] = b->cfg.kneel_params[k];
  p.solver = b->model->host.solver == 1 ? hs::SOLVER_PGS : hs::SOLVER_NEWTON;
  p.outputs = b->cfg.outputs;
  p.schedule = b->cfg.schedule;
  p.dbg_lose_pair1 = b->lose_env1;          // (launch_step maps it to the queue unit)
  return p;
}

int launch(hs_batch* b, int mode, const float* act, const uint8_t* mask, const void* nq, const void* nvz, int nsub,
           void* stream, int nsteps = 1, const hs_tape_out* tape = nullptr, const hs::RolloutArgs* ro = nullptr) {
  if (!b) return fail("null batch");
  DeviceGuard g(b->device);
  if (order_streams(b, (hipStream_t)stream)) return -1;
  hipError_t e;
  auto p = params_of(b, mode, nsub);
  p.nsteps = nsteps;
  int nv = b->model->host.nv;
  if (b->precision == HS_FP64) {
    hs::TapeOut<double> to{tape ? (double*)tape->obs : nullptr, tape ? (double*)tape->reward : nullptr,
                           tape ? tape->terminated : nullptr, tape ? tape->truncated : nullptr};
    e = hs::launch_step<double>((const hs::DevModel<double>*)b->dmodel, nv, env_buffers<double>(b), act, mask,
                                (const double*)nq, (const double*)nvz, p, b->n, (hipStream_t)stream, &to, ro);
  } else {
    hs::TapeOut<float> to{tape ? (float*)tape->obs : nullptr, tape ? (float*)tape->reward : nullptr,
                          tape ? tape->terminated : nullptr, tape ? tape->truncated : nullptr};
    e = hs::launch_step<float>((const hs::DevModel<float>*)b->dmodel, nv, env_buffers<float>(b), act, mask,
                               (const float*)nq, (const float*)nvz, p, b->n, (hipStream_t)stream, &to);
  }
  if (e == hipErrorInvalidValue) return fail("no kernel instance for this model's nv (compiled: nv = 27)");
  return hip_ok(e, "step kernel launch") ? 0 : -1;
}

// -- tape launches (hs_step_tape, hs_rollout) --------------------------------------------------
// Each env finishes at most one episode per tape launch (its terminal obs / info rows are then written
// once, see hs_kernels.hip step_pair): launches of at most the shortest episode's length.  An episode
// starts at time = one timestep (the reset's mj_step) and ends at time >= duration (custom_env.py:213)
// or at max_steps.
int min_episode_len(const hs_batch* b) {
  const auto& h = b->model->host;
  const double dt = h.timestep * b->cfg.frame_skip;
  const double spans = std::floor((b->cfg.duration - h.timestep) / dt - 1e-9);
  return (int)std::max(1.0, std::min((double)b->cfg.max_steps, spans));
}

struct Region { void* p; size_t bytes; };

// the env state a tape launch changes (restored when it aborts on a resident-tier overflow)
std::vector<Region> state_regions(const hs_batch* b) {
  const auto& h = b->model->host;
  const size_t N = (size_t)b->n, es = b->precision == HS_FP64 ? 8 : 4;
  return {{b->buf.qpos, N * h.nq * es}, {b->buf.qvel, N * h.nv * es}, {b->buf.qacc_warmstart, N * h.nv * es},
          {b->buf.ctrl, N * h.nu * es}, {b->buf.time, N * es}, {b->buf.total_reward, N * es},
          {b->buf.step_count, N * 4}, {b->buf.episode, N * 4}, {b->buf.warning, N * HS_NWARN * 4},
          {b->redo_total, sizeof(unsigned long long)}};
}

// Back up `regs`, run `go` (the tape launch), and read the abort word: 0 = done, 1 = aborted (the
// regions are restored and the redo list cleared), -1 = error.  Synchronizes the stream.
template <typename F>
int guarded_tape(hs_batch* b, const std::vector<Region>& regs, hipStream_t st, F&& go) {
  size_t total = 0;
  for (auto& r : regs) total += (r.bytes + 255) & ~(size_t)255;
  if (total > b->tape_backup_bytes) {
    if (b->tape_backup) (void)hipFree(b->tape_backup);
    b->tape_backup = nullptr;
    b->tape_backup_bytes = 0;
    if (!hip_ok(hipMalloc(&b->tape_backup, total), "hipMalloc(tape backup)")) return -1;
    b->tape_backup_bytes = total;
  }
  size_t off = 0;
  for (auto& r : regs) {
    if (!hip_ok(hipMemcpyAsync((char*)b->tape_backup + off, r.p, r.bytes, hipMemcpyDeviceToDevice, st), "tape backup"))
      return -1;
    off += (r.bytes + 255) & ~(size_t)255;
  }
  if (!hip_ok(hipMemsetAsync(b->qsync + hs::QS_ABORT, 0, sizeof(int), st), "tape abort word")) return -1;
  // HIP events right around the kernel launch on its stream (hs_last_tape_ms: the bench's roofline of
  // the fused rollout kernel); one pair per tape launch, which is one per several env steps
  for (auto& e : b->tape_ev)
    if (!e && !hip_ok(hipEventCreate(&e), "hipEventCreate")) return -1;
  if (!hip_ok(hipEventRecord(b->tape_ev[0], st), "tape event")) return -1;
  int rc = go();
  if (rc) return rc < 0 ? rc : -1;
  if (!hip_ok(hipEventRecord(b->tape_ev[1], st), "tape event")) return -1;
  int aborted = 0;
  if (!hip_ok(hipMemcpyAsync(&aborted, b->qsync + hs::QS_ABORT, sizeof(int), hipMemcpyDeviceToHost, st),
              "tape abort word") ||
      !hip_ok(hipStreamSynchronize(st), "tape launch"))
    return -1;
  if (!hip_ok(hipEventElapsedTime(&b->last_tape_ms, b->tape_ev[0], b->tape_ev[1]), "tape event time")) return -1;
  if (!aborted) return 0;
  off = 0;
  for (auto& r : regs) {
    if (!hip_ok(hipMemcpyAsync(r.p, (char*)b->tape_backup + off, r.bytes, hipMemcpyDeviceToDevice, st), "tape restore"))
      return -1;
    off += (r.bytes + 255) & ~(size_t)255;
  }
  if (!hip_ok(hipMemsetAsync(b->redo, 0, 2 * sizeof(int), st), "tape redo list")) return -1;
  b->tape_aborts++;
  return 1;
}

template <typename T>
bool upload_model(hs_batch* b, std::string& err) {
  auto* d = new hs::DevModel<T>();
  if (!hs::build_dev_model<T>(b->model->host, *d, err)) { delete d; return false; }
  if (!hip_ok(hipMalloc(&b->dmodel, sizeof(hs::DevModel<T>)), "hipMalloc(model)")) { delete d; err = g_err; return false; }
  bool ok = hip_ok(hipMemcpy(b->dmodel, d, sizeof(hs::DevModel<T>), hipMemcpyHostToDevice), "upload model");
  delete d;
  if (!ok) err = g_err;
  return ok;
}

template <typename T>
bool init_state(hs_batch* b) {
  const auto& m = b->model->host;
  int N = b->n;
  std::vector<T> q((size_t)N * m.nq);
  for (int i = 0; i < N; i++)
    for (int k = 0; k < m.nq; k++) q[(size_t)i * m.nq + k] = (T)m.qpos0[k];
  size_t es = sizeof(T);
  return hip_ok(hipMemcpy(b->buf.qpos, q.data(), q.size() * es, hipMemcpyHostToDevice), "init qpos") &&
         hip_ok(hipMemset(b->buf.qvel, 0, (size_t)N * m.nv * es), "init") &&
         hip_ok(hipMemset(b->buf.qacc_warmstart, 0, (size_t)N * m.nv * es), "init") &&
         hip_ok(hipMemset(b->buf.ctrl, 0, (size_t)N * m.nu * es), "init") &&
         hip_ok(hipMemset(b->buf.time, 0, (size_t)N * es), "init") &&
         hip_ok(hipMemset(b->buf.step_count, 0, (size_t)N * 4), "init") &&
         hip_ok(hipMemset(b->buf.episode, 0, (size_t)N * 4), "init") &&
         hip_ok(hipMemset(b->buf.total_reward, 0, (size_t)N * es), "init") &&
         hip_ok(hipMemset(b->buf.warning, 0, (size_t)N * HS_NWARN * 4), "init") &&
         hip_ok(hipMemset(b->buf.obs, 0, (size_t)N * b->obs_dim * es), "init") &&
         hip_ok(hipMemset(b->buf.terminal_obs, 0, (size_t)N * b->obs_dim * es), "init") &&
         hip_ok(hipMemset(b->buf.reward, 0, (size_t)N * es), "init") &&
         hip_ok(hipMemset(b->buf.terminated, 0, (size_t)N), "init") &&
         hip_ok(hipMemset(b->buf.truncated, 0, (size_t)N), "init") &&
         hip_ok(hipMemset(b->buf.aux, 0, (size_t)N * hs::AUXDIM * es), "init") &&
         (!b->buf.cfrc_ext || hip_ok(hipMemset(b->buf.cfrc_ext, 0, (size_t)N * m.nbody * 6 * es), "init")) &&
         (!b->buf.subtree_linvel || hip_ok(hipMemset(b->buf.subtree_linvel, 0, (size_t)N * m.nbody * 3 * es), "init")) &&
         (!b->buf.terminal_step_count || hip_ok(hipMemset(b->buf.terminal_step_count, 0, (size_t)N * 4), "init")) &&
         (!b->buf.terminal_total_reward || hip_ok(hipMemset(b->buf.terminal_total_reward, 0, (size_t)N * es), "init")) &&
         hip_ok(hipMemset(b->redo, 0, (size_t)(N + 2) * sizeof(int)), "init") &&
         hip_ok(hipMemset(b->redo_total, 0, sizeof(unsigned long long)), "init") &&
         hip_ok(hipMemset(b->qsync, 0, hs::qsync_words(N) * sizeof(int)), "init") &&
         // a recycled UC block holds another batch's rows: a lost hand-off reads this row's warning
         // counters and time (hs_kernels.hip step_pair), so they start at 0, not at stale bits
         hip_ok(hipMemset(b->mid, 0, (size_t)N * hs::MIDDIM * es), "init");
}

template <typename T>
int state_io(hs_batch* b, int dir, double* qpos, double* qvel, double* warm, double* time, double* ctrl) {
  const auto& m = b->model->host;
  size_t N = (size_t)b->n;
  struct Item { void* dev; double* host; size_t n; } items[] = {
      {b->buf.qpos, qpos, N * m.nq}, {b->buf.qvel, qvel, N * m.nv}, {b->buf.qacc_warmstart, warm, N * m.nv},
      {b->buf.time, time, N}, {b->buf.ctrl, ctrl, N * m.nu}};
  for (auto& it : items) {
    if (!it.host) continue;
    std::vector<T> tmp(it.n);
    if (dir == 0) {
      if (!hip_ok(hipMemcpy(tmp.data(), it.dev, it.n * sizeof(T), hipMemcpyDeviceToHost), "state get")) return -1;
      for (size_t k = 0; k < it.n; k++) it.host[k] = (double)tmp[k];
    } else {
      for (size_t k = 0; k < it.n; k++) tmp[k] = (T)it.host[k];
      if (!hip_ok(hipMemcpy(it.dev, tmp.data(), it.n * sizeof(T), hipMemcpyHostToDevice), "state set")) return -1;
    }
  }
  return 0;
}
template <typename T>
int kinematics_io(hs_batch* b, int env, const double* qpos, double* xpos, double* xmat, double* gxpos,
                  double* gzaxis, double* com) {
  const auto& m = b->model->host;
  T* dq = nullptr;
  T* dout = nullptr;
  int rc = -1;
  std::vector<T> out(hs::KINDIM);
  if (!hip_ok(hipMalloc(&dq, m.nq * sizeof(T)), "kinematics alloc") ||
      !hip_ok(hipMalloc(&dout, hs::KINDIM * sizeof(T)), "kinematics alloc"))
    goto done;
  if (qpos) {
    std::vector<T> q(qpos, qpos + m.nq);
    if (!hip_ok(hipMemcpy(dq, q.data(), m.nq * sizeof(T), hipMemcpyHostToDevice), "kinematics qpos")) goto done;
  } else if (!hip_ok(hipMemcpy(dq, (const T*)b->buf.qpos + (size_t)env * m.nq, m.nq * sizeof(T),
                               hipMemcpyDeviceToDevice), "kinematics qpos")) {
    goto done;
  }
  if (!hip_ok(hs::launch_kinematics<T>((const hs::DevModel<T>*)b->dmodel, m.nv, dq, dout, nullptr), "kinematics launch") ||
      !hip_ok(hipMemcpy(out.data(), dout, hs::KINDIM * sizeof(T), hipMemcpyDeviceToHost), "kinematics out"))
    goto done;
  {
    struct Part { double* dst; int off, n; } parts[] = {
        {xpos, 0, m.nbody * 3}, {xmat, hs::MAXBODY * 3, m.nbody * 9}, {gxpos, hs::MAXBODY * 12, m.ngeom * 3},
        {gzaxis, hs::MAXBODY * 12 + hs::MAXGEOM * 3, m.ngeom * 3}, {com, hs::MAXBODY * 12 + hs::MAXGEOM * 6, 3}};
    for (auto& p : parts)
      if (p.dst)
        for (int k = 0; k < p.n; k++) p.dst[k] = (double)out[p.off + k];
  }
  rc = 0;
done:
  if (dq) (void)hipFree(dq);
  if (dout) (void)hipFree(dout);
  return rc;
}
}  // namespace

extern "C" {

const char* hs_last_error(void) { return g_err.c_str(); }
const char* hs_version(void) { return "hsim 0.1.0 (gfx950)"; }

hs_model* hs_model_load(const char* xml_path, char* err, int errsz) {
  auto* m = new hs_model();
  std::string e;
  if (!xml_path || !hs::compile_mjcf_file(xml_path, m->host, e)) {
    if (!xml_path) e = "null path";
    g_err = e;
    if (err && errsz > 0) { std::strncpy(err, e.c_str(), errsz - 1); err[errsz - 1] = 0; }
    delete m;
    return nullptr;
  }
  return m;
}

void hs_model_free(hs_model* m) { delete m; }

int hs_model_field(const hs_model* m, const char* name, double* out, int n) {
  if (!m || !name) return fail("null argument");
  int r = hs::model_field(m->host, name, out, n);
  if (r < 0) return fail(std::string("unknown model field '") + name + "'");
  return r;
}

hs_batch* hs_batch_create(const hs_model* m, int n_envs, int device, uint64_t seed, int precision,
                          const hs_buffers* external) {
  if (!m || n_envs <= 0) { fail("hs_batch_create: null model or n_envs <= 0"); return nullptr; }
  if ((precision & ~HS_FULL_STATE) != HS_FP32 && (precision & ~HS_FULL_STATE) != HS_FP64) {
    fail("precision must be HS_FP32 or HS_FP64 (optionally | HS_FULL_STATE)");
    return nullptr;
  }
  if ((precision & HS_FULL_STATE) && external && (!external->cfrc_ext || !external->subtree_linvel)) {
    fail("HS_FULL_STATE needs external cfrc_ext and subtree_linvel buffers");
    return nullptr;
  }
  int ndev = 0;
  hipError_t de = hipGetDeviceCount(&ndev);
  if (de != hipSuccess || ndev == 0) {
    fail(std::string("no HIP device available (hipGetDeviceCount: ") + hipGetErrorString(de) + ", count " +
         std::to_string(ndev) + ")");
    return nullptr;
  }
  if (device < 0 || device >= ndev) { fail("device index out of range"); return nullptr; }
  DeviceGuard g(device);
  auto* b = new hs_batch();
  b->model = m;
  b->n = n_envs;
  b->device = device;
  b->seed = seed;
  b->full_state = (precision & HS_FULL_STATE) != 0;
  precision &= ~HS_FULL_STATE;
  b->precision = precision;
  b->obs_dim = obs_dim_of(m->host) + (b->full_state ? 6 * (m->host.nbody - 1) : 0);
  b->cfg.frame_skip = 5;
  b->cfg.max_steps = 750;
  b->cfg.reward_id = HS_REWARD_STAND;
  b->cfg.autoreset = 1;
  b->cfg.max_newton = m->host.iterations;     // <option iterations>
  b->cfg.outputs = HS_OUT_AUX | HS_OUT_CTRL;
  b->cfg.duration = 15.0;
  b->cfg.init_height = 1.282;
  b->cfg.noise_scale = 0.01;
  const double kneel[9] = {1.282, 0.85, 3.14159265358979323846 / 6, 0.1, 0.3, 0.3, 0.2, 0.1, 0.1};
  std::memcpy(b->cfg.kneel_params, kneel, sizeof kneel);
  std::string err;
  bool ok = precision == HS_FP64 ? upload_model<double>(b, err) : upload_model<float>(b, err);
  if (!ok) { g_err = err; delete b; return nullptr; }
  size_t es = precision == HS_FP64 ? 8 : 4, N = (size_t)n_envs;
  const auto& h = m->host;
  if (external) {
    b->buf = *external;
    b->owns = false;
  } else {
    b->owns = true;
    auto al = [&](void** p, size_t bytes) { return hip_ok(hipMalloc(p, bytes > 0 ? bytes : 4), "hipMalloc"); };
    ok = al(&b->buf.qpos, N * h.nq * es) && al(&b->buf.qvel, N * h.nv * es) &&
         al(&b->buf.qacc_warmstart, N * h.nv * es) && al(&b->buf.ctrl, N * h.nu * es) && al(&b->buf.time, N * es) &&
         al((void**)&b->buf.step_count, N * 4) && al((void**)&b->buf.episode, N * 4) &&
         al(&b->buf.total_reward, N * es) && al((void**)&b->buf.warning, N * HS_NWARN * 4) &&
         al(&b->buf.obs, N * b->obs_dim * es) && al(&b->buf.terminal_obs, N * b->obs_dim * es) &&
         al(&b->buf.reward, N * es) && al((void**)&b->buf.terminated, N) && al((void**)&b->buf.truncated, N) &&
         al(&b->buf.aux, N * hs::AUXDIM * es) && al(&b->buf.cfrc_ext, N * h.nbody * 6 * es) &&
         al(&b->buf.subtree_linvel, N * h.nbody * 3 * es) && al((void**)&b->buf.terminal_step_count, N * 4) &&
         al(&b->buf.terminal_total_reward, N * es);
    if (!ok) { hs_batch_destroy(b); return nullptr; }
  }
  if (!hip_ok(hipMalloc(&b->dbg, hs::DBGDIM * 8), "hipMalloc(dbg)") ||
      !hip_ok(hipMalloc((void**)&b->redo, (N + 2) * sizeof(int)), "hipMalloc(redo)") ||
      !hip_ok(hipMalloc((void**)&b->redo_total, sizeof(unsigned long long)), "hipMalloc(redo_total)") ||
      // chunk-queue hand-off rows, claim counters and pair flags: UNCACHED device memory from the UC
      // pool above, so a hand-off between waves on different CUs / XCDs needs no L2 write-back or
      // invalidate (hs_kernels.hip step_pair)
      !(uc_alloc(device, N * hs::MIDDIM * es, &b->mid) ? true
          : (g_err = "hipExtMallocWithFlags(mid, uncached) failed", false)) ||
      !(uc_alloc(device, hs::qsync_words((int)N) * sizeof(int), (void**)&b->qsync) ? true
          : (g_err = "hipExtMallocWithFlags(qsync, uncached) failed", false))) {
    hs_batch_destroy(b);
    return nullptr;
  }
  ok = precision == HS_FP64 ? init_state<double>(b) : init_state<float>(b);
  if (!ok) { hs_batch_destroy(b); return nullptr; }
  return b;
}

void hs_batch_destroy(hs_batch* b) {
  if (!b) return;
  DeviceGuard g(b->device);
  if (b->owns) {
    void* ptrs[] = {b->buf.qpos, b->buf.qvel, b->buf.qacc_warmstart, b->buf.ctrl, b->buf.time, b->buf.step_count,
                    b->buf.episode, b->buf.total_reward, b->buf.warning, b->buf.obs, b->buf.terminal_obs,
                    b->buf.reward, b->buf.terminated, b->buf.truncated, b->buf.aux, b->buf.cfrc_ext,
                    b->buf.subtree_linvel, b->buf.terminal_step_count, b->buf.terminal_total_reward};
    for (void* p : ptrs)
      if (p) (void)hipFree(p);
  }
  if (b->dmodel) (void)hipFree(b->dmodel);
  if (b->dbg) (void)hipFree(b->dbg);
  if (b->redo) (void)hipFree(b->redo);
  if (b->redo_total) (void)hipFree(b->redo_total);
  if (b->mid) uc_release(b->device, (size_t)b->n * hs::MIDDIM * (b->precision == HS_FP64 ? 8 : 4), b->mid);
  if (b->qsync) uc_release(b->device, hs::qsync_words(b->n) * sizeof(int), b->qsync);
  if (b->tape_backup) (void)hipFree(b->tape_backup);
  if (b->order_ev) (void)hipEventDestroy(b->order_ev);
  for (auto& e : b->tape_ev)
    if (e) (void)hipEventDestroy(e);
  delete b;
}

int hs_batch_get_info(const hs_batch* b, hs_batch_info* out) {
  if (!b || !out) return fail("null argument");
  const auto& h = b->model->host;
  out->n_envs = b->n;
  out->precision = b->precision;
  out->nq = h.nq; out->nv = h.nv; out->nu = h.nu; out->nbody = h.nbody;
  out->obs_dim = b->obs_dim;
  out->elem_size = b->precision == HS_FP64 ? 8 : 4;
  out->resident_con = b->precision == HS_FP64 ? hs::MAXCON_F64 : hs::MAXCON;
  out->resident_efc = b->precision == HS_FP64 ? hs::MAXEFC_F64 : hs::MAXEFC;
  out->wide_con = hs::MAXCON_WIDE;
  out->wide_efc = hs::MAXEFC_WIDE;
  const hs::ContactBound cb = hs::contact_bound(h);
  out->bound_con_all = cb.con_all;
  out->bound_efc_all = cb.efc_all;
  out->bound_con_floor = cb.con_floor;
  out->bound_efc_floor = cb.efc_floor;
  {
    DeviceGuard g(b->device);
    const bool pgs = b->model->host.solver == 1;
    out->resident_waves = b->precision == HS_FP64 ? hs::resident_waves<double>(pgs) : hs::resident_waves<float>(pgs);
  }
  return 0;
}

int hs_get_buffers(const hs_batch* b, hs_buffers* out) {
  if (!b || !out) return fail("null argument");
  *out = b->buf;
  return 0;
}

int hs_set_config(hs_batch* b, const hs_env_config* cfg) {
  if (!b || !cfg) return fail("null argument");
  if (cfg->frame_skip < 1) return fail("frame_skip must be >= 1");
  if (cfg->max_newton < 1) return fail("max_newton must be >= 1");
  if (cfg->reward_id < HS_REWARD_NONE || cfg->reward_id > HS_REWARD_WALK) return fail("unknown reward id");
  if (cfg->outputs & ~(HS_OUT_AUX | HS_OUT_CTRL)) return fail("unknown output bits");
  if (cfg->schedule != HS_SCHED_AUTO && cfg->schedule != HS_SCHED_DIRECT && cfg->schedule != HS_SCHED_SINGLE &&
      cfg->schedule != HS_SCHED_FIXED_ORDER)
    return fail("unknown schedule");
  b->cfg = *cfg;
  return 0;
}

int hs_set_seed(hs_batch* b, uint64_t seed) {
  if (!b) return fail("null batch");
  b->seed = seed;
  return 0;
}

int hs_get_config(const hs_batch* b, hs_env_config* cfg) {
  if (!b || !cfg) return fail("null argument");
  *cfg = b->cfg;
  return 0;
}

int hs_reset(hs_batch* b, const uint8_t* mask, const void* qpos_noise, const void* qvel_noise, void* stream) {
  int rc = launch(b, hs::MODE_RESET, nullptr, mask, qpos_noise, qvel_noise, 1, stream);
  if (rc == 0 && !mask) b->ctrl_stale = false;     // every env's data.ctrl is 0 again (mj_resetData)
  return rc;
}

int hs_step(hs_batch* b, const float* actions, void* stream) {
  if (!actions) return fail("hs_step: actions must not be NULL");
  if (!b) return fail("null batch");
  int rc = launch(b, hs::MODE_ENV_STEP, actions, nullptr, b->ar_qpos_noise, b->ar_qvel_noise, b->cfg.frame_skip, stream);
  // a step with the ctrl copy on rewrites every env's data.ctrl (commit), one with it off leaves it stale
  if (rc == 0) b->ctrl_stale = !(b->cfg.outputs & HS_OUT_CTRL);
  return rc;
}

int hs_step_tape(hs_batch* b, const float* actions, int n_steps, const hs_tape_out* out, void* stream) {
  if (!b) return fail("null batch");
  if (!actions) return fail("hs_step_tape: actions must not be NULL");
  if (n_steps < 1) return fail("hs_step_tape: n_steps must be >= 1");
  if (out && (!out->obs || !out->reward || !out->terminated || !out->truncated))
    return fail("hs_step_tape: pass all four per-step output arrays, or out = NULL");
  DeviceGuard g(b->device);
  if (order_streams(b, (hipStream_t)stream)) return -1;
  const auto& h = b->model->host;
  const size_t N = (size_t)b->n, es = b->precision == HS_FP64 ? 8 : 4, nu = (size_t)h.nu;
  hipStream_t st = (hipStream_t)stream;
  // n_steps hs_step calls, each step's outputs copied into its slice (the reference path, and the
  // replay of an aborted tape launch)
  auto per_step = [&]() -> int {
    for (int t = 0; t < n_steps; t++) {
      int rc = hs_step(b, actions + (size_t)t * N * nu, stream);
      if (rc) return rc;
      if (out) {
        const size_t d = (size_t)b->obs_dim;
        if (!hip_ok(hipMemcpyAsync((char*)out->obs + t * N * d * es, b->buf.obs, N * d * es, hipMemcpyDeviceToDevice, st),
                    "tape obs") ||
            !hip_ok(hipMemcpyAsync((char*)out->reward + t * N * es, b->buf.reward, N * es, hipMemcpyDeviceToDevice, st),
                    "tape reward") ||
            !hip_ok(hipMemcpyAsync(out->terminated + t * N, b->buf.terminated, N, hipMemcpyDeviceToDevice, st),
                    "tape terminated") ||
            !hip_ok(hipMemcpyAsync(out->truncated + t * N, b->buf.truncated, N, hipMemcpyDeviceToDevice, st),
                    "tape truncated"))
          return -1;
      }
    }
    return 0;
  };
  const int resident = b->precision == HS_FP64 ? hs::resident_waves<double>(h.solver == 1)
                                               : hs::resident_waves<float>(h.solver == 1);
  const bool tape_sched = b->cfg.schedule == HS_SCHED_AUTO || b->cfg.schedule == HS_SCHED_FIXED_ORDER;
  // without auto-reset a finished env keeps rewriting its terminal info every step (one launch
  // must write each batch address once, see hs_kernels.hip step_pair): step by step
  if (n_steps == 1 || !tape_sched || !b->cfg.autoreset || resident <= 0 || !b->mid || !b->qsync) return per_step();
  // one launch covers at most the shortest episode and at most QTAG_STEPS steps (its hand-off tags)
  const int min_len = std::min(min_episode_len(b), hs::QTAG_STEPS);
  if (n_steps > min_len) {
    for (int t0 = 0; t0 < n_steps; t0 += min_len) {
      const int k = std::min(min_len, n_steps - t0);
      hs_tape_out sub{};
      if (out) {
        sub.obs = (char*)out->obs + (size_t)t0 * N * b->obs_dim * es;
        sub.reward = (char*)out->reward + (size_t)t0 * N * es;
        sub.terminated = out->terminated + (size_t)t0 * N;
        sub.truncated = out->truncated + (size_t)t0 * N;
      }
      int rc = hs_step_tape(b, actions + (size_t)t0 * N * nu, k, out ? &sub : nullptr, stream);
      if (rc) return rc;
    }
    return 0;
  }
  // an env that overflows the resident tier stops the tape launch (QS_ABORT), and the tape is then
  // replayed step by step from the saved state (the wide tier re-runs the overflowing steps) -- the
  // same results, bitwise, as n_steps hs_step calls either way
  int rc = guarded_tape(b, state_regions(b), st, [&] {
    return launch(b, hs::MODE_ENV_STEP, actions, nullptr, b->ar_qpos_noise, b->ar_qvel_noise, b->cfg.frame_skip,
                  stream, n_steps, out);
  });
  if (rc < 0) return rc;
  if (rc == 1) return per_step();
  b->ctrl_stale = !(b->cfg.outputs & HS_OUT_CTRL);
  if (out) {   // the batch's own output buffers hold the last step, as after n_steps hs_step calls
    const size_t d = (size_t)b->obs_dim, t = (size_t)n_steps - 1;
    if (!hip_ok(hipMemcpyAsync(b->buf.obs, (char*)out->obs + t * N * d * es, N * d * es, hipMemcpyDeviceToDevice, st),
                "tape obs") ||
        !hip_ok(hipMemcpyAsync(b->buf.reward, (char*)out->reward + t * N * es, N * es, hipMemcpyDeviceToDevice, st),
                "tape reward") ||
        !hip_ok(hipMemcpyAsync(b->buf.terminated, out->terminated + t * N, N, hipMemcpyDeviceToDevice, st),
                "tape terminated") ||
        !hip_ok(hipMemcpyAsync(b->buf.truncated, out->truncated + t * N, N, hipMemcpyDeviceToDevice, st),
                "tape truncated"))
      return -1;
  }
  return 0;
}

int hs_rollout_max_steps(const hs_batch* b) {
  if (!b) return fail("null batch");
  return std::min(min_episode_len(b), hs::QTAG_STEPS);
}

int hs_rollout(hs_batch* b, const hs_policy* pol, const hs_rollout_bufs* rb, int t_begin, int n_steps, int t_total,
               void* stream) {
  if (!b || !pol || !rb) return fail("null argument");
  const auto& h = b->model->host;
  if (b->precision != HS_FP64 || h.solver == 1)
    return fail("hs_rollout: the fused rollout runs on the fp64 Newton engine");
  if (!b->cfg.autoreset || b->ar_qpos_noise || b->cfg.reward_id == HS_REWARD_NONE)
    return fail("hs_rollout: needs auto-reset with the on-device reset noise and a device reward");
  if (b->cfg.schedule != HS_SCHED_AUTO && b->cfg.schedule != HS_SCHED_FIXED_ORDER)
    return fail("hs_rollout: needs the chunk-queue schedule (HS_SCHED_AUTO or HS_SCHED_FIXED_ORDER)");
  if (pol->obs_dim != b->obs_dim || pol->act_dim != h.nu || pol->act_dim > 32 || pol->obs_dim % 4 ||
      pol->obs_dim > 512 || pol->ld1 < 256 || pol->ld1 % 4)
    return fail("hs_rollout: policy shape (obs_dim " + std::to_string(pol->obs_dim) + ", act_dim " +
                std::to_string(pol->act_dim) + ", ld1 " + std::to_string(pol->ld1) +
                ") does not fit the fused forward (obs_dim = the batch's, a multiple of 4 and <= 512; act_dim = nu "
                "<= 32; hidden layers of 256)");
  if (n_steps < 1 || t_begin < 0 || t_begin + n_steps > t_total || n_steps > min_episode_len(b) ||
      n_steps > hs::QTAG_STEPS)
    return fail("hs_rollout: steps [t_begin, t_begin + n_steps) must lie in [0, t_total) and n_steps in [1, " +
                std::to_string(std::min(min_episode_len(b), hs::QTAG_STEPS)) + "] (hs_rollout_max_steps)");
  for (const void* q : {(const void*)pol->w1, (const void*)pol->b1, (const void*)pol->w2, (const void*)pol->b2,
                        (const void*)pol->w3, (const void*)pol->b3, (const void*)pol->log_std, (const void*)rb->obs,
                        (const void*)rb->obs_last, (const void*)rb->actions, (const void*)rb->log_probs,
                        (const void*)rb->episode_starts, (const void*)rb->rewards, (const void*)rb->dones,
                        (const void*)rb->episode_returns, (const void*)rb->boot, (const void*)rb->terminal_obs,
                        (const void*)rb->ep_acc, (const void*)rb->episode_start, (const void*)rb->actions_clipped,
                        (const void*)rb->counter_base})
    if (!q) return fail("hs_rollout: every policy weight and rollout buffer must be given");
  DeviceGuard g(b->device);
  if (order_streams(b, (hipStream_t)stream)) return -1;
  const int resident = hs::resident_waves<double>(false);
  if (resident <= 0 || !b->mid || !b->qsync) return fail("hs_rollout: no resident-wave count / queue buffers");
  hs::RolloutArgs ro{};
  ro.w1 = pol->w1; ro.b1 = pol->b1; ro.w2 = pol->w2; ro.b2 = pol->b2; ro.w3 = pol->w3; ro.b3 = pol->b3;
  ro.log_std = pol->log_std;
  ro.ld1 = pol->ld1; ro.D = pol->obs_dim; ro.A = pol->act_dim;
  ro.t_begin = t_begin; ro.t_total = t_total;
  ro.obs = rb->obs; ro.obs_last = rb->obs_last; ro.act = rb->actions; ro.logp = rb->log_probs;
  ro.start = rb->episode_starts; ro.rew = rb->rewards; ro.done = rb->dones; ro.epret = rb->episode_returns;
  ro.boot = rb->boot; ro.tobs = rb->terminal_obs; ro.ep_acc = rb->ep_acc; ro.episode_start = rb->episode_start;
  ro.act_clip = rb->actions_clipped; ro.ctr_base = rb->counter_base;
  ro.k0 = (uint32_t)rb->seed; ro.k1 = (uint32_t)(rb->seed >> 32); ro.deterministic = rb->deterministic;
  const size_t N = (size_t)b->n;
  std::vector<Region> regs = state_regions(b);
  regs.push_back({rb->ep_acc, N * sizeof(double)});
  regs.push_back({rb->episode_start, N * sizeof(float)});
  regs.push_back({rb->actions_clipped, N * (size_t)pol->act_dim * sizeof(float)});
  hipStream_t st = (hipStream_t)stream;
  int rc = guarded_tape(b, regs, st, [&] {
    return launch(b, hs::MODE_ENV_STEP, rb->actions_clipped, nullptr, nullptr, nullptr, b->cfg.frame_skip, stream,
                  n_steps, nullptr, &ro);
  });
  if (rc == 0) b->ctrl_stale = !(b->cfg.outputs & HS_OUT_CTRL);
  return rc;
}

int hs_debug_lose_handoff(hs_batch* b, int env) {
  if (!b) return fail("null batch");
  if (env < -1 || env >= b->n) return fail("env index out of range");
  b->lose_env1 = env < 0 ? 0 : env + 1;
  return 0;
}

int hs_set_autoreset_noise(hs_batch* b, const void* qpos_noise, const void* qvel_noise) {
  if (!b) return fail("null batch");
  if ((qpos_noise == nullptr) != (qvel_noise == nullptr)) return fail("bind both noise arrays or neither");
  b->ar_qpos_noise = qpos_noise;
  b->ar_qvel_noise = qvel_noise;
  return 0;
}

int hs_physics_step(hs_batch* b, const float* ctrl, int nsub, void* stream) {
  if (nsub < 1) return fail("nsub must be >= 1");
  if (!b) return fail("null batch");
  if (!ctrl && b->ctrl_stale)
    return fail("hs_physics_step: ctrl == NULL keeps data.ctrl, but env steps ran with HS_OUT_CTRL off so the "
                "ctrl buffer is stale; pass ctrl, set it with hs_state_io, or enable HS_OUT_CTRL");
  int rc = launch(b, hs::MODE_PHYSICS, ctrl, nullptr, nullptr, nullptr, nsub, stream);
  if (rc == 0 && ctrl) b->ctrl_stale = false;
  return rc;
}

int hs_state_io(hs_batch* b, int dir, double* qpos, double* qvel, double* qacc_warmstart, double* time, double* ctrl) {
  if (!b) return fail("null batch");
  if (dir != 0 && dir != 1) return fail("dir must be 0 (get) or 1 (set)");
  if (dir == 0 && ctrl && b->ctrl_stale)
    return fail("hs_state_io: ctrl requested, but env steps ran with HS_OUT_CTRL off (the ctrl buffer is stale)");
  DeviceGuard g(b->device);
  if (!hip_ok(hipDeviceSynchronize(), "sync")) return -1;
  int rc = b->precision == HS_FP64 ? state_io<double>(b, dir, qpos, qvel, qacc_warmstart, time, ctrl)
                                   : state_io<float>(b, dir, qpos, qvel, qacc_warmstart, time, ctrl);
  if (rc == 0 && dir == 1 && ctrl) b->ctrl_stale = false;   // only once the new ctrl is on the device
  return rc;
}

int hs_kinematics(hs_batch* b, int env, const double* qpos, double* xpos, double* xmat, double* geom_xpos,
                  double* geom_zaxis, double* com) {
  if (!b) return fail("null batch");
  if (env < 0 || env >= b->n) return fail("env index out of range");
  DeviceGuard g(b->device);
  if (!hip_ok(hipDeviceSynchronize(), "sync")) return -1;
  return b->precision == HS_FP64 ? kinematics_io<double>(b, env, qpos, xpos, xmat, geom_xpos, geom_zaxis, com)
                                 : kinematics_io<float>(b, env, qpos, xpos, xmat, geom_xpos, geom_zaxis, com);
}

int hs_set_debug(hs_batch* b, int enable) {
  if (!b) return fail("null batch");
  b->debug = enable != 0;
  return 0;
}

int hs_get_debug(hs_batch* b, double* out, int n) {
  if (!b || !out) return fail("null argument");
  if (n < hs::DBGDIM) return fail("debug buffer too small");
  DeviceGuard g(b->device);
  if (!hip_ok(hipDeviceSynchronize(), "sync")) return -1;
  if (b->precision == HS_FP64) return hip_ok(hipMemcpy(out, b->dbg, hs::DBGDIM * 8, hipMemcpyDeviceToHost), "dbg") ? 0 : -1;
  std::vector<float> t(hs::DBGDIM);
  if (!hip_ok(hipMemcpy(t.data(), b->dbg, hs::DBGDIM * 4, hipMemcpyDeviceToHost), "dbg")) return -1;
  for (int k = 0; k < hs::DBGDIM; k++) out[k] = t[k];
  return 0;
}

int hs_ppo_act(const float* mean, int mean_ld, const float* value, int value_ld, const float* log_std,
               const float* episode_start, uint64_t seed, uint64_t counter, const uint64_t* counter_base,
               int deterministic, float* actions,
               float* actions_clipped, float* log_prob, float* values, float* episode_starts_out, int N, int A,
               void* stream) {
  if (N < 0 || A < 1 || A > 32) return fail("hs_ppo_act: need N >= 0 and 1 <= A <= 32");
  if (mean_ld < A || value_ld < 1) return fail("hs_ppo_act: bad leading dimension");
  if (N == 0) return 0;
  if (!mean || !value || !log_std || !episode_start || !actions || !actions_clipped || !log_prob || !values ||
      !episode_starts_out)
    return fail("hs_ppo_act: null buffer");
  return hip_ok(hs::launch_ppo_act(mean, mean_ld, value, value_ld, log_std, episode_start, seed, counter, counter_base,
                                   deterministic,
                                   actions, actions_clipped, log_prob, values, episode_starts_out, N, A,
                                   (hipStream_t)stream),
                "ppo_act_kernel")
             ? 0
             : -1;
}

int hs_ppo_post(const float* reward, const uint8_t* terminated, const uint8_t* truncated, const float* terminal_value,
                const float* terminal_obs, float* boot_obs_out, uint8_t* boot_out, int obs_dim, float gamma,
                const float* obs, float* obs_out, uint64_t obs_floats, float* reward_out, uint8_t* done_out,
                double* ep_acc, double* ep_return_out, float* episode_start, int N, void* stream) {
  if (N < 0) return fail("hs_ppo_post: negative size");
  if (N == 0) return 0;
  if (!reward || !terminated || !truncated || !reward_out || !done_out || !ep_acc || !ep_return_out || !episode_start)
    return fail("hs_ppo_post: null buffer");
  if (!terminal_value && (!terminal_obs || !boot_obs_out || !boot_out || obs_dim < 1))
    return fail("hs_ppo_post: need terminal_value, or terminal_obs + boot_obs_out + boot_out + obs_dim (deferred)");
  if (!obs) obs_floats = 0;
  if (obs_floats && !obs_out) return fail("hs_ppo_post: null obs_out");
  return hip_ok(hs::launch_ppo_post(reward, terminated, truncated, terminal_value, terminal_obs, boot_obs_out, boot_out,
                                    obs_dim, gamma, obs, obs_out, (size_t)obs_floats, reward_out, done_out, ep_acc,
                                    ep_return_out, episode_start, N, (hipStream_t)stream),
                "ppo_post_kernel")
             ? 0
             : -1;
}

int hs_gauss_logp(const float* mean, int mean_ld, const float* actions, const float* log_std, float* logp, int N,
                  int A, void* stream) {
  if (N < 0 || A < 1 || A > 32 || mean_ld < A) return fail("hs_gauss_logp: need N >= 0, 1 <= A <= 32, mean_ld >= A");
  if (N == 0) return 0;
  if (!mean || !actions || !log_std || !logp) return fail("hs_gauss_logp: null buffer");
  return hip_ok(hs::launch_gauss_logp(mean, mean_ld, actions, log_std, logp, N, A, (hipStream_t)stream),
                "gauss_logp_kernel")
             ? 0
             : -1;
}

int hs_gauss_logp_grad(const float* mean, int mean_ld, const float* actions, const float* log_std,
                       const float* g_logp, float* g_mean, float* gls_rows, int N, int A, void* stream) {
  if (N < 0 || A < 1 || mean_ld < A) return fail("hs_gauss_logp_grad: need N >= 0, A >= 1, mean_ld >= A");
  if (N == 0) return 0;
  if (!mean || !actions || !log_std || !g_logp || !g_mean || !gls_rows) return fail("hs_gauss_logp_grad: null buffer");
  return hip_ok(hs::launch_gauss_logp_grad(mean, mean_ld, actions, log_std, g_logp, g_mean, gls_rows, N, A,
                                           (hipStream_t)stream),
                "gauss_logp_grad_kernel")
             ? 0
             : -1;
}

uint64_t hs_ppo_loss_workspace(int B) { return B > 0 ? hs::ppo_loss_workspace(B) : 0; }

int hs_ppo_loss(const float* log_prob, const float* values, const int64_t* idx, const float* advantages,
                const float* returns, const float* old_log_prob, int B, float clip, int normalize_advantage,
                float* policy_loss, float* value_loss, float* workspace, void* stream) {
  if (B < 0) return fail("hs_ppo_loss: negative size");
  if (B == 0) return 0;
  if (!log_prob || !values || !idx || !advantages || !returns || !old_log_prob || !policy_loss || !value_loss ||
      !workspace)
    return fail("hs_ppo_loss: null buffer");
  return hip_ok(hs::launch_ppo_loss_fwd(log_prob, values, idx, advantages, returns, old_log_prob, B, clip,
                                        normalize_advantage, policy_loss, value_loss, workspace, (hipStream_t)stream),
                "ppo loss kernels")
             ? 0
             : -1;
}

int hs_ppo_loss_grad(const float* log_prob, const float* values, int B, float clip, const float* workspace,
                     const float* g_pg, const float* g_vf, float* g_log_prob, float* g_values, void* stream) {
  if (B < 0) return fail("hs_ppo_loss_grad: negative size");
  if (B == 0) return 0;
  if (!log_prob || !values || !workspace || !g_pg || !g_vf || !g_log_prob || !g_values)
    return fail("hs_ppo_loss_grad: null buffer");
  return hip_ok(hs::launch_ppo_loss_bwd(log_prob, values, B, clip, workspace, g_pg, g_vf, g_log_prob, g_values,
                                        (hipStream_t)stream),
                "ppo_loss_bwd_kernel")
             ? 0
             : -1;
}

uint64_t hs_adam_workspace(uint64_t total_numel) { return (uint64_t)hs::adam_partials((long long)total_numel); }

int hs_adam_clip(int nt, float* const* params, const float* const* grads, float* const* exp_avg,
                 float* const* exp_avg_sq, float* const* step, const int64_t* numel, float* workspace, float max_norm,
                 double lr, double beta1, double beta2, double eps, void* stream) {
  if (nt < 1 || nt > 1024) return fail("hs_adam_clip: need 1 <= nt <= 1024 tensors");
  if (!params || !grads || !exp_avg || !exp_avg_sq || !step || !numel || !workspace)
    return fail("hs_adam_clip: null argument");
  std::vector<long long> n(nt);
  for (int t = 0; t < nt; t++) {
    if (!params[t] || !grads[t] || !exp_avg[t] || !exp_avg_sq[t] || !step[t] || numel[t] < 0)
      return fail("hs_adam_clip: null tensor or negative size");
    n[t] = (long long)numel[t];
  }
  return hip_ok(hs::launch_adam_clip(nt, params, grads, exp_avg, exp_avg_sq, step, n.data(), workspace, max_norm, lr,
                                     beta1, beta2, eps, (hipStream_t)stream),
                "adam kernels")
             ? 0
             : -1;
}

int hs_mlp2_forward(const float* X, int ldx, int D, int N, const float* W1, int ld1, const float* b1, const float* W2,
                    int ld2, const float* b2, const float* W3, int ld3, const float* b3, int A, float* out, int ldo,
                    void* stream) {
  if (N < 0 || D < 1 || D > 512 || A < 1 || A > 32 || ld1 < D || ld2 < 256 || ld3 < 256 || ldx < D || ldo < A)
    return fail("hs_mlp2_forward: need N >= 0, 1 <= D <= 512, 1 <= A <= 32, ld1 >= D, ld2 >= 256, ld3 >= 256, "
                "ldx >= D, ldo >= A");
  if (N == 0) return 0;
  if (!X || !W1 || !b1 || !W2 || !b2 || !W3 || !b3 || !out) return fail("hs_mlp2_forward: null buffer");
  return hip_ok(hs::launch_mlp2_fwd(X, ldx, D, N, W1, ld1, b1, W2, ld2, b2, W3, ld3, b3, A, out, ldo,
                                    (hipStream_t)stream),
                "mlp2_fwd_kernel")
             ? 0
             : -1;
}

uint64_t hs_colsum_partial_rows(uint64_t rows, uint64_t cols) { return hs::colsum_partial_rows(rows, cols); }

int hs_relu_grad_colsum(const float* g, const float* y, uint64_t rows, uint64_t cols, float* gm, float* partial,
                        void* stream) {
  if (!rows || !cols) return 0;
  if (!g || !y || !gm || !partial) return fail("hs_relu_grad_colsum: null buffer");
  return hip_ok(hs::launch_relu_colsum(g, y, rows, cols, gm, partial, (hipStream_t)stream), "relu_colsum_kernel") ? 0
                                                                                                                 : -1;
}

uint64_t hs_dgrad_mask_partial_rows(int B, int K) { return hs::dgrad_mask_partial_rows(B, K); }
uint64_t hs_dgrad_mask_workspace(int K) { return hs::dgrad_mask_workspace(K); }

int hs_dgrad_mask(const float* G, int ldg, int K, const float* W, int ldw, const float* X, int ldx, int B, int N,
                  float* GX, float* partial, float* workspace, void* stream) {
  if (B < 0 || N != 256 || K < 1 || (K > 32 && (K % 16 != 0 || K > 512)) || ldg < K || ldw < N || ldx < N)
    return fail("hs_dgrad_mask: need B >= 0, N == 256, K <= 32 or K % 16 == 0 with K <= 512, ldg >= K, ldw >= N, "
                "ldx >= N");
  if (B == 0) return 0;
  if (!G || !W || !X || !GX || !partial) return fail("hs_dgrad_mask: null buffer");
  if (K > 32 && (((uintptr_t)G & 15) || (ldg & 3))) return fail("hs_dgrad_mask: K > 32 needs 16-byte aligned G rows");
  if (hs::dgrad_mask_workspace(K) && !workspace) return fail("hs_dgrad_mask: workspace required");
  return hip_ok(hs::launch_dgrad_mask(G, ldg, K, W, ldw, X, ldx, B, N, GX, partial, workspace, (hipStream_t)stream),
                "dgrad_mask kernel")
             ? 0
             : -1;
}

int hs_colsum_pair(const float* x0, uint64_t rows0, uint64_t cols0, float* out0, const float* x1, uint64_t rows1,
                   uint64_t cols1, float* out1, void* stream) {
  if ((cols0 && (!x0 || !out0)) || (cols1 && (!x1 || !out1))) return fail("hs_colsum_pair: null buffer");
  return hip_ok(hs::launch_colsum_pair(x0, rows0, cols0, out0, x1, rows1, cols1, out1, (hipStream_t)stream),
                "colsum_pair_kernel")
             ? 0
             : -1;
}

uint64_t hs_colsum_workspace(uint64_t rows, uint64_t cols) { return hs::colsum_workspace(rows, cols); }

int hs_colsum(const float* x, uint64_t rows, uint64_t cols, const float* row_weight, float* workspace, float* out,
              void* stream) {
  if (cols == 0) return 0;
  if (!out || (rows && !x)) return fail("hs_colsum: null buffer");
  if (hs::colsum_workspace(rows, cols) && !workspace) return fail("hs_colsum: workspace required");
  return hip_ok(hs::launch_colsum(x, rows, cols, row_weight, workspace, out, (hipStream_t)stream), "colsum_kernel")
             ? 0
             : -1;
}

int hs_gae(const float* rewards, const float* values, const float* episode_starts, const float* last_values,
           const float* last_dones, float* advantages, float* returns, int T, int N, float gamma, float gae_lambda,
           void* stream) {
  if (T < 0 || N < 0) return fail("hs_gae: negative size");
  if (T == 0 || N == 0) return 0;
  if (!rewards || !values || !episode_starts || !last_values || !last_dones || !advantages || !returns)
    return fail("hs_gae: null buffer");
  {  // the T >= 256 path keeps per-chunk maps / carries in the output rows: outputs must not overlap inputs
    const size_t tn = (size_t)T * (size_t)N * sizeof(float);
    auto overlap = [](const void* a, size_t na, const void* b, size_t nb) {
      const char *pa = (const char*)a, *pb = (const char*)b;
      return pa < pb + nb && pb < pa + na;
    };
    const void* outs[2] = {advantages, returns};
    const void* ins[3] = {rewards, values, episode_starts};
    if (overlap(advantages, tn, returns, tn)) return fail("hs_gae: advantages and returns overlap");
    for (const void* o : outs) {
      for (const void* in : ins)
        if (overlap(o, tn, in, tn)) return fail("hs_gae: an output ([T][N] advantages / returns) overlaps an input");
      if (overlap(o, tn, last_values, (size_t)N * sizeof(float)) || overlap(o, tn, last_dones, (size_t)N * sizeof(float)))
        return fail("hs_gae: an output overlaps last_values / last_dones");
    }
  }
  return hip_ok(hs::launch_gae(rewards, values, episode_starts, last_values, last_dones, advantages, returns, T, N,
                               gamma, gae_lambda, (hipStream_t)stream),
                "gae_kernel")
             ? 0
             : -1;
}

int hs_reward_eval(const hs_model* m, int precision, int reward_id, const double* kneel_params, int n,
                   const void* qpos, const void* qvel, const void* ctrl, const void* time, const void* subtree_com0,
                   const void* subtree_linvel0, const void* cfrc_ext, const void* qfrc_actuator, void* out,
                   void* stream) {
  if (!m) return fail("hs_reward_eval: null model");
  if (n < 0) return fail("hs_reward_eval: negative n");
  if (reward_id != HS_REWARD_STAND && reward_id != HS_REWARD_KNEELING && reward_id != HS_REWARD_WALK)
    return fail("hs_reward_eval: unknown reward id " + std::to_string(reward_id));
  const int prec = precision & 0xFF;
  if (prec != HS_FP32 && prec != HS_FP64) return fail("hs_reward_eval: precision must be HS_FP32 or HS_FP64");
  const hs::HostModel& h = m->host;
  if (h.nv < 6 || h.nv > 32 || h.nu > 32 || h.nbody < 2 || h.nq < 7)
    return fail("hs_reward_eval: the model needs a free root joint, nv <= 32, nu <= 32 and >= 2 bodies");
  if (n == 0) return 0;
  if (!qpos || !qvel || !ctrl || !time || !subtree_com0 || !subtree_linvel0 || !cfrc_ext || !qfrc_actuator || !out)
    return fail("hs_reward_eval: null buffer");
  static const double kdef[9] = {1.282, 0.85, 3.14159265358979323846 / 6, 0.1, 0.3, 0.3, 0.2, 0.1, 0.1};
  const double* kn = kneel_params ? kneel_params : kdef;
  auto run = [&](auto zero) -> int {
    using T = decltype(zero);
    hs::RewardEvalArgs<T> a{};
    a.reward_id = reward_id;
    a.n = n;
    a.nq = h.nq;
    a.nv = h.nv;
    a.nu = h.nu;
    a.nbody = h.nbody;
    for (int k = 0; k < 9; k++) a.kneel[k] = kn[k];
    a.qpos = (const T*)qpos;
    a.qvel = (const T*)qvel;
    a.ctrl = (const T*)ctrl;
    a.time = (const T*)time;
    a.subtree_com0 = (const T*)subtree_com0;
    a.subtree_linvel0 = (const T*)subtree_linvel0;
    a.cfrc_ext = (const T*)cfrc_ext;
    a.qfrc_actuator = (const T*)qfrc_actuator;
    a.out = (T*)out;
    return hip_ok(hs::launch_reward_eval<T>(a, (hipStream_t)stream), "reward_eval_kernel") ? 0 : -1;
  };
  return prec == HS_FP64 ? run(0.0) : run(0.0f);
}

int hs_reward(hs_batch* b, int reward_id, const double* kneel_params, void* out, void* stream) {
  if (!b || !out) return fail("hs_reward: null argument");
  if (reward_id != HS_REWARD_STAND && reward_id != HS_REWARD_KNEELING && reward_id != HS_REWARD_WALK)
    return fail("hs_reward: unknown reward id " + std::to_string(reward_id));
  if (!(b->cfg.outputs & HS_OUT_AUX) || !(b->cfg.outputs & HS_OUT_CTRL) || b->ctrl_stale)
    return fail("hs_reward: needs the aux row (subtree com) and the data.ctrl copy (HS_OUT_AUX | HS_OUT_CTRL) "
                "written by the last step");
  const hs::HostModel& h = b->model->host;
  DeviceGuard g(b->device);
  if (order_streams(b, (hipStream_t)stream)) return -1;
  const int o4 = (h.nq - 2) + h.nv + 16 * h.nbody;   // qfrc_actuator's offset in the obs row (custom_env.py:250)
  const double* kn = kneel_params ? kneel_params : b->cfg.kneel_params;
  auto run = [&](auto zero) -> int {
    using T = decltype(zero);
    hs::RewardEvalArgs<T> a{};
    a.reward_id = reward_id;
    a.n = b->n;
    a.nq = h.nq;
    a.nv = h.nv;
    a.nu = h.nu;
    a.nbody = h.nbody;
    for (int k = 0; k < 9; k++) a.kneel[k] = kn[k];
    a.qpos = (const T*)b->buf.qpos;
    a.qvel = (const T*)b->buf.qvel;
    a.ctrl = (const T*)b->buf.ctrl;
    a.time = (const T*)b->buf.time;
    a.subtree_com0 = (const T*)b->buf.aux + hs::MAXDOF;   // aux row: qacc[MAXDOF], com[3], ...
    a.ld_com = hs::AUXDIM;
    a.subtree_linvel0 = (const T*)b->buf.subtree_linvel;   // zeros unless HS_FULL_STATE (mj_step leaves it)
    a.ld_linv = 3 * h.nbody;
    a.cfrc_ext = (const T*)b->buf.cfrc_ext;
    a.qfrc_actuator = (const T*)b->buf.obs + o4;
    a.ld_qfrc = b->obs_dim;
    a.out = (T*)out;
    return hip_ok(hs::launch_reward_eval<T>(a, (hipStream_t)stream), "reward_eval_kernel") ? 0 : -1;
  };
  return b->precision == HS_FP64 ? run(0.0) : run(0.0f);
}

int hs_pack_outputs(hs_batch* b, double* out, int ncols, int warnings, void* stream) {
  if (!b || !out) return fail("hs_pack_outputs: null argument");
  if (ncols < 0 || ncols > 7) return fail("hs_pack_outputs: ncols must be in [0, 7]");
  DeviceGuard g(b->device);
  if (order_streams(b, (hipStream_t)stream)) return -1;
  auto run = [&](auto zero) -> int {
    using T = decltype(zero);
    hs::PackArgs<T> a{};
    a.n = b->n;
    a.obs_dim = b->obs_dim;
    a.ncols = ncols;
    a.nwarn = warnings ? HS_NWARN : 0;
    a.nwarn_stride = HS_NWARN;
    a.obs = (const T*)b->buf.obs;
    a.reward = (const T*)b->buf.reward;
    a.terminated = b->buf.terminated;
    a.truncated = b->buf.truncated;
    a.total_reward = (const T*)b->buf.total_reward;
    a.step_count = b->buf.step_count;
    a.term_step_count = b->buf.terminal_step_count;
    a.term_total_reward = (const T*)b->buf.terminal_total_reward;
    a.warning = b->buf.warning;
    a.out = out;
    return hip_ok(hs::launch_pack<T>(a, (hipStream_t)stream), "pack_kernel") ? 0 : -1;
  };
  return b->precision == HS_FP64 ? run(0.0) : run(0.0f);
}

int hs_batch_counters(const hs_batch* b, uint64_t* wide_reruns) {
  if (!b || !wide_reruns) return fail("null argument");
  DeviceGuard g(b->device);
  unsigned long long v = 0;
  if (!hip_ok(hipDeviceSynchronize(), "sync") ||
      !hip_ok(hipMemcpy(&v, b->redo_total, sizeof v, hipMemcpyDeviceToHost), "counters"))
    return -1;
  *wide_reruns = v;
  return 0;
}

int hs_last_tape_ms(const hs_batch* b, double* ms) {
  if (!b || !ms) return fail("null argument");
  *ms = (double)b->last_tape_ms;
  return 0;
}

int hs_tape_aborts(const hs_batch* b, uint64_t* n) {
  if (!b || !n) return fail("null argument");
  *n = b->tape_aborts;
  return 0;
}

int hs_stream_orders(const hs_batch* b, uint64_t* n) {
  if (!b || !n) return fail("null argument");
  *n = b->stream_orders;
  return 0;
}

int hs_synchronize(hs_batch* b) {
  if (!b) return fail("null batch");
  DeviceGuard g(b->device);
  return hip_ok(hipDeviceSynchronize(), "hipDeviceSynchronize") ? 0 : -1;
}

}  // extern "C"

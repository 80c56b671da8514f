"""A batch of humanoid envs resident in HBM, stepped by the HIP kernels through the C ABI.

``HsBatch`` allocates every per-env buffer as a torch tensor on the chosen GPU and binds them
to the native batch (``hs_batch_create(..., external=buffers)``), so observations / rewards /
dones are device tensors that a PyTorch policy consumes without leaving HBM.
"""
from __future__ import annotations

import ctypes as C
import math

import numpy as np

from . import _lib
from ._lib import check, lib

KNEEL_DEFAULTS = (1.282, 0.85, math.pi / 6, 0.1, 0.3, 0.3, 0.2, 0.1, 0.1)
KNEEL_KEYS = ("target_height", "min_height", "max_roll_pitch", "com_radius", "energy_weight", "posture_weight",
              "com_weight", "foot_weight", "alive_weight")


def _torch():
    import torch
    return torch


# MuJoCo's own warning texts for the three bad-state resets (mjWARN_BADQPOS / QVEL / QACC)
WARN_KINDS = ("Nan, Inf or huge value in QPOS", "Nan, Inf or huge value in QVEL", "Nan, Inf or huge value in QACC",
              "contacts dropped past the wide contact tier", "chunk-queue hand-off lost")


def report_warnings(new, where="step"):
    """Surface new warning counts (include/hsim.h HS_WARN_*, one value per kind) the way the reference
    run surfaces them: MuJoCo's mj_step prints mju_warning and resets a bad state (mj_resetData) and the
    run goes on (custom_env.py:160) -- here one RuntimeWarning per call with the counts; a lost
    chunk-queue hand-off is a scheduling failure of the step kernel, not physics, so it raises."""
    new = np.asarray(new, dtype=np.int64)
    if len(new) > 4 and new[4] > 0:
        raise _lib.HsimError(f"{WARN_KINDS[4]} in {int(new[4])} env step(s) of this {where}: a scheduling failure of "
                             "the step kernel (e.g. more concurrent queued batches than the GPU holds waves for), "
                             "not physics -- those envs were reset and the results are not valid")
    parts = [f"{WARN_KINDS[k]} in {int(new[k])} env step(s) of this {where}" for k in range(min(4, len(new)))
             if new[k] > 0]
    if parts:
        import warnings
        warnings.warn("mj_step warning: " + "; ".join(parts) + (" -- those envs were reset (mj_resetData)"
                      if new[:3].any() else ""), RuntimeWarning, stacklevel=3)


def reward_eval(model, name, qpos, qvel, ctrl, time, subtree_com0, subtree_linvel0, cfrc_ext, qfrc_actuator,
                params=None, registry=None):
    """``REWARD_FUNCTIONS[name](data, params)`` for n states at once, computed by the device reward
    code of the step kernel (``hs_reward_eval``; reward_functions.py:66-269).  Arguments are CUDA
    tensors of one float dtype (float64 = the fp64 engine's formulas, float32 = the fp32 engine's):
    qpos [n][nq], qvel [n][nv], ctrl [n][nu], time [n], subtree_com0 / subtree_linvel0 [n][3],
    cfrc_ext [n][nbody][6], qfrc_actuator [n][nv].  ``params`` are the kneeling reward's overrides
    (merged over its defaults like reward_functions.py:83).  Returns a [n] tensor.  Unknown names raise
    ValueError like custom_env.py:268-269; user callables have no device formula (HsimError)."""
    from .reward_functions import device_reward_id
    torch = _torch()
    rid = device_reward_id(name, registry)
    if rid is None:
        raise _lib.HsimError(f"reward {name!r} is a host callable: no device formula")
    args = [qpos, qvel, ctrl, time, subtree_com0, subtree_linvel0, cfrc_ext, qfrc_actuator]
    dt = qpos.dtype
    if dt not in (torch.float32, torch.float64):
        raise TypeError("reward_eval: float32 or float64 tensors")
    n = qpos.shape[0]
    shapes = [(n, model.nq), (n, model.nv), (n, model.nu), (n,), (n, 3), (n, 3), (n, model.nbody, 6),
              (n, model.nv)]
    for a, s in zip(args, shapes):
        if not a.is_cuda or a.dtype != dt or tuple(a.shape) != s or not a.is_contiguous():
            raise ValueError(f"reward_eval: expected a contiguous CUDA {dt} tensor of shape {s}, got "
                             f"{tuple(a.shape)} {a.dtype} on {a.device}")
    kn = None
    if rid == 1:
        p = {**dict(zip(KNEEL_KEYS, KNEEL_DEFAULTS)), **(params or {})}
        kn = (C.c_double * 9)(*[float(p[k]) for k in KNEEL_KEYS])
    out = torch.empty(n, dtype=dt, device=qpos.device)
    with torch.cuda.device(qpos.device):
        st = torch.cuda.current_stream().cuda_stream
        check(lib().hs_reward_eval(model.handle, 1 if dt == torch.float64 else 0, rid,
                                   C.cast(kn, C.c_void_p) if kn is not None else None, n,
                                   *[a.data_ptr() for a in args], out.data_ptr(), st))
    return out


class HsBatch:
    def __init__(self, model, n_envs, device=0, seed=0, precision="fp32", full_state=False, groups=1):
        """``groups`` > 1 splits the envs into that many native sub-batches (contiguous env ranges
        bound to slices of the same tensors), each launched on its own HIP stream: a group's
        Newton-iteration tail can overlap the other groups' next launches.  That needs the groups
        to run free (``step(..., join=False)`` then ``join()``): a per-step join (the default, what
        a policy that reads every env's obs needs) makes each step as long as its slowest group.
        Results per env are identical; reset-noise streams differ (per-group seeds)."""
        torch = _torch()
        if not torch.cuda.is_available():
            raise RuntimeError("HsBatch needs a ROCm GPU (torch.cuda.is_available() is False)")
        self.model = model
        self.n = int(n_envs)
        self.device = torch.device("cuda", int(device))
        self.precision = precision
        prec = _lib.HS_FP64 if precision == "fp64" else _lib.HS_FP32
        self.dtype = torch.float64 if prec == _lib.HS_FP64 else torch.float32
        nq, nv, nu, nb = model.nq, model.nv, model.nu, model.nbody
        self.full_state = bool(full_state)
        # custom_env.py:242-256 (352 for humanoid.xml); full_state adds cfrc_ext[1:] (their :247)
        self.obs_dim = (nq - 2) + nv + 10 * nb + 6 * nb + nv + (6 * (nb - 1) if self.full_state else 0)
        N, f, i32, u8 = self.n, self.dtype, torch.int32, torch.uint8
        z = lambda *s, dt=f: torch.zeros(*s, dtype=dt, device=self.device)  # noqa: E731
        self.t = dict(qpos=z(N, nq), qvel=z(N, nv), qacc_warmstart=z(N, nv), ctrl=z(N, nu), time=z(N),
                      step_count=z(N, dt=i32), episode=z(N, dt=i32), total_reward=z(N),
                      warning=z(N, _lib.HS_NWARN, dt=i32), obs=z(N, self.obs_dim), terminal_obs=z(N, self.obs_dim),
                      reward=z(N), terminated=z(N, dt=u8), truncated=z(N, dt=u8), aux=z(N, _lib.HS_AUXDIM),
                      cfrc_ext=z(N, nb, 6), subtree_linvel=z(N, nb, 3), terminal_step_count=z(N, dt=i32),
                      terminal_total_reward=z(N))
        torch.cuda.synchronize(self.device)
        flags = prec | (_lib.HS_FULL_STATE if self.full_state else 0)
        G = max(1, min(int(groups), self.n))
        bounds = [self.n * g // G for g in range(G + 1)]
        self._groups = []                       # (handle, lo, hi)
        for g in range(G):
            lo, hi = bounds[g], bounds[g + 1]
            bufs = _lib.hs_buffers(**{k: v.data_ptr() + lo * v.stride(0) * v.element_size() for k, v in self.t.items()})
            gseed = (int(seed) + 0x9E3779B97F4A7C15 * g) & (2 ** 64 - 1)
            h = lib().hs_batch_create(model.handle, hi - lo, self.device.index, gseed, flags, C.byref(bufs))
            if not h:
                self.close()
                raise _lib.HsimError(lib().hs_last_error().decode())
            self._groups.append((h, lo, hi))
        self._h = self._groups[0][0]
        # group 0 runs on the caller's current stream, groups 1.. on their own: G groups use exactly G
        # streams (a process has GPU_MAX_HW_QUEUES = 4 hardware queues; two streams sharing one serialise)
        self._streams = [None] + [torch.cuda.Stream(self.device) for _ in range(G - 1)] if G > 1 else None
        self._events = [torch.cuda.Event()] if G > 1 else None
        self._free = False
        self.cfg = _lib.hs_env_config()
        check(lib().hs_get_config(self._h, C.byref(self.cfg)))
        info = _lib.hs_batch_info()
        check(lib().hs_batch_get_info(self._h, C.byref(info)))
        # per-env (contacts, constraint rows) of the resident kernel tier and of the wide re-run tier
        self.resident_capacity = (info.resident_con, info.resident_efc)
        self.wide_capacity = (info.wide_con, info.wide_efc)
        self.resident_waves = info.resident_waves
        # static worst case (contacts, rows) of one env: every pair touching / every geom on the floor
        self.contact_bound_all = (info.bound_con_all, info.bound_efc_all)
        self.contact_bound_floor = (info.bound_con_floor, info.bound_efc_floor)

    def queued(self, nsub=None):
        """True when an env step of this batch runs on the chunk-queue schedule (HS_SCHED_AUTO, more
        env pairs than resident waves, >= 2 substeps; include/hsim.h)."""
        nsub = self.cfg.frame_skip if nsub is None else nsub
        n = max(hi - lo for _, lo, hi in self._groups)
        return (self.cfg.schedule in (_lib.HS_SCHED_AUTO, _lib.HS_SCHED_FIXED_ORDER) and nsub >= 2
                and 0 < self.resident_waves < (n + 1) // 2)

    def schedule_name(self, nsub=None):
        """The schedule an env step of this batch runs on (the largest group's; hs_kernels.hip
        launch_step): "queue" (chunk queue), "single" (one wave per env) or "paired"."""
        if self.queued(nsub):
            return "queue"
        n = max(hi - lo for _, lo, hi in self._groups)
        s = self.cfg.schedule
        if s == _lib.HS_SCHED_SINGLE or (s == _lib.HS_SCHED_AUTO and 0 < self.resident_waves and n <= self.resident_waves):
            return "single"
        return "paired"

    # -- tensors (device views, valid until the next call) ---------------------------------
    def __getattr__(self, name):
        t = self.__dict__.get("t")
        if t is not None and name in t:
            return t[name]
        raise AttributeError(name)

    @property
    def stream(self):
        return _torch().cuda.current_stream(self.device).cuda_stream

    # -- configuration ---------------------------------------------------------------------
    def configure(self, frame_skip=None, duration=None, reward_id=None, max_steps=None, autoreset=None,
                  max_newton=None, init_height=None, noise_scale=None, kneel_params=None, aux=None, ctrl=None,
                  schedule=None):
        """``schedule``: "auto" (default: one wave per env when every env fits the resident waves, a
        chunk queue when the env pairs outnumber them, else one wave per env pair; include/hsim.h
        HS_SCHED_AUTO), "direct" (one wave per env pair), "single" (one wave per env) or
        "fixed_order" (auto with the chunk queue's claims in a fixed permutation instead of cost
        order); results are bitwise identical.
        ``aux`` / ``ctrl``: write the optional aux row (qacc, subtree com, contact / row counts,
        solver iterations) and the data.ctrl copy at every commit (both on by default; data views,
        host rewards and statistics read them, the on-device trainer does not)."""
        c = self.cfg
        if aux is not None:
            c.outputs = (c.outputs & ~_lib.HS_OUT_AUX) | (_lib.HS_OUT_AUX if aux else 0)
        if ctrl is not None:
            c.outputs = (c.outputs & ~_lib.HS_OUT_CTRL) | (_lib.HS_OUT_CTRL if ctrl else 0)
        if schedule is not None:
            c.schedule = {"auto": _lib.HS_SCHED_AUTO, "direct": _lib.HS_SCHED_DIRECT,
                          "single": _lib.HS_SCHED_SINGLE, "fixed_order": _lib.HS_SCHED_FIXED_ORDER}[schedule]
        if frame_skip is not None:
            c.frame_skip = int(frame_skip)
        if duration is not None:
            c.duration = float(duration)
        if reward_id is not None:
            c.reward_id = int(reward_id)
        if max_steps is not None:
            c.max_steps = int(max_steps)
        if autoreset is not None:
            c.autoreset = int(bool(autoreset))
        if max_newton is not None:
            c.max_newton = int(max_newton)
        if init_height is not None:
            c.init_height = float(init_height)
        if noise_scale is not None:
            c.noise_scale = float(noise_scale)
        if kneel_params is not None:
            p = {**dict(zip(KNEEL_KEYS, KNEEL_DEFAULTS)), **kneel_params}
            for k, key in enumerate(KNEEL_KEYS):
                c.kneel_params[k] = float(p[key])
        for h, _, _ in self._groups:
            check(lib().hs_set_config(h, C.byref(c)))

    def set_seed(self, seed):
        for g, (h, _, _) in enumerate(self._groups):
            check(lib().hs_set_seed(h, (int(seed) + 0x9E3779B97F4A7C15 * g) & (2 ** 64 - 1)))

    def _launch(self, fn, *tensors, join=True):
        """fn(handle, lo, hi, stream) per group; multi-group launches fan out to the group streams
        and (join=True) join back into the caller's current stream.  A free-running session
        (join=False) waits on the caller's stream once, at its first launch (inputs produced before
        it); later free launches add no cross-stream waits (5 streams share the 4 hardware queues
        of a process, GPU_MAX_HW_QUEUES=4, and per-step waits would serialise them again)."""
        if self._streams is None:
            h, lo, hi = self._groups[0]
            fn(h, lo, hi, self.stream)
            return
        torch = _torch()
        cur = torch.cuda.current_stream(self.device)
        if join or not self._free:
            self._events[0].record(cur)
            for st in self._streams[1:]:
                st.wait_event(self._events[0])
        self._free = not join
        for (h, lo, hi), st in zip(self._groups, self._streams):
            if st is not None:
                for t in tensors:
                    if t is not None:
                        t.record_stream(st)
            fn(h, lo, hi, (cur if st is None else st).cuda_stream)
        if join:
            self.join()

    def join(self):
        """Make the caller's current stream wait for every group's last launch."""
        if self._streams is None:
            return
        cur = _torch().cuda.current_stream(self.device)
        for st in self._streams[1:]:
            cur.wait_stream(st)
        self._free = False

    # -- stepping --------------------------------------------------------------------------
    def reset(self, mask=None, qpos_noise=None, qvel_noise=None):
        """custom_env.py:97-150 for the envs selected by ``mask`` (None = all)."""
        torch = _torch()
        keep = []
        def dev(x, dt):
            if x is None:
                return None
            x = torch.as_tensor(x, device=self.device).to(dt).contiguous()
            keep.append(x)
            return x
        mk, qn, vn = dev(mask, torch.uint8), dev(qpos_noise, self.dtype), dev(qvel_noise, self.dtype)

        def off(x, lo):
            return None if x is None else x.data_ptr() + lo * x.stride(0) * x.element_size()
        self._launch(lambda h, lo, hi, st: check(lib().hs_reset(h, off(mk, lo), off(qn, lo), off(vn, lo), st)),
                     mk, qn, vn)
        return self.t["obs"]

    def set_autoreset_noise(self, qpos_noise=None, qvel_noise=None):
        """Bind [N, nq] / [N, nv] device tensors (batch dtype) holding each env's NEXT reset noise
        for the auto-reset inside ``step`` (None: the on-device counter RNG).  The tensors are
        kept referenced; refresh the rows of envs that reset (hs_set_autoreset_noise)."""
        torch = _torch()
        if qpos_noise is None:
            self._ar_noise = None
            for h, _, _ in self._groups:
                check(lib().hs_set_autoreset_noise(h, None, None))
            return
        qn = torch.as_tensor(qpos_noise, device=self.device).to(self.dtype).contiguous()
        vn = torch.as_tensor(qvel_noise, device=self.device).to(self.dtype).contiguous()
        assert qn.shape == (self.n, self.model.nq) and vn.shape == (self.n, self.model.nv)
        self._ar_noise = (qn, vn)
        for h, lo, hi in self._groups:
            check(lib().hs_set_autoreset_noise(h, qn.data_ptr() + lo * qn.stride(0) * qn.element_size(),
                                               vn.data_ptr() + lo * vn.stride(0) * vn.element_size()))
        return qn, vn

    def step(self, actions, join=True):
        """custom_env.py:152-230 batched; ``actions`` [N, nu] float32 on device.  With stream
        groups and join=False the groups run free; call ``join()`` before reading outputs."""
        torch = _torch()
        a = torch.as_tensor(actions, device=self.device).to(torch.float32).contiguous()
        assert a.shape == (self.n, self.model.nu), a.shape
        row = a.stride(0) * a.element_size()
        self._launch(lambda h, lo, hi, st: check(lib().hs_step(h, a.data_ptr() + lo * row, st)), a, join=join)
        return self.t["obs"], self.t["reward"], self.t["terminated"], self.t["truncated"]

    def step_tape(self, actions, outputs=True):
        """K consecutive ``step`` calls over an action tape [K, N, nu] (float32, on device) in one
        launch (hs_step_tape: a pair's step t + 1 starts once its own step t is committed, so the
        launch does not end every step on its slowest pair).  Bitwise the results of K ``step``
        calls.  outputs=True returns the per-step (obs [K, N, obs_dim], reward [K, N], terminated,
        truncated [K, N] uint8); the batch's own buffers hold the last step either way.  Open loop:
        benchmarks, trajectory evaluation -- a policy in the loop steps with ``step`` (or, for the PPO pi
        net, inside the launch: hs_rollout, PPO._rollout_fused).  Synchronous;
        one stream group only."""
        torch = _torch()
        if len(self._groups) != 1:
            raise NotImplementedError("step_tape: one stream group only")
        a = torch.as_tensor(actions, device=self.device).to(torch.float32).contiguous()
        if a.dim() != 3 or a.shape[1:] != (self.n, self.model.nu):
            raise ValueError(f"step_tape: actions must be [K, {self.n}, {self.model.nu}], got {tuple(a.shape)}")
        K = a.shape[0]
        res, out = None, None
        if outputs:
            res = (torch.empty(K, self.n, self.obs_dim, dtype=self.dtype, device=self.device),
                   torch.empty(K, self.n, dtype=self.dtype, device=self.device),
                   torch.empty(K, self.n, dtype=torch.uint8, device=self.device),
                   torch.empty(K, self.n, dtype=torch.uint8, device=self.device))
            out = _lib.hs_tape_out(*[x.data_ptr() for x in res])
        h = self._groups[0][0]
        check(lib().hs_step_tape(h, a.data_ptr(), K, C.byref(out) if out is not None else None, self.stream))
        if outputs:
            return res
        return self.t["obs"], self.t["reward"], self.t["terminated"], self.t["truncated"]

    # -- host copies of a step's outputs (the Gym / SB3 numpy surfaces) ----------------------
    _HOST_COLS = ("reward", "terminated", "truncated", "total_reward", "step_count", "terminal_step_count",
                  "terminal_total_reward")

    def host_outputs(self, ncols=3, warnings=False):
        """One step's outputs on the host in ONE device-to-host copy: the obs and the first ``ncols``
        of (reward, terminated, truncated, total_reward, step_count, terminal_step_count,
        terminal_total_reward), packed on the device into one float64 buffer, copied into pinned
        host memory and synchronized once.  Returns (obs [N, obs_dim] float64, cols [ncols, N]
        float64), views of a fresh pinned block (torch's caching host allocator recycles it once
        both are dropped).  ``warnings=True`` also packs the warning counters summed over the envs
        (HS_NWARN values, cumulative since the batch was created) and returns them third, as int64.
        One native pack launch (hs_pack_outputs) for a single-group batch."""
        torch = _torch()
        N, D = self.n, self.obs_dim
        nwr = N * _lib.HS_NWARN if warnings else 0          # per-env warning rows (summed on the host)
        size = N * D + ncols * N + nwr
        dev = self.__dict__.get("_pack_dev")
        if dev is None or dev.numel() != size:
            dev = self._pack_dev = torch.empty(size, dtype=torch.float64, device=self.device)
        st = torch.cuda.current_stream(self.device)
        if len(self._groups) == 1:   # one pack launch (hs_pack_outputs)
            check(lib().hs_pack_outputs(self._h, dev.data_ptr(), int(ncols), 1 if warnings else 0, st.cuda_stream))
        else:
            dev[:N * D].view(N, D).copy_(self.t["obs"])
            cols = dev[N * D:N * D + ncols * N].view(ncols, N)
            for k in range(ncols):
                cols[k].copy_(self.t[self._HOST_COLS[k]])
            if nwr:
                dev[N * D + ncols * N:].view(_lib.HS_NWARN, N).copy_(self.t["warning"].t())
        host = torch.empty(size, dtype=torch.float64, pin_memory=True)
        host.copy_(dev, non_blocking=True)
        st.synchronize()
        a = host.numpy()
        obs, c = a[:N * D].reshape(N, D), a[N * D:N * D + ncols * N].reshape(ncols, N)
        if not nwr:
            return obs, c
        return obs, c, a[N * D + ncols * N:].reshape(_lib.HS_NWARN, N).sum(1).astype(np.int64)

    def tape_aborts(self):
        """Tape launches replayed step by step because an env overflowed the resident tier."""
        v = C.c_uint64(0)
        check(lib().hs_tape_aborts(self._groups[0][0], C.byref(v)))
        return int(v.value)

    def compute_reward(self, name, params=None, registry=None):
        """``REWARD_FUNCTIONS[name](data_i, params)`` for every env's current state on the device
        (``hs_reward``: the step kernel's reward code on the batch's own buffers; custom_env.py:263-271
        ``_compute_reward``; ``self.reward`` stays the last step's reward buffer).
        Needs the aux row and the data.ctrl copy (``configure(aux=True, ctrl=True)``, the default).
        Returns an [N] tensor of the batch precision."""
        from .reward_functions import device_reward_id
        torch = _torch()
        rid = device_reward_id(name, registry)
        if rid is None:
            raise _lib.HsimError(f"reward {name!r} is a host callable: no device formula")
        kn = None
        if params is not None:
            p = {**dict(zip(KNEEL_KEYS, KNEEL_DEFAULTS)), **params}
            kn = (C.c_double * 9)(*[float(p[k]) for k in KNEEL_KEYS])
        out = torch.empty(self.n, dtype=self.dtype, device=self.device)

        def go(h, lo, hi, st):
            check(lib().hs_reward(h, rid, C.cast(kn, C.c_void_p) if kn is not None else None,
                                  out.data_ptr() + lo * out.element_size(), st))
        self._launch(go, out)
        return out

    def last_tape_ms(self):
        """Duration (ms, HIP events on its stream) of the last tape / fused-rollout kernel launch."""
        v = C.c_double(0)
        check(lib().hs_last_tape_ms(self._groups[0][0], C.byref(v)))
        return float(v.value)

    def stream_orders(self):
        """Cross-stream waits the library inserted because calls of this batch came on different
        streams (include/hsim.h: one batch's launches are always ordered)."""
        tot = 0
        for h, _, _ in self._groups:
            v = C.c_uint64(0)
            check(lib().hs_stream_orders(h, C.byref(v)))
            tot += int(v.value)
        return tot

    def physics_step(self, ctrl=None, nsub=1):
        """nsub raw mj_step's with the given ctrl [N, nu] (None keeps the current ctrl)."""
        torch = _torch()
        c = None
        if ctrl is not None:
            c = torch.as_tensor(ctrl, device=self.device).to(torch.float32).contiguous()
            assert c.shape == (self.n, self.model.nu), c.shape
            self._keep = c

        def go(h, lo, hi, st):
            p = None if c is None else c.data_ptr() + lo * c.stride(0) * c.element_size()
            check(lib().hs_physics_step(h, p, int(nsub), st))
        self._launch(go, c)

    # -- host state access (through the C ABI, synchronous, fp64) ---------------------------
    def get_state(self):
        """qpos / qvel / qacc_warmstart / time (and ctrl, while the data.ctrl copy is written:
        ``configure(ctrl=True)``, the default) as fp64 host arrays."""
        N, m = self.n, self.model
        out = dict(qpos=np.zeros((N, m.nq)), qvel=np.zeros((N, m.nv)), qacc_warmstart=np.zeros((N, m.nv)),
                   time=np.zeros(N), ctrl=np.zeros((N, m.nu)))
        keys = ("qpos", "qvel", "qacc_warmstart", "time", "ctrl")
        if not self.cfg.outputs & _lib.HS_OUT_CTRL:
            del out["ctrl"]
        for h, lo, hi in self._groups:
            check(lib().hs_state_io(h, 0, *[out[k][lo:hi].ctypes.data if k in out else None for k in keys]))
        return out

    def set_state(self, qpos=None, qvel=None, qacc_warmstart=None, time=None, ctrl=None):
        def p(x, shape):
            if x is None:
                return None, None
            a = np.ascontiguousarray(np.broadcast_to(np.asarray(x, np.float64), shape))
            return a, a.ctypes.data
        N, m = self.n, self.model
        keep = [p(qpos, (N, m.nq)), p(qvel, (N, m.nv)), p(qacc_warmstart, (N, m.nv)), p(time, (N,)), p(ctrl, (N, m.nu))]
        for h, lo, hi in self._groups:
            check(lib().hs_state_io(h, 1, *[None if a is None else a[lo:hi].ctypes.data for a, _ in keep]))

    def kinematics(self, env=0, qpos=None):
        """mj_kinematics + mj_comPos of one env on the GPU (hs_kinematics): body xpos / xmat,
        geom_xpos / geom_zaxis and the root subtree COM, fp64 on the host.  ``qpos`` poses that
        configuration instead of the env's current one.  Visualisation only (one sync launch)."""
        env = int(env)
        for h, lo, hi in self._groups:
            if lo <= env < hi:
                break
        else:
            raise IndexError(f"env {env} out of range [0, {self.n})")
        m = self.model
        out = {"xpos": np.zeros((m.nbody, 3)), "xmat": np.zeros((m.nbody, 9)), "geom_xpos": np.zeros((m.ngeom, 3)),
               "geom_zaxis": np.zeros((m.ngeom, 3)), "com": np.zeros(3)}
        q = None if qpos is None else np.ascontiguousarray(qpos, np.float64)
        if q is not None and q.shape != (m.nq,):
            raise ValueError(f"qpos must have shape ({m.nq},)")
        check(lib().hs_kinematics(h, env - lo, None if q is None else q.ctypes.data,
                                  *[out[k].ctypes.data for k in ("xpos", "xmat", "geom_xpos", "geom_zaxis", "com")]))
        return out

    def set_debug(self, on=True):
        check(lib().hs_set_debug(self._h, int(bool(on))))

    def debug_lose_handoff(self, env):
        """Test hook (hs_debug_lose_handoff): the chunk-queue hand-off of ``env``'s pair is treated
        as lost in the following queued launches (the pair is reset as mj_checkPos resets a bad state
        and counted in the HS_WARN_HANDOFF column of ``warning``);
        ``env=None`` turns it off."""
        for h, lo, hi in self._groups:
            inside = env is not None and lo <= int(env) < hi
            check(lib().hs_debug_lose_handoff(h, int(env) - lo if inside else -1))

    def get_debug(self):
        out = np.zeros(_lib.DBGDIM)
        check(lib().hs_get_debug(self._h, out.ctypes.data, _lib.DBGDIM))
        return out

    def wide_reruns(self):
        """Env steps re-run by the wide contact tier so far (resident tier overflowed; see
        hs_model.h).  Synchronous."""
        tot = 0
        for h, _, _ in self._groups:
            v = C.c_uint64(0)
            check(lib().hs_batch_counters(h, C.byref(v)))
            tot += int(v.value)
        return tot

    def synchronize(self):
        for h, _, _ in self._groups:
            check(lib().hs_synchronize(h))

    def close(self):
        for h, _, _ in self.__dict__.get("_groups", []):
            if h:
                lib().hs_batch_destroy(h)
        self._groups = []
        self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

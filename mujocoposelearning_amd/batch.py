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


class HsBatch:
    def __init__(self, model, n_envs, device=0, seed=0, precision="fp32", full_state=False):
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
                      cfrc_ext=z(N, nb, 6), subtree_linvel=z(N, nb, 3))
        bufs = _lib.hs_buffers(**{k: v.data_ptr() for k, v in self.t.items()})
        torch.cuda.synchronize(self.device)
        flags = prec | (_lib.HS_FULL_STATE if self.full_state else 0)
        h = lib().hs_batch_create(model.handle, self.n, self.device.index, int(seed) & (2 ** 64 - 1), flags,
                                  C.byref(bufs))
        if not h:
            raise _lib.HsimError(lib().hs_last_error().decode())
        self._h = h
        self.cfg = _lib.hs_env_config()
        check(lib().hs_get_config(h, C.byref(self.cfg)))

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
                  max_newton=None, init_height=None, noise_scale=None, kneel_params=None):
        c = self.cfg
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
        check(lib().hs_set_config(self._h, C.byref(c)))

    def set_seed(self, seed):
        check(lib().hs_set_seed(self._h, int(seed) & (2 ** 64 - 1)))

    # -- stepping --------------------------------------------------------------------------
    def reset(self, mask=None, qpos_noise=None, qvel_noise=None):
        """custom_env.py:97-150 for the envs selected by ``mask`` (None = all)."""
        torch = _torch()
        keep = []
        def ptr(x, dt):
            if x is None:
                return None
            x = torch.as_tensor(x, device=self.device).to(dt).contiguous()
            keep.append(x)
            return x.data_ptr()
        check(lib().hs_reset(self._h, ptr(mask, torch.uint8), ptr(qpos_noise, self.dtype), ptr(qvel_noise, self.dtype),
                             self.stream))
        return self.t["obs"]

    def step(self, actions):
        """custom_env.py:152-230 batched; ``actions`` [N, nu] float32 on device."""
        torch = _torch()
        a = torch.as_tensor(actions, device=self.device).to(torch.float32).contiguous()
        assert a.shape == (self.n, self.model.nu), a.shape
        check(lib().hs_step(self._h, a.data_ptr(), self.stream))
        return self.t["obs"], self.t["reward"], self.t["terminated"], self.t["truncated"]

    def physics_step(self, ctrl=None, nsub=1):
        """nsub raw mj_step's with the given ctrl [N, nu] (None keeps the current ctrl)."""
        torch = _torch()
        p = None
        if ctrl is not None:
            c = torch.as_tensor(ctrl, device=self.device).to(torch.float32).contiguous()
            assert c.shape == (self.n, self.model.nu), c.shape
            p = c.data_ptr()
            self._keep = c
        check(lib().hs_physics_step(self._h, p, int(nsub), self.stream))

    # -- host state access (through the C ABI, synchronous, fp64) ---------------------------
    def get_state(self):
        N, m = self.n, self.model
        out = dict(qpos=np.zeros((N, m.nq)), qvel=np.zeros((N, m.nv)), qacc_warmstart=np.zeros((N, m.nv)),
                   time=np.zeros(N), ctrl=np.zeros((N, m.nu)))
        check(lib().hs_state_io(self._h, 0, out["qpos"].ctypes.data, out["qvel"].ctypes.data,
                                out["qacc_warmstart"].ctypes.data, out["time"].ctypes.data, out["ctrl"].ctypes.data))
        return out

    def set_state(self, qpos=None, qvel=None, qacc_warmstart=None, time=None, ctrl=None):
        def p(x, shape):
            if x is None:
                return None, None
            a = np.ascontiguousarray(np.broadcast_to(np.asarray(x, np.float64), shape))
            return a, a.ctypes.data
        N, m = self.n, self.model
        keep = [p(qpos, (N, m.nq)), p(qvel, (N, m.nv)), p(qacc_warmstart, (N, m.nv)), p(time, (N,)), p(ctrl, (N, m.nu))]
        check(lib().hs_state_io(self._h, 1, *[k[1] for k in keep]))

    def set_debug(self, on=True):
        check(lib().hs_set_debug(self._h, int(bool(on))))

    def get_debug(self):
        out = np.zeros(_lib.DBGDIM)
        check(lib().hs_get_debug(self._h, out.ctypes.data, _lib.DBGDIM))
        return out

    def synchronize(self):
        check(lib().hs_synchronize(self._h))

    def close(self):
        h = self.__dict__.get("_h")
        if h:
            lib().hs_batch_destroy(h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

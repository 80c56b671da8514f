"""HumanoidVecEnv -- replaces SB3 ``SubprocVecEnv([make_env(env_config, i) ...])`` (train_sb3.py:203).

All envs of a rank live in one HsBatch in HBM; one ``hs_step`` launch steps all of them.
Two surfaces:

* SB3 VecEnv API (``reset``, ``step_async``/``step_wait``, ``get_attr``, ``set_attr``,
  ``env_method``, ``seed``, ``env_is_wrapped``, ``close``) returning numpy arrays with SB3's
  auto-reset semantics: on ``done`` the returned obs is the post-reset obs and
  ``infos[i]["terminal_observation"]`` holds the last obs; ``infos[i]["TimeLimit.truncated"]``
  = truncated and not terminated.  It subclasses SB3's ``VecEnv`` when SB3 is installed, so
  ``PPO("MlpPolicy", HumanoidVecEnv(...))`` works unchanged.
* Device fast path ``step_tensors(actions)`` / ``reset_tensors()`` returning torch tensors
  that never leave HBM (used by the on-device PPO trainer and bench.py).

Reset noise: unseeded, it comes from an on-device counter RNG (seed, env, episode).  After
``seed(s)`` (what SB3's ``PPO(seed=s)`` calls) every env i draws its resets -- the explicit
``reset()`` and every auto-reset -- from its own legacy MT19937 stream ``np.random.seed(s + i)``,
exactly as SubprocVecEnv worker i does (custom_env.py:99-110; SB3 VecEnv.seed gives worker i
seed + i and the worker's global numpy stream continues across auto-resets).
"""
from __future__ import annotations

import copy
from collections.abc import Sequence

import numpy as np

from . import _lib
from . import reward_functions as _rf
from ._lib import HsimError
from .batch import HsBatch, report_warnings
from .model import HsModel
from .spaces import Box

try:  # pragma: no cover - only where SB3 is installed
    from stable_baselines3.common.vec_env.base_vec_env import VecEnv as _Base
    HAVE_SB3 = True
except ImportError:
    HAVE_SB3 = False

    class _Base:
        def __init__(self, num_envs, observation_space, action_space):
            self.num_envs = num_envs
            self.observation_space = observation_space
            self.action_space = action_space

        def step(self, actions):
            self.step_async(actions)
            return self.step_wait()


class HumanoidVecEnv(_Base):
    def __init__(self, env_config, n_envs=None, device=0, precision="fp32", seed=0, model=None, max_newton=None,
                 groups="auto"):
        """``env_config``: the env_config dict (train_sb3.py:183-200), a model path, or SB3's
        ``[make_env(env_config, i) for i in range(n)]`` list of factories (train_sb3.py:203): all
        envs of one rank share one config, recovered from the first factory, and ``n_envs``
        defaults to the list length."""
        if isinstance(env_config, (list, tuple)):
            if not env_config or not all(callable(f) for f in env_config):
                raise TypeError("env_fns must be a non-empty list of env factories")
            if n_envs is not None and n_envs != len(env_config):
                raise ValueError(f"n_envs={n_envs} but {len(env_config)} env factories")
            n_envs = len(env_config)
            env_config = _config_of_factory(env_config[0])
        elif callable(env_config):
            env_config = _config_of_factory(env_config)
        if n_envs is None:
            n_envs = 8                      # train_sb3.py's env_kwargs.get('n_envs', 8)
        cfg = env_config if isinstance(env_config, dict) else {"model_path": env_config}
        self.env_config = dict(cfg)
        self.model = model if model is not None else HsModel(cfg["model_path"])
        if groups == "auto":      # one launch per step (stream groups only pay off when run free, see HsBatch)
            groups = 1
        self.batch = HsBatch(self.model, n_envs, device=device, precision=precision, seed=seed,
                             full_state=bool(cfg.get("full_state_obs", False)), groups=groups)
        self.duration = float(cfg.get("duration", 15))
        self.frame_skip = int(cfg.get("frame_skip", 5))
        self.reward_config = cfg.get("reward_config", {"type": "default"})
        rtype = self.reward_config.get("type", "default")
        rid = _rf.device_reward_id(rtype)
        params = self.reward_config.get("params")
        # user-registered reward callables run on the host over per-env data views (slow, correct):
        # the kernel then steps without a reward and without auto-reset, so the callable sees the
        # pre-reset state; finished envs are reset by a second (masked) launch
        self._host_reward = None if rid is not None else _rf.REWARD_FUNCTIONS[rtype]
        # each SubprocVecEnv worker holds its own copy of reward_config (the callables may mutate params)
        self._host_params = ([copy.deepcopy(params) for _ in range(n_envs)] if self._host_reward is not None
                             else None)
        self.batch.configure(frame_skip=self.frame_skip, duration=self.duration, max_steps=750,
                             reward_id=rid if rid is not None else -1, autoreset=1 if rid is not None else 0,
                             max_newton=max_newton, init_height=1.282, noise_scale=0.01,
                             kneel_params=params if rid == 1 and params else None)
        obs_space = Box(low=-np.inf, high=np.inf, shape=(self.batch.obs_dim,), dtype=np.float64)
        act_space = Box(low=-1, high=1, shape=(self.model.nu,), dtype=np.float32)
        super().__init__(n_envs, obs_space, act_space)
        self._actions = None
        self._seed = seed
        self._seeds = None          # pending SB3 seeds (applied by the next reset)
        self._streams = None        # per-env np.random.RandomState once seeded (host noise mode)
        self.render_mode = None

    # ---------------------------------------------------------------- device fast path
    # Protocol the on-device trainer (ppo.PPO) relies on: num_envs, obs_dim, act_dim, device,
    # reset_tensors(), step_tensors(actions), terminal_obs.
    @property
    def obs_dim(self):
        return self.batch.obs_dim

    @property
    def act_dim(self):
        return self.model.nu

    @property
    def device(self):
        return self.batch.device

    @property
    def graph_safe(self):
        """step_tensors is launches only (device reward, one stream, no host sync), so a trainer
        may capture it in a HIP graph.  Not while SB3-seeded host reset-noise streams are active
        (or pending from ``seed()``): step_tensors then reads the done flags back every step."""
        return (self._host_reward is None and getattr(self.batch, "_streams", None) is None
                and self._streams is None and self._seeds is None)

    def rollout_handle(self):
        """The hs_batch handle a fused PPO rollout (hs_rollout) may step, or None: the fp64 Newton
        engine with the device reward and on-device reset noise (graph_safe), one stream group and
        auto-reset on."""
        b = self.batch
        if (not self.graph_safe or b.precision != "fp64" or not b.cfg.autoreset or len(b._groups) != 1
                or int(self.model.field("opt_solver")[0]) != 0):
            return None
        return b._groups[0][0]

    @property
    def terminal_obs(self):
        """[N, obs_dim] device tensor: pre-reset obs of envs whose episode ended in the last step."""
        return self.batch.terminal_obs

    def reset_tensors(self):
        """reset() on the device: returns the [N, obs_dim] device obs tensor."""
        if self._seeds is not None:      # SB3: worker i runs env.reset(seed=seed + i) -> np.random.seed
            self._streams = [np.random.RandomState(s) for s in self._seeds]
            self._seeds = None
        if self._streams is None:
            return self.batch.reset()
        qn, vn = self._draw_noise(range(self.num_envs))
        obs = self.batch.reset(qpos_noise=qn, qvel_noise=vn)
        if self._host_reward is None:    # device auto-reset reads the pre-drawn next noise
            self._bind_next_noise()
        return obs

    def step_tensors(self, actions):
        """actions: [N, nu] float32 tensor on the env's GPU (clipped to [-1, 1] by the caller, as
        SB3 does).  Returns device views (obs, reward, terminated, truncated) valid until the next
        call; ``self.batch.terminal_obs`` holds pre-reset obs of envs that just finished."""
        if self._host_reward is not None:
            return self._step_host_reward(actions)
        out = self.batch.step(actions)
        if self._streams is not None:     # host noise streams: refresh the envs that auto-reset (syncs)
            self._refresh_noise(((out[2] != 0) | (out[3] != 0)).cpu().numpy())
        return out

    def _step_host_reward(self, actions):
        """custom_env.py:201-211 with a host reward callable: step (no auto-reset), evaluate
        ``REWARD_FUNCTIONS[type](data_i, params_i)`` per env on the pre-reset state (0 when
        truncated), then reset the finished envs (SB3 auto-reset) with one masked launch."""
        import torch
        b = self.batch
        obs, rew, term, trunc = b.step(actions)
        views = _HostViews(b, self.model)
        tr = trunc.cpu().numpy().astype(bool)
        r = np.zeros(self.num_envs)
        for i in range(self.num_envs):
            if not tr[i]:
                r[i] = float(self._host_reward(views.env(i), self._host_params[i] if self._host_params else None))
        rew.copy_(torch.as_tensor(r, device=rew.device, dtype=rew.dtype))
        b.total_reward.add_(rew)
        done = (term != 0) | (trunc != 0)
        if bool(done.any()):
            b.terminal_obs[done] = obs[done]
            b.terminal_step_count[done] = b.step_count[done]
            b.terminal_total_reward[done] = b.total_reward[done]
            if self._streams is None:
                b.reset(mask=done.to(torch.uint8))
            else:
                qn, vn = self._draw_noise(np.flatnonzero(done.cpu().numpy()))
                b.reset(mask=done.to(torch.uint8), qpos_noise=qn, qvel_noise=vn)
        return b.obs, rew, term, trunc

    # ---------------------------------------------------------------- SB3 VecEnv API
    def reset(self):
        return self.reset_tensors().double().cpu().numpy()

    def episode_length(self):
        """Env steps per episode: until time >= duration (custom_env.py:213; the reset's one mj_step
        already took time to one timestep), at most the 750-step truncation (custom_env.py:203)."""
        dt = self.model.opt.timestep
        k = int(np.ceil((self.duration - dt) / (self.frame_skip * dt) - 1e-9))
        return max(1, min(750, k))

    def stagger_episode_clocks(self):
        """Spread the envs' episode clocks over one episode: env i carries on as if it were
        floor(i L / N) of the L env steps into its current episode (time and step count advanced,
        state untouched), so its first episode ends early and from then on the envs reset at evenly
        spread times.  A training-schedule choice, not SubprocVecEnv semantics: with n_steps x n_envs
        rollouts far shorter than an episode (32 x 4096) it lets every rollout see every phase of an
        episode, as the reference's 8 envs x 2048 steps (three whole episodes per env) do
        (profiles/learning_curve_r5.md: all seeds stand with it, few without)."""
        import torch
        n, L = self.num_envs, self.episode_length()
        k = np.floor(np.arange(n) * L / n)
        dt = self.model.opt.timestep
        t = self.batch.t
        t["time"].copy_(torch.as_tensor(dt + k * self.frame_skip * dt, dtype=t["time"].dtype))
        t["step_count"].copy_(torch.as_tensor(k, dtype=t["step_count"].dtype))

    # ---------------------------------------------------------------- host reset-noise streams
    def _draw_noise(self, envs):
        """The next reset's raw noise of each env in ``envs`` from its own stream, in
        custom_env.py:109-110's draw order (qpos then qvel); rows of other envs are zero."""
        m = self.model
        qn, vn = np.zeros((self.num_envs, m.nq)), np.zeros((self.num_envs, m.nv))
        for i in envs:
            r = self._streams[i]
            qn[i] = r.uniform(low=-0.01, high=0.01, size=m.nq)
            vn[i] = r.uniform(low=-0.01, high=0.01, size=m.nv)
        return qn, vn

    def _bind_next_noise(self):
        """Pre-draw every env's next (auto-)reset noise and bind it to the step kernel."""
        qn, vn = self._draw_noise(range(self.num_envs))
        self._next_noise = self.batch.set_autoreset_noise(qn, vn)

    def _refresh_noise(self, done):
        """Envs that just auto-reset consumed their bound noise: draw their next one."""
        import torch
        idx = np.flatnonzero(done)
        if self._streams is None or idx.size == 0:
            return
        qn, vn = self._draw_noise(idx)
        t = torch.as_tensor(idx, device=self.batch.device)
        self._next_noise[0][t] = torch.as_tensor(qn[idx], device=self.batch.device, dtype=self.batch.dtype)
        self._next_noise[1][t] = torch.as_tensor(vn[idx], device=self.batch.device, dtype=self.batch.dtype)

    def step_async(self, actions):
        """SB3 VecEnv.step_async: the actions go to the device through a pinned staging buffer."""
        import torch
        a = np.asarray(actions, dtype=np.float32).reshape(self.num_envs, -1)
        pin = getattr(self, "_act_pin", None)
        if pin is None or tuple(pin.shape) != a.shape:
            pin = self._act_pin = torch.empty(a.shape, dtype=torch.float32, pin_memory=True)
            self._act_dev = torch.empty(a.shape, dtype=torch.float32, device=self.batch.device)
        torch.cuda.current_stream(self.batch.device).synchronize()   # the previous upload has left the pinned buffer
        pin.numpy()[...] = a
        self._act_dev.copy_(pin, non_blocking=True)
        self._actions = self._act_dev

    def step_wait(self):
        """SB3 VecEnv.step_wait: (obs, rewards, dones, infos) as numpy with SubprocVecEnv's
        auto-reset semantics (train_sb3.py:203; custom_env.py:216-230 info keys).  The step's
        outputs come back in ONE packed device-to-host copy; ``infos`` is a lazy sequence whose
        dicts are built on first access (``StepInfos``) -- equal to the per-env info dicts
        SubprocVecEnv returns, including ``terminal_observation`` and ``TimeLimit.truncated``."""
        import torch
        a = self._actions
        if not isinstance(a, torch.Tensor):
            a = torch.as_tensor(a, device=self.batch.device)
        self.step_tensors(a)
        obs_np, cols, warn = self.batch.host_outputs(ncols=7, warnings=True)
        self._report_new_warnings(warn)
        rew_np = cols[0].copy()
        term_np, trunc_np = cols[1] != 0, cols[2] != 0
        dones = term_np | trunc_np
        idx = np.flatnonzero(dones)
        term_obs = None
        step_count, tot = cols[4], cols[3]
        if idx.size:
            # the finished episodes' final info (SubprocVecEnv returns the last step's info before
            # the worker resets: step_count 667 / 750, the episode's total_reward; custom_env.py:216-224)
            rows = torch.as_tensor(idx, device=self.batch.device)
            term_obs = self.batch.terminal_obs.index_select(0, rows).double().cpu().numpy()
            step_count = np.where(dones, cols[5], step_count)
            tot = np.where(dones, cols[6], tot)
        return obs_np, rew_np, dones, StepInfos(obs_np, term_np, trunc_np, step_count, tot, idx, term_obs)

    def _report_new_warnings(self, tot):
        """The warning counters this step added (the packed copy carries their sums): bad-state resets
        warn as MuJoCo's mj_step does, a lost hand-off raises HsimError (batch.report_warnings), so
        SB3's own PPO on this VecEnv sees them too."""
        prev = self.__dict__.get("_warn_seen")
        self._warn_seen = tot
        new = tot - prev if prev is not None else tot
        if new.any():
            report_warnings(new, "step")

    def warning_counts(self):
        """The per-env warning counters (include/hsim.h HS_WARN_*: bad qpos / qvel / qacc resets,
        contacts dropped past the wide tier, lost chunk-queue hand-offs) summed over the envs, as a
        host int64 array -- cumulative since the batch was created."""
        return self.batch.warning.sum(0).cpu().numpy().astype(np.int64)

    def close(self):
        self.batch.close()

    def seed(self, seed=None):
        """SB3 VecEnv.seed: env i gets seed + i, applied at the next ``reset()``; from then on every
        reset and auto-reset of env i draws its noise from np.random.RandomState(seed + i), as
        SubprocVecEnv worker i's global numpy stream does (custom_env.py:99-110).  Also re-seeds
        the on-device RNG (used when no host streams are active)."""
        if seed is None:
            seed = int(np.random.randint(0, np.iinfo(np.uint32).max, dtype=np.uint32))
        self._seed = int(seed)
        self.batch.set_seed(self._seed)
        self._seeds = [self._seed + i for i in range(self.num_envs)]
        return list(self._seeds)

    def get_attr(self, attr_name, indices=None):
        idx = self._indices(indices)
        val = getattr(self, attr_name)
        return [val for _ in idx]

    def set_attr(self, attr_name, value, indices=None):
        setattr(self, attr_name, value)

    def env_method(self, method_name, *method_args, indices=None, **method_kwargs):
        idx = self._indices(indices)
        fn = getattr(self, method_name)
        return [fn(*method_args, **method_kwargs) for _ in idx]

    def env_is_wrapped(self, wrapper_class, indices=None):
        return [False for _ in self._indices(indices)]

    def get_images(self, indices=None, camera="side", height=480, width=640):
        """SB3 VecEnv.get_images: one rgb frame per env (render.Renderer over GPU kinematics;
        host ray casting, ~0.15 s per 480x640 frame, so meant for a few envs)."""
        from types import SimpleNamespace

        from .render import Renderer
        if getattr(self, "_renderer", None) is None or (self._renderer.height, self._renderer.width) != (height, width):
            self._renderer = Renderer(self.model, height=height, width=width)
        out = []
        for i in self._indices(indices):
            self._renderer.update_scene(SimpleNamespace(_env=SimpleNamespace(_batch=self.batch, _idx=int(i))),
                                        camera=camera)
            out.append(self._renderer.render())
        return out

    def _indices(self, indices):
        if indices is None:
            return range(self.num_envs)
        if isinstance(indices, int):
            return [indices]
        return indices


class StepInfos(Sequence):
    """The ``infos`` of one ``step_wait``: a read-only sequence of the per-env info dicts
    SubprocVecEnv returns (custom_env.py:216-230 keys; for a finished env also
    ``terminal_observation`` and ``TimeLimit.truncated``).  The dicts are built by the native
    builder (``csrc/hs_infos.c``) on the first access, all at once, and then kept (a consumer may
    annotate one, as SB3's VecMonitor does with ``episode``); a consumer that reads none pays
    nothing.  Building 4096 dicts in Python costs ~5 ms per step, more than the physics."""

    __slots__ = ("_cols", "_idx", "_tobs", "_cache", "_n")

    def __init__(self, obs, term, trunc, step_count, total, done_idx, term_obs):
        h = obs[:, 0].copy()
        if done_idx.size:
            h[done_idx] = term_obs[:, 0]
        self._n = len(term)
        # numpy columns until the first access (their conversion to Python scalars is deferred too)
        self._cols = (h, step_count.copy(), trunc.copy(), term.copy(), total.copy())
        self._idx = done_idx
        self._tobs = term_obs
        self._cache = None

    def __len__(self):
        return self._n

    def _all(self):
        if self._cache is None:
            h, sc, tr, te, tot = self._cols
            pos = {int(i): k for k, i in enumerate(self._idx)}
            args = (h.tolist(), sc.astype(np.int64).tolist(), tr.tolist(), te.tolist(), tot.tolist(), pos, self._tobs)
            try:        # the native builder (csrc/hs_infos.c, built for the interpreter of the Makefile)
                from . import _hsinfo
                self._cache = _hsinfo.build(*args, 0, self._n)
            except ImportError:
                self._cache = _build_infos_py(*args)
        return self._cache

    def __getitem__(self, i):
        return self._all()[i]

    def __iter__(self):
        return iter(self._all())

    def __repr__(self):
        return f"StepInfos({len(self)} envs)"


def _build_infos_py(h, sc, tr, te, tot, pos, tobs):
    """The info dicts in Python (what csrc/hs_infos.c builds): custom_env.py:216-224 keys, plus
    SB3's terminal_observation / TimeLimit.truncated for the envs that finished this step."""
    out = []
    for i in range(len(h)):
        d = {"reward_components": {}, "height": h[i], "step_count": sc[i], "truncated": tr[i],
             "truncation_info": {"reason": "timeout"} if tr[i] else {}, "terminated": te[i], "total_reward": tot[i]}
        k = pos.get(i)
        if k is not None:
            d["terminal_observation"] = tobs[k]
            d["TimeLimit.truncated"] = bool(tr[i] and not te[i])
        out.append(d)
    return out


def _config_of_factory(fn):
    """env_config of an SB3 env factory: ``make_env(env_config, rank)`` returns a closure over the
    config dict (train_sb3.py:108-115), read from the closure cells; otherwise the factory is
    called once and its env's ``env_config`` read."""
    for cell in getattr(fn, "__closure__", None) or ():
        v = cell.cell_contents
        if isinstance(v, dict) and "model_path" in v:
            return v
    env = fn()
    cfg = getattr(env, "env_config", None)
    if hasattr(env, "close"):
        env.close()
    if not isinstance(cfg, dict):
        raise TypeError("cannot recover env_config from the env factory")
    return cfg


class _HostViews:
    """Host copies of one step's batched state (one device->host transfer per field) with per-env
    MjData-like views for host reward callables (the fields reward_functions.py reads)."""

    def __init__(self, batch, model):
        self.m = model
        need = _lib.HS_OUT_AUX | _lib.HS_OUT_CTRL
        if (batch.cfg.outputs & need) != need:
            raise HsimError("host reward views need the aux row and the ctrl copy (HsBatch.configure(aux=True, ctrl=True))")
        self.qpos = batch.qpos.double().cpu().numpy()
        self.qvel = batch.qvel.double().cpu().numpy()
        self.ctrl = batch.ctrl.double().cpu().numpy()
        self.time = batch.time.double().cpu().numpy()
        self.obs = batch.obs.double().cpu().numpy()
        self.com = batch.aux[:, 32:35].double().cpu().numpy()
        self.parent = None
        fs = batch.full_state
        self.cfrc = batch.cfrc_ext.double().cpu().numpy() if fs else None
        self.linv = batch.subtree_linvel.double().cpu().numpy() if fs else None

    def env(self, i):
        from types import SimpleNamespace
        m = self.m
        o2 = (m.nq - 2) + m.nv
        o3, o4 = o2 + 10 * m.nbody, o2 + 16 * m.nbody
        from .env import subtree_com_from_cinert
        if self.parent is None:
            self.parent = m.field("body_parentid").astype(int)
        cinert = self.obs[i, o2:o3].reshape(m.nbody, 10)
        com = subtree_com_from_cinert(cinert, self.com[i], self.parent)
        return SimpleNamespace(
            qpos=self.qpos[i], qvel=self.qvel[i], ctrl=self.ctrl[i], time=float(self.time[i]),
            cinert=cinert, cvel=self.obs[i, o3:o4].reshape(m.nbody, 6),
            qfrc_actuator=self.obs[i, o4:o4 + m.nv], subtree_com=com,
            cfrc_ext=self.cfrc[i] if self.cfrc is not None else np.zeros((m.nbody, 6)),
            subtree_linvel=self.linv[i] if self.linv is not None else np.zeros((m.nbody, 3)))

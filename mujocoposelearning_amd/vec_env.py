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

Auto-reset noise comes from an on-device counter RNG (seed, env, episode) instead of numpy's
global MT19937 (the per-env HumanoidEnv keeps the exact numpy stream).
"""
from __future__ import annotations

import numpy as np

from . import reward_functions as _rf
from .batch import HsBatch
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
    def __init__(self, env_config, n_envs=8, device=0, precision="fp32", seed=0, model=None, max_newton=None,
                 groups="auto"):
        if callable(env_config):            # SB3 style list of env_fns is not meaningful on device
            raise TypeError("pass the env_config dict (train_sb3.py:183-200), not env factories")
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
        if rid is None:
            raise NotImplementedError(f"reward '{rtype}' is a user callable; the batched env needs a device reward "
                                      f"(use HumanoidEnv for host-side custom rewards)")
        params = self.reward_config.get("params")
        self.batch.configure(frame_skip=self.frame_skip, duration=self.duration, max_steps=750, reward_id=rid,
                             autoreset=1, max_newton=max_newton, init_height=1.282, noise_scale=0.01,
                             kneel_params=params if rid == 1 and params else None)
        obs_space = Box(low=-np.inf, high=np.inf, shape=(self.batch.obs_dim,), dtype=np.float64)
        act_space = Box(low=-1, high=1, shape=(self.model.nu,), dtype=np.float32)
        super().__init__(n_envs, obs_space, act_space)
        self._actions = None
        self._seed = seed
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
    def terminal_obs(self):
        """[N, obs_dim] device tensor: pre-reset obs of envs whose episode ended in the last step."""
        return self.batch.terminal_obs

    def reset_tensors(self):
        return self.batch.reset()

    def step_tensors(self, actions):
        """actions: [N, nu] float32 tensor on the env's GPU (clipped to [-1, 1] by the caller, as
        SB3 does).  Returns device views (obs, reward, terminated, truncated) valid until the next
        call; ``self.batch.terminal_obs`` holds pre-reset obs of envs that just finished."""
        return self.batch.step(actions)

    # ---------------------------------------------------------------- SB3 VecEnv API
    def reset(self):
        obs = self.batch.reset()
        return obs.double().cpu().numpy()

    def step_async(self, actions):
        self._actions = np.asarray(actions, dtype=np.float32).reshape(self.num_envs, -1)

    def step_wait(self):
        import torch
        a = torch.as_tensor(self._actions, device=self.batch.device)
        obs, rew, term, trunc = self.batch.step(a)
        obs_np = obs.double().cpu().numpy()
        rew_np = rew.double().cpu().numpy()
        term_np = term.cpu().numpy().astype(bool)
        trunc_np = trunc.cpu().numpy().astype(bool)
        dones = term_np | trunc_np
        tot = self.batch.total_reward.double().cpu().numpy()
        step_count = self.batch.step_count.cpu().numpy()
        term_obs = self.batch.terminal_obs.double().cpu().numpy() if dones.any() else None
        infos = []
        for i in range(self.num_envs):
            info = {"height": None, "step_count": int(step_count[i]), "truncated": bool(trunc_np[i]),
                    "truncation_info": {"reason": "timeout"} if trunc_np[i] else {}, "terminated": bool(term_np[i]),
                    "total_reward": float(tot[i]), "reward_components": {}}
            if dones[i]:
                info["terminal_observation"] = term_obs[i]
                info["TimeLimit.truncated"] = bool(trunc_np[i] and not term_np[i])
                info["height"] = float(term_obs[i][0])
            else:
                info["height"] = float(obs_np[i][0])
            infos.append(info)
        return obs_np, rew_np, dones, infos

    def close(self):
        self.batch.close()

    def seed(self, seed=None):
        """Re-seeds the on-device reset RNG (affects subsequent resets / auto-resets)."""
        self._seed = 0 if seed is None else int(seed)
        self.batch.set_seed(self._seed)
        return [self._seed + i for i in range(self.num_envs)]

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

    def get_images(self):
        raise NotImplementedError("rendering is out of scope for this engine")

    def _indices(self, indices):
        if indices is None:
            return range(self.num_envs)
        if isinstance(indices, int):
            return [indices]
        return indices

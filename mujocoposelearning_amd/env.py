"""HumanoidEnv -- drop-in for the reference custom_env.py:HumanoidEnv, stepped on the GPU.

Same constructor keys and defaults (custom_env.py:21-43), same ``reset``/``step`` return
tuples and info keys (custom_env.py:133-150, 216-230), same 352-float observation layout with
the same stale derived fields (custom_env.py:232-261), same reward plug-in dispatch including
the ``ValueError`` for unknown types (custom_env.py:263-271).  Reset noise is drawn from
numpy's global legacy RNG exactly as the reference (custom_env.py:99-117), so
``reset(seed=s)`` reproduces the reference's initial state bit-for-bit before the physics step.

Additive env_config keys: ``device`` (GPU index, default 0), ``precision`` ('fp64' default
for this single-env surface, 'fp32'), ``max_newton``.
"""
from __future__ import annotations

from pathlib import Path

import numpy as np

from . import _lib
from . import reward_functions as _rf
from ._lib import HsimError
from .batch import HsBatch, report_warnings
from .model import HsModel
from .render import Renderer, write_video
from .spaces import Box, Env

CLIP_OBSERVATION_VALUE = np.inf   # custom_env.py:9
ACTION_CLIP_VALUE = 1             # custom_env.py:10


def subtree_com_from_cinert(cinert, com0, parent):
    """Per-body subtree COM (MuJoCo mj_comPos) from one forward pass's cinert.

    cinert[b] = [I(6), m_b (xipos_b - com0) (3), m_b] with com0 the root subtree's COM, so
    subtree_com[b] = com0 + sum_{c in subtree(b)} m_c d_c / sum m_c (children have larger ids
    than their parents, so one backward pass accumulates the subtrees).  A massless subtree gets
    com0 (MuJoCo: the body's xipos; no such body in the supported model class carries joints)."""
    cinert = np.asarray(cinert, np.float64)
    nb = cinert.shape[0]
    md = cinert[:, 6:9].copy()
    mass = cinert[:, 9].copy()
    for b in range(nb - 1, 0, -1):
        p = int(parent[b])
        md[p] += md[b]
        mass[p] += mass[b]
    out = np.empty((nb, 3))
    for b in range(nb):
        out[b] = com0 + (md[b] / mass[b] if mass[b] > 1e-15 else 0.0)
    return out


class HsData:
    """Read-only MjData-like view of one env (fields the reward plug-ins read)."""

    def __init__(self, env):
        self._env = env

    def _b(self):
        return self._env._batch

    def _obs(self):
        return self._b().obs[self._env._idx].double().cpu().numpy()

    @property
    def qpos(self):
        return self._b().qpos[self._env._idx].double().cpu().numpy()

    @property
    def qvel(self):
        return self._b().qvel[self._env._idx].double().cpu().numpy()

    @property
    def ctrl(self):
        return self._b().ctrl[self._env._idx].double().cpu().numpy()

    @property
    def time(self):
        return float(self._b().time[self._env._idx].item())

    @property
    def qacc_warmstart(self):
        return self._b().qacc_warmstart[self._env._idx].double().cpu().numpy()

    def _slices(self):
        m = self._env.model
        o1 = m.nq - 2
        o2 = o1 + m.nv
        o3 = o2 + 10 * m.nbody
        o4 = o3 + 6 * m.nbody
        return o1, o2, o3, o4

    @property
    def cinert(self):
        o1, o2, o3, o4 = self._slices()
        return self._obs()[o2:o3].reshape(self._env.model.nbody, 10)

    @property
    def cvel(self):
        o1, o2, o3, o4 = self._slices()
        return self._obs()[o3:o4].reshape(self._env.model.nbody, 6)

    @property
    def qfrc_actuator(self):
        o1, o2, o3, o4 = self._slices()
        return self._obs()[o4:o4 + self._env.model.nv]

    @property
    def subtree_com(self):
        """MjData.subtree_com of the last forward pass, every body (mj_comPos): rebuilt from the
        same pass's cinert (obs rows, custom_env.py:240) and the root COM (aux row)."""
        b = self._b()
        if not (b.cfg.outputs & _lib.HS_OUT_AUX):
            raise HsimError("data.subtree_com needs the aux output (HsBatch.configure(aux=True))")
        com0 = b.aux[self._env._idx, 32:35].double().cpu().numpy()
        return subtree_com_from_cinert(self.cinert, com0, self._env._body_parent)

    @property
    def subtree_linvel(self):
        """Zeros as in the reference (lazy in mj_step); computed with ``full_state_obs``."""
        if not self._b().full_state:
            return np.zeros((self._env.model.nbody, 3))
        return self._b().subtree_linvel[self._env._idx].double().cpu().numpy()

    @property
    def cfrc_ext(self):
        """Zeros as in the reference (lazy in mj_step); computed with ``full_state_obs``."""
        if not self._b().full_state:
            return np.zeros((self._env.model.nbody, 6))
        return self._b().cfrc_ext[self._env._idx].double().cpu().numpy()

    @property
    def warning(self):
        return self._b().warning[self._env._idx].cpu().numpy()


class HumanoidEnv(Env):
    metadata = {"render_modes": ["rgb_array"], "render_fps": 60}

    def __init__(self, env_config):
        super().__init__()
        if isinstance(env_config, dict):
            self.model_path = env_config.get('model_path')
            self.duration = env_config.get('duration', 15)
            self.framerate = env_config.get('framerate', 60)
            self.render_mode = env_config.get('render_mode')
            self.render_interval = env_config.get('render_interval', 100)
            self.reward_config = env_config.get('reward_config', {'type': 'default'})
            self.frame_skip = env_config.get('frame_skip', 5)
            self.grace_period_length = env_config.get('grace_period_length', 300)
            self.grace_period_steps = 0
            self.total_reward = 0.0
            self.run_name = env_config.get('run_name')
            device = env_config.get('device', 0)
            precision = env_config.get('precision', 'fp64')
            max_newton = env_config.get('max_newton', 100)
            # opt-in: cfrc_ext / subtree_linvel computed (reference: zeros) and obs += cfrc_ext[1:]
            full_state = bool(env_config.get('full_state_obs', False))
        else:
            self.model_path = env_config
            self.duration = 15
            self.framerate = 60
            self.render_mode = None
            self.render_interval = 100
            self.reward_config = {'type': 'default'}
            self.frame_skip = 5
            self.grace_period_steps = 0
            self.total_reward = 0.0
            device, precision, max_newton, full_state = 0, 'fp64', 100, False
        self.model = HsModel(self.model_path)
        self._body_parent = self.model.field("body_parentid").astype(int)
        self._batch = HsBatch(self.model, 1, device=device, precision=precision, full_state=full_state)
        self._idx = 0
        self.data = HsData(self)
        self.frames = []
        self.renderer = None
        self.step_count = 0
        self.init_qpos = self.model.qpos0.copy()
        self.init_qpos[2] = 1.282
        self.init_qpos[3:7] = [1, 0, 0, 0]
        self.init_qvel = np.zeros(self.model.nv)
        self._configure(max_newton)
        obs_size = self._batch.obs_dim
        self.observation_space = Box(low=-CLIP_OBSERVATION_VALUE, high=CLIP_OBSERVATION_VALUE, shape=(obs_size,),
                                     dtype=np.float64)
        self.action_space = Box(low=-ACTION_CLIP_VALUE, high=ACTION_CLIP_VALUE, shape=(self.model.nu,),
                                dtype=np.float32)
        if self.render_mode == "rgb_array":   # custom_env.py:63-66
            self.renderer = Renderer(self.model)
        self.reset()

    def _configure(self, max_newton):
        rtype = self.reward_config.get('type', 'default')
        self._reward_dev = _rf.DEVICE_REWARD_IDS.get(_rf.REWARD_FUNCTIONS.get(rtype))
        params = self.reward_config.get('params')
        kneel = params if (self._reward_dev == 1 and params) else None
        self._batch.configure(frame_skip=self.frame_skip, duration=float(self.duration), max_steps=750,
                              reward_id=self._reward_dev if self._reward_dev is not None else -1, autoreset=0,
                              max_newton=max_newton, init_height=float(self.init_qpos[2]), noise_scale=0.01,
                              kneel_params=kneel)

    def reset(self, *, seed=None, options=None):
        """custom_env.py:97-150."""
        if seed is not None:
            np.random.seed(seed)
        pos_noise = np.random.uniform(low=-0.01, high=0.01, size=self.model.nq)
        vel_noise = np.random.uniform(low=-0.01, high=0.01, size=self.model.nv)
        # the kernel applies pos_noise[2] *= 0.1, pos_noise[3:7] = 0 and the init pose (custom_env.py:105-117)
        self._batch.reset(qpos_noise=pos_noise[None], qvel_noise=vel_noise[None])
        self.frames = []          # custom_env.py:123-127
        if self.renderer:
            self.renderer.close()
            self.renderer = None
        state = self._get_state()
        info = {
            'reward_components': {'forward': 0.0, 'standing': 0.0, 'healthy_pose': 0.0, 'alive': 0.0, 'total': 0.0},
            'height': float(state[0]),
            'forward_velocity': float(state[self.model.nq - 2]),
            'truncated': False,
            'terminated': False,
        }
        self.step_count = 0
        self.total_reward = 0.0
        return state, info

    def step(self, action):
        """custom_env.py:152-230 (frame_skip substeps on the GPU, reward on the GPU for built-ins)."""
        import torch
        self.step_count += 1
        a = torch.as_tensor(np.asarray(action, dtype=np.float32).reshape(1, -1), device=self._batch.device)
        self._batch.step(a)
        # obs, reward, done flags and the warning counters in one copy; a bad-state reset warns as
        # mj_step's mju_warning does, a lost hand-off raises (batch.report_warnings)
        obs, cols, warn = self._batch.host_outputs(ncols=3, warnings=True)
        new = warn - self.__dict__.get("_warn_seen", 0)     # counters start at 0 with the batch
        self._warn_seen = warn
        if new.any():
            report_warnings(new, "step")
        state = obs[0]
        height = state[0]
        truncated = bool(cols[2, 0])
        truncation_info = {}
        if truncated:
            truncation_info['reason'] = 'timeout'
            reward = 0.0
        else:
            reward = float(cols[0, 0]) if self._reward_dev is not None else self._compute_reward()
            params = self.reward_config.get('params')
            if params is not None and self._reward_dev in (0, 2):
                params["previous_qpos"] = self.data.qpos.copy()   # stand/walk side effect (reward_functions.py:208)
        self.total_reward += reward
        terminated = bool(cols[1, 0])
        info = {
            'reward_components': getattr(self, 'reward_components', {}),
            'height': height,
            'step_count': self.step_count,
            'truncated': truncated,
            'truncation_info': truncation_info,
            'terminated': terminated,
            'total_reward': self.total_reward,
        }
        if self.render_mode == "rgb_array":   # custom_env.py:227-228
            self.render()
        return state, reward, terminated, truncated, info

    def _get_state(self):
        return self._batch.obs[0].double().cpu().numpy()

    def _compute_reward(self):
        reward_type = self.reward_config.get('type', 'default')
        reward_params = self.reward_config.get('params', None)
        if reward_type not in _rf.REWARD_FUNCTIONS:
            raise ValueError(f"Unknown reward type: {reward_type}")
        return _rf.REWARD_FUNCTIONS[reward_type](self.data, reward_params)

    def render(self):
        """custom_env.py:273-289: one 480x640 frame from the 'side' camera while the frame count is
        below time x framerate (render.Renderer: host ray casting over GPU-computed poses)."""
        if self.render_mode != "rgb_array":
            return
        if self.renderer is None:
            self.renderer = Renderer(self.model, height=480, width=640)
        if len(self.frames) < self.data.time * self.framerate:
            camera_id = self.model.camera('side').id
            self.renderer.update_scene(self.data, camera=camera_id)
            self.frames.append(self.renderer.render())

    def save_video(self, episode_num):
        """custom_env.py:291-321, written as recordings/[run_name/]episode_<n>.gif: mediapy's h264
        mp4 encoder (ffmpeg) is not in this image.  Returns the path (None without frames)."""
        recordings_dir = Path("recordings")
        if getattr(self, 'run_name', None):
            recordings_dir = recordings_dir / self.run_name
        recordings_dir.mkdir(parents=True, exist_ok=True)
        video_path = recordings_dir / f"episode_{episode_num}.gif"
        if video_path.exists():
            video_path.unlink()
        out = None
        if len(self.frames) > 0:
            out = str(write_video(str(video_path), self.frames, fps=self.framerate))
        else:
            print("No frames to save!")
        self.frames = []
        if self.renderer:
            self.renderer.close()
            self.renderer = None
        return out

    def close(self):
        if self.renderer:
            self.renderer.close()
            self.renderer = None
        self._batch.close()

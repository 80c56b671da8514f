"""ORACLE (test infrastructure only): CPU restatement of the reference HumanoidEnv semantics
(custom_env.py:18-271) on top of the fp64 mj_step restatement.  Used by tests (env KATs,
GPU parity) and by bench.py's cpu_baseline leg (the reference's n_envs=8 CPU path, timed
as a port because MuJoCo/SB3 are not installable here).
"""
import numpy as np

from . import rewards
from .oracle import Oracle


class OracleHumanoidEnv:
    def __init__(self, env_config, M=None):
        self.model_path = env_config.get('model_path')
        self.duration = env_config.get('duration', 15)
        self.reward_config = env_config.get('reward_config', {'type': 'default'})
        self.frame_skip = env_config.get('frame_skip', 5)
        self.full = bool(env_config.get('full_state_obs', False))   # hsim's opt-in full-state mode
        self.sim = Oracle(self.model_path, M=M)
        self.M = self.sim.M
        self.init_qpos = self.M["qpos0"].copy()
        self.init_qpos[2] = 1.282
        self.init_qpos[3:7] = [1, 0, 0, 0]
        self.step_count = 0
        self.total_reward = 0.0
        self.reset()

    def reset(self, seed=None, pos_noise=None, vel_noise=None):
        """custom_env.py:97-150 (noise from numpy's global legacy RNG unless given)."""
        if seed is not None:
            np.random.seed(seed)
        self.sim.reset_data()
        self.sim.qpos[:] = self.init_qpos
        self.sim.qvel[:] = 0
        if pos_noise is None:
            pos_noise = np.random.uniform(low=-0.01, high=0.01, size=self.M["nq"])
        if vel_noise is None:
            vel_noise = np.random.uniform(low=-0.01, high=0.01, size=self.M["nv"])
        pos_noise = np.array(pos_noise, dtype=np.float64)
        pos_noise[2] *= 0.1
        pos_noise[3:7] = 0
        self.sim.qpos[:] += pos_noise
        self.sim.qvel[:] += vel_noise
        self.sim.step(None, 1, full=self.full)
        self.step_count = 0
        self.total_reward = 0.0
        return self.get_state(), {}

    def get_state(self):
        """custom_env.py:232-261: qpos[2:], qvel, cinert, cvel, qfrc_actuator."""
        nb = self.M["nbody"]
        parts = [self.sim.qpos[2:], self.sim.qvel, self.sim.get("cinert").reshape(nb * 10),
                 self.sim.get("cvel").reshape(nb * 6), self.sim.get("qfrc_actuator")]
        if self.full:   # + cfrc_ext[1:] (custom_env.py:247, commented out in the reference)
            parts.append(self.sim.get("cfrc_ext")[1:].reshape(-1))
        return np.concatenate(parts)

    def compute_reward(self):
        t = self.reward_config.get('type', 'default')
        q, v = self.sim.qpos[None], self.sim.qvel[None]
        return float(rewards.reward(t, q, v, self.sim.ctrl[None], np.array([self.sim.time]),
                                    self.sim.get("subtree_com")[:1], self.sim.get("subtree_linvel")[:1],
                                    self.sim.get("cfrc_ext")[None], self.sim.get("qfrc_actuator")[None],
                                    self.reward_config.get('params'))[0])

    def step(self, action):
        self.step_count += 1
        a = np.asarray(action, dtype=np.float32).astype(np.float64)
        self.sim.step(a, self.frame_skip, full=self.full)
        state = self.get_state()
        truncated = self.step_count >= 750
        reward = 0.0 if truncated else self.compute_reward()
        self.total_reward += reward
        terminated = self.sim.time >= self.duration
        return state, reward, terminated, truncated, {}

"""Reward plug-in registry -- same surface as the reference reward_functions.py.

``REWARD_FUNCTIONS[name](env_data, params) -> float`` with identical keys
(``default``, ``kneeling``, ``stand``, ``walk``; reward_functions.py:264-269) and semantics.
Each built-in also has a DEVICE implementation inside the step kernel (``hs_kernels.hip``
``compute_reward``); envs use the device path for built-ins and fall back to calling the
Python function on a read-only ``data`` view for user-registered callables (slow, correct).
"""
import numpy as np

from .utils import quaternion_to_euler


def robust_kneeling_reward(env_data, params=None):
    """reward_functions.py:66-154."""
    default_params = {'target_height': 1.282, 'min_height': 0.85, 'max_roll_pitch': np.pi / 6, 'com_radius': 0.1,
                      'energy_weight': 0.3, 'posture_weight': 0.3, 'com_weight': 0.2, 'foot_weight': 0.1,
                      'alive_weight': 0.1}
    params = {**default_params, **(params or {})}
    qpos, qvel = env_data.qpos, env_data.qvel
    h = qpos[2]
    if h < params['min_height']:
        return h ** 2
    roll, pitch, _ = quaternion_to_euler(qpos[3:7])
    # same association as the reference (:97-98): the error is divided before it is scaled
    orientation_error = (roll ** 2 + pitch ** 2) / (params['max_roll_pitch'] ** 2)
    posture = 0.7 * np.exp(-5.0 * orientation_error) + \
        0.3 * np.exp(-5.0 * np.square(h - params['target_height']))
    com_pos, com_vel = env_data.subtree_com[0], env_data.subtree_linvel[0]
    dist = np.sqrt(com_pos[0] ** 2 + com_pos[1] ** 2)
    com = 0.7 * np.exp(-10.0 * (dist / params['com_radius'])) + 0.3 * np.exp(-0.1 * np.sum(com_vel ** 2))
    lf, rf = np.sum(np.abs(env_data.cfrc_ext[-2])), np.sum(np.abs(env_data.cfrc_ext[-1]))
    foot = min(lf, rf) / (lf + rf + 1e-8)
    av = qvel[6:]
    af = env_data.qfrc_actuator[-len(av):]
    energy = np.exp(-0.01 * np.sum(np.square(af * av)))
    alive = 1.0 - np.exp(-0.5 * env_data.time)
    return (params['posture_weight'] * posture + params['com_weight'] * com + params['foot_weight'] * foot +
            params['energy_weight'] * energy + params['alive_weight'] * alive)


def stand_reward(env_data, params=None):
    """reward_functions.py:156-211 (the 'default' and 'stand' entries)."""
    h = env_data.qpos[2]
    vx = env_data.qvel[0]
    roll, pitch, _ = quaternion_to_euler(env_data.qpos[3:7])
    lf, rf = np.sum(np.abs(env_data.cfrc_ext[-2])), np.sum(np.abs(env_data.cfrc_ext[-1]))
    if h < 0.8:
        return 0.0
    vel = np.exp(-2.0 * ((vx - 1.0) ** 2))
    posture = 0.5 * np.exp(-2.0 * ((h - 1.282) ** 2)) + 0.5 * np.exp(-3.0 * (roll ** 2 + pitch ** 2))
    torque = np.exp(-0.05 * np.sum(np.square(env_data.ctrl)))
    foot = 1.0 - min(lf, rf) / (lf + rf + 1e-8)
    reward = 0.4 * vel + 0.3 * posture + 0.2 * foot + 0.1 * torque
    if params is not None:
        params["previous_qpos"] = env_data.qpos.copy()
    return reward


def walk_reward(env_data, params=None):
    """reward_functions.py:213-261."""
    h = env_data.qpos[2]
    vx = env_data.qvel[0]
    roll, pitch, _ = quaternion_to_euler(env_data.qpos[3:7])
    if h < 0.8:
        return 0.1 * h / 0.8
    vel = np.exp(-0.5 * ((vx - 10.0) ** 2))
    posture = 0.5 * np.exp(-2.0 * ((h - 1.282) ** 2)) + 0.5 * np.exp(-3.0 * (roll ** 2 + pitch ** 2))
    torque = np.exp(-0.05 * np.sum(np.square(env_data.ctrl)))
    reward = vel + posture * torque
    if params is not None:
        params["previous_qpos"] = env_data.qpos.copy()
    return reward


REWARD_FUNCTIONS = {
    'default': stand_reward,
    'kneeling': robust_kneeling_reward,
    'stand': stand_reward,
    'walk': walk_reward,
}

# built-in callables -> device kernel ids (hsim.h HS_REWARD_*)
DEVICE_REWARD_IDS = {stand_reward: 0, robust_kneeling_reward: 1, walk_reward: 2}


def device_reward_id(name, registry=None):
    """Kernel id for REWARD_FUNCTIONS[name], or None when it is a user callable (host path).
    Unknown names raise ValueError exactly like custom_env.py:268-269."""
    reg = REWARD_FUNCTIONS if registry is None else registry
    if name not in reg:
        raise ValueError(f"Unknown reward type: {name}")
    return DEVICE_REWARD_IDS.get(reg[name])

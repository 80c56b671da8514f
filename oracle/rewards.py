"""ORACLE (test infrastructure only): numpy restatement of the reference reward plug-ins.

Batched over leading axis N.  Follows, line by line in semantics:
  * utils.py:3-21                quaternion_to_euler (pitch = arcsin, NOT clipped -> NaN)
  * reward_functions.py:66-154   robust_kneeling_reward (defaults :71-83, h < 0.85 -> h^2)
  * reward_functions.py:156-211  stand_reward (h < 0.8 -> 0.0; feet = cfrc_ext[-2], [-1])
  * reward_functions.py:213-261  walk_reward (h < 0.8 -> 0.1 h / 0.8)
  * reward_functions.py:264-269  REWARD_FUNCTIONS registry
Pinned by tests/golden/reward_golden.npz (outputs of the reference functions themselves).
"""
import numpy as np

KNEEL_DEFAULTS = {'target_height': 1.282, 'min_height': 0.85, 'max_roll_pitch': np.pi / 6, 'com_radius': 0.1,
                  'energy_weight': 0.3, 'posture_weight': 0.3, 'com_weight': 0.2, 'foot_weight': 0.1,
                  'alive_weight': 0.1}


def quaternion_to_euler(quat):
    quat = np.asarray(quat, dtype=np.float64)
    w, x, y, z = quat[..., 0], quat[..., 1], quat[..., 2], quat[..., 3]
    roll = np.arctan2(2 * (w * x + y * z), 1 - 2 * (x * x + y * y))
    with np.errstate(invalid="ignore"):
        pitch = np.arcsin(2 * (w * y - z * x))
    yaw = np.arctan2(2 * (w * z + x * y), 1 - 2 * (y * y + z * z))
    return roll, pitch, yaw


def stand(qpos, qvel, ctrl, cfrc_ext):
    h = qpos[:, 2]
    roll, pitch, _ = quaternion_to_euler(qpos[:, 3:7])
    lf = np.abs(cfrc_ext[:, -2]).sum(-1)
    rf = np.abs(cfrc_ext[:, -1]).sum(-1)
    vel_r = np.exp(-2.0 * (qvel[:, 0] - 1.0) ** 2)
    post = 0.5 * np.exp(-2.0 * (h - 1.282) ** 2) + 0.5 * np.exp(-3.0 * (roll ** 2 + pitch ** 2))
    torque = np.exp(-0.05 * np.sum(np.square(ctrl), -1))
    foot = 1.0 - np.minimum(lf, rf) / (lf + rf + 1e-8)
    r = 0.4 * vel_r + 0.3 * post + 0.2 * foot + 0.1 * torque
    return np.where(h < 0.8, 0.0, r)


def kneeling(qpos, qvel, time, subtree_com0, subtree_linvel0, cfrc_ext, qfrc_actuator, params=None):
    p = {**KNEEL_DEFAULTS, **(params or {})}
    h = qpos[:, 2]
    roll, pitch, _ = quaternion_to_euler(qpos[:, 3:7])
    post = np.exp(-5.0 * ((roll ** 2 + pitch ** 2) / (p['max_roll_pitch'] ** 2)))   # :97-98 association
    hr = np.exp(-5.0 * np.square(h - p['target_height']))
    posture = 0.7 * post + 0.3 * hr
    dist = np.sqrt(subtree_com0[:, 0] ** 2 + subtree_com0[:, 1] ** 2)
    com = 0.7 * np.exp(-10.0 * (dist / p['com_radius'])) + 0.3 * np.exp(-0.1 * np.sum(subtree_linvel0 ** 2, -1))
    lf = np.abs(cfrc_ext[:, -2]).sum(-1)
    rf = np.abs(cfrc_ext[:, -1]).sum(-1)
    foot = np.minimum(lf, rf) / (lf + rf + 1e-8)
    nj = qvel.shape[1] - 6
    energy = np.exp(-0.01 * np.sum(np.square(qfrc_actuator[:, -nj:] * qvel[:, 6:]), -1))
    alive = 1.0 - np.exp(-0.5 * time)
    r = (p['posture_weight'] * posture + p['com_weight'] * com + p['foot_weight'] * foot +
         p['energy_weight'] * energy + p['alive_weight'] * alive)
    return np.where(h < p['min_height'], h ** 2, r)


def walk(qpos, qvel, ctrl):
    h = qpos[:, 2]
    roll, pitch, _ = quaternion_to_euler(qpos[:, 3:7])
    vel_r = np.exp(-0.5 * (qvel[:, 0] - 10.0) ** 2)
    post = 0.5 * np.exp(-2.0 * (h - 1.282) ** 2) + 0.5 * np.exp(-3.0 * (roll ** 2 + pitch ** 2))
    torque = np.exp(-0.05 * np.sum(np.square(ctrl), -1))
    return np.where(h < 0.8, 0.1 * h / 0.8, vel_r + post * torque)


def reward(name, qpos, qvel, ctrl, time, subtree_com0, subtree_linvel0, cfrc_ext, qfrc_actuator, params=None):
    if name in ("default", "stand"):
        return stand(qpos, qvel, ctrl, cfrc_ext)
    if name == "kneeling":
        return kneeling(qpos, qvel, time, subtree_com0, subtree_linvel0, cfrc_ext, qfrc_actuator, params)
    if name == "walk":
        return walk(qpos, qvel, ctrl)
    raise ValueError(f"Unknown reward type: {name}")

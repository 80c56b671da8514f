"""Trajectory keyframe writer -- mirrors generate_trajectories.py:6-72 of the reference.

Rolls a policy out in a HumanoidEnv (duration 30, reward 'walk', the env's default frame_skip of
5, as the reference configures it) and appends the states to the model XML's <keyframe>
section: an 'initial_pose' key after reset, then one unnamed key every ``step_interval`` env
steps with ``time = step * model.opt.timestep`` (the reference's formula; it does not include
frame_skip), qpos / qvel printed with 6 decimals.  The rollout stops at termination or
truncation (750 env steps).
"""
from __future__ import annotations

import os
import xml.etree.ElementTree as ET

import numpy as np


def _fmt(v):
    return " ".join(f"{x:.6f}" for x in np.asarray(v, dtype=np.float64))


def write_trajectory_xml(env, predict, xml_path, out_path, num_steps=1000, step_interval=5, timestep=None):
    """``env``: a HumanoidEnv-like object (reset(), step(a), data.qpos / data.qvel);
    ``predict(obs) -> action`` (e.g. ``lambda o: ppo.predict(o)[0]``).  Returns ``out_path``."""
    tree = ET.parse(xml_path)
    root = tree.getroot()
    keyframe = root.find("keyframe")
    if keyframe is None:
        keyframe = ET.SubElement(root, "keyframe")
    if timestep is None:
        timestep = float(env.model.opt.timestep)
    obs, _ = env.reset()
    key = ET.SubElement(keyframe, "key")
    key.set("name", "initial_pose")
    key.set("time", "0.000")
    key.set("qpos", _fmt(env.data.qpos))
    key.set("qvel", _fmt(env.data.qvel))
    for step in range(num_steps):
        if step % step_interval == 0:
            key = ET.SubElement(keyframe, "key")
            key.set("time", f"{step * timestep:.3f}")
            key.set("qpos", _fmt(env.data.qpos))
            key.set("qvel", _fmt(env.data.qvel))
        obs, reward, terminated, truncated, _ = env.step(predict(obs))
        if terminated or truncated:
            break
    os.makedirs(os.path.dirname(os.path.abspath(out_path)), exist_ok=True)
    tree.write(str(out_path), encoding="utf-8", xml_declaration=True)
    return str(out_path)


def generate_trajectory_xml(model_path, xml_path, out_path, num_steps=1000, step_interval=5, device=0):
    """generate_trajectories.py:6-72: load an SB3-layout checkpoint (ours or SB3's own zip), roll
    it out on the GPU engine with SB3's stochastic predict() (the reference calls
    model.predict(obs) without deterministic=True) and write the keyframe XML."""
    import json
    import zipfile

    import torch

    from .env import HumanoidEnv
    from .ppo import ActorCritic
    from .sb3_format import load_sb3_zip
    env = HumanoidEnv({"model_path": str(xml_path), "render_mode": None, "duration": 30.0,
                       "reward_config": {"type": "walk"}, "device": device})
    zp = str(model_path) if str(model_path).endswith(".zip") else str(model_path) + ".zip"
    with zipfile.ZipFile(zp) as z:
        data = json.loads(z.read("data")) if "data" in z.namelist() else {}
    pk = data.get("policy_kwargs") if isinstance(data.get("policy_kwargs"), dict) else {}
    net = pk.get("net_arch", {"pi": [64, 64], "vf": [64, 64]})          # SB3 MlpPolicy defaults
    if isinstance(net, (list, tuple)):
        net = {"pi": list(net), "vf": list(net)}
    act = pk.get("activation_fn", "Tanh")
    act = getattr(torch.nn, act) if isinstance(act, str) else torch.nn.Tanh
    policy = ActorCritic(env.observation_space.shape[0], env.action_space.shape[0], net["pi"], net["vf"], act)
    load_sb3_zip(zp, policy)
    policy.eval()

    def predict(obs):
        with torch.no_grad():
            a, _, _ = policy.act(torch.as_tensor(obs[None], dtype=torch.float32))
        return a[0].clamp(-1, 1).numpy()
    return write_trajectory_xml(env, predict, xml_path, out_path, num_steps, step_interval)

"""train_humanoid(env_kwargs, ppo_kwargs) -- mirrors the reference entry point
(train_sb3.py:170-240, called from main.py with config.py's dicts) on the device engine.

Differences by design (the hot path is on device):
* ``SubprocVecEnv([make_env(env_config, i) for i in range(n_envs)])`` (train_sb3.py:203) becomes
  ONE HumanoidVecEnv per rank holding this rank's contiguous shard of the n_envs envs.
* SB3 ``PPO("MlpPolicy", env, **ppo_kwargs)`` (train_sb3.py:208-214) becomes ppo.PPO with the
  same keyword arguments; under torch.distributed (one process per GPU, launched by torchrun)
  gradients are all-reduced once per optimizer step.
* Callbacks (progress bar, reward stats, video recorder, train_sb3.py:41-106) and tensorboard are
  out of scope; ``callback(model)`` receives the PPO object after each iteration.
"""
from __future__ import annotations

import os

import torch

from .ppo import PPO
from .vec_env import HumanoidVecEnv

from .model import HUMANOID_XML as DEFAULT_XML   # noqa: E402  (the reference's XML/humanoid.xml)


def shard_envs(n_envs: int, world_size: int, rank: int):
    """Contiguous env-id range [start, stop) of ``rank``; sizes differ by at most 1."""
    if n_envs < world_size:
        raise ValueError(f"n_envs={n_envs} < world_size={world_size}: every rank needs at least one env")
    base, extra = divmod(n_envs, world_size)
    start = rank * base + min(rank, extra)
    return start, start + base + (1 if rank < extra else 0)


def env_config_from_kwargs(env_kwargs: dict, xml_path: str = DEFAULT_XML) -> dict:
    """train_sb3.py:183-200 (duration fixed at 10.0, reward default 'walk', frame_skip default 3)."""
    return {
        "model_path": str(xml_path),
        "render_mode": None,
        "framerate": env_kwargs.get("framerate", 60),
        "duration": 10.0,
        "reward_config": {"type": env_kwargs.get("reward_function", "walk")},
        "frame_skip": env_kwargs.get("frame_skip", 3),
    }


def _resolve_activation(ppo_kwargs: dict) -> dict:
    """main.py:5-17 converts a string activation_fn to the torch.nn class."""
    kw = dict(ppo_kwargs)
    pk = dict(kw.get("policy_kwargs") or {})
    if isinstance(pk.get("activation_fn"), str):
        pk["activation_fn"] = getattr(torch.nn, pk["activation_fn"])
    if pk:
        kw["policy_kwargs"] = pk
    return kw


def train_humanoid(env_kwargs: dict, ppo_kwargs: dict, xml_path: str = DEFAULT_XML, storage_path=None,
                   precision: str = "fp64", seed: int = 0, callback=None):
    import torch.distributed as dist
    world = dist.get_world_size() if dist.is_available() and dist.is_initialized() else 1
    rank = dist.get_rank() if dist.is_available() and dist.is_initialized() else 0
    local_rank = int(os.environ.get("LOCAL_RANK", rank if world > 1 else 0))
    n_total = int(env_kwargs.get("n_envs", 8))
    start, stop = shard_envs(n_total, world, rank)
    env = HumanoidVecEnv(env_config_from_kwargs(env_kwargs, xml_path), n_envs=stop - start, device=local_rank,
                         precision=precision, seed=seed * 1_000_003 + start)
    if env.graph_safe:     # device reward: the trainer reads neither the aux row nor the ctrl copy
        env.batch.configure(aux=False, ctrl=False)
    kw = _resolve_activation(ppo_kwargs)
    model = PPO(env, seed=seed, world_size=world, rank=rank, **kw)
    model.learn(total_timesteps=env_kwargs.get("total_timesteps", 20_000_000), callback=callback)
    if storage_path is not None and rank == 0:
        os.makedirs(storage_path, exist_ok=True)
        model.save(os.path.join(storage_path, "final_model"))     # -> final_model.zip (SB3 layout)
    env.close()
    return model

"""train_humanoid(env_kwargs, ppo_kwargs) -- mirrors the reference entry point
(train_sb3.py:170-240, called from main.py with config.py's dicts) on the device engine.

Differences by design (the hot path is on device):
* ``SubprocVecEnv([make_env(env_config, i) for i in range(n_envs)])`` (train_sb3.py:203) becomes
  ONE HumanoidVecEnv per rank holding this rank's contiguous shard of the n_envs envs.
* SB3 ``PPO("MlpPolicy", env, **ppo_kwargs)`` (train_sb3.py:208-214) becomes ppo.PPO with the
  same keyword arguments; under a launcher (one process per GPU, torchrun) train_humanoid
  initialises the nccl (RCCL) group itself (init_distributed) and gradients are all-reduced once
  per optimizer step, in lockstep for any n_envs.
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


def init_distributed(backend: str | None = None):
    """One process per GPU under a launcher (torchrun / ``python -m torch.distributed.run``):
    initialise the process group from the launcher's environment (RANK, WORLD_SIZE, LOCAL_RANK,
    MASTER_ADDR/PORT), with ``nccl`` -- RCCL over xGMI on ROCm -- bound to GPU LOCAL_RANK.

    Returns (world, rank, local_rank).  Without a launcher (WORLD_SIZE unset or 1) and without an
    existing group it returns (1, 0, 0) and creates nothing.  A group the caller already created
    is used as is.  Under a multi-rank launcher with no visible GPU and no explicit ``backend`` it
    raises: N unsynchronised single-GPU trainers must never start silently."""
    import torch.distributed as dist
    if dist.is_available() and dist.is_initialized():
        return dist.get_world_size(), dist.get_rank(), int(os.environ.get("LOCAL_RANK", dist.get_rank()))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    if world <= 1:
        return 1, 0, 0
    local_rank = int(os.environ.get("LOCAL_RANK", os.environ.get("RANK", "0")))
    if backend is None:
        if not torch.cuda.is_available():
            raise RuntimeError(f"WORLD_SIZE={world} but no GPU is visible: the nccl (RCCL) group needs one "
                               "GPU per rank (pass backend='gloo' for a CPU rehearsal)")
        backend = "nccl"
    if backend == "nccl":
        torch.cuda.set_device(local_rank)
        dist.init_process_group("nccl", device_id=torch.device("cuda", local_rank))
    else:
        dist.init_process_group(backend)
    if dist.get_world_size() != world:
        raise RuntimeError(f"process group has {dist.get_world_size()} ranks, WORLD_SIZE={world}")
    return world, dist.get_rank(), local_rank


def train_humanoid(env_kwargs: dict, ppo_kwargs: dict, xml_path: str = DEFAULT_XML, storage_path=None,
                   precision: str = "fp64", seed: int = 0, callback=None, backend: str | None = None):
    world, rank, local_rank = init_distributed(backend)
    n_total = int(env_kwargs.get("n_envs", 8))
    start, stop = shard_envs(n_total, world, rank)
    env = HumanoidVecEnv(env_config_from_kwargs(env_kwargs, xml_path), n_envs=stop - start, device=local_rank,
                         precision=precision, seed=seed * 1_000_003 + start)
    if env.graph_safe:     # device reward: the trainer reads neither the aux row nor the ctrl copy
        env.batch.configure(aux=False, ctrl=False)
    kw = _resolve_activation(ppo_kwargs)
    # env_kwargs["stagger_episodes"] (hsim option, off by default: SubprocVecEnv resets every env
    # together): spread the episode clocks so that short rollouts see every episode phase
    model = PPO(env, seed=seed, world_size=world, rank=rank,
                stagger_episodes=bool(env_kwargs.get("stagger_episodes", False)), **kw)
    model.learn(total_timesteps=env_kwargs.get("total_timesteps", 20_000_000), callback=callback)
    if storage_path is not None and rank == 0:
        os.makedirs(storage_path, exist_ok=True)
        model.save(os.path.join(storage_path, "final_model"))     # -> final_model.zip (SB3 layout)
    env.close()
    return model


def load_config_from_file(path: str) -> dict:
    """main.py:6-18: a Python file exposing ``config = {"env_kwargs": ..., "ppo_kwargs": ...}``
    (e.g. the reference's config.py).  The file is executed, as main.py does: pass only configs you
    trust."""
    ns: dict = {}
    with open(path) as f:
        exec(compile(f.read(), path, "exec"), ns)
    cfg = ns.get("config")
    if not isinstance(cfg, dict) or "env_kwargs" not in cfg or "ppo_kwargs" not in cfg:
        raise ValueError(f"{path}: expected a dict `config` with 'env_kwargs' and 'ppo_kwargs'")
    return cfg


def main(argv=None) -> int:
    """Launch entry:
    ``python -m torch.distributed.run --nproc-per-node 8 --master-addr 127.0.0.1 -m
    mujocoposelearning_amd.train --config config.py``, or plain ``python -m
    mujocoposelearning_amd.train`` for one GPU.  The reference's CLI is out of scope;
    this is the minimal loader of its config files."""
    import argparse
    ap = argparse.ArgumentParser(prog="mujocoposelearning_amd.train")
    ap.add_argument("--config", help="Python config file exposing `config` (main.py:6-18)")
    ap.add_argument("--precision", default="fp64", choices=("fp32", "fp64"))
    ap.add_argument("--seed", type=int, default=0)
    ap.add_argument("--save-dir", default=None)
    ap.add_argument("--backend", default=None, help="process-group backend under a launcher (default nccl)")
    a = ap.parse_args(argv)
    cfg = load_config_from_file(a.config) if a.config else {"env_kwargs": {}, "ppo_kwargs": {}}

    def log(m):
        if m.rank == 0:
            lg = m.logger
            print(f"iter {lg['iteration']} steps {lg['timesteps']} ep_rew_mean {lg['ep_rew_mean']:.3f} "
                  f"rollout {lg['rollout_s']:.3f}s train {lg['train_s']:.3f}s", flush=True)
        return True
    train_humanoid(cfg["env_kwargs"], cfg["ppo_kwargs"], precision=a.precision, seed=a.seed,
                   storage_path=a.save_dir, callback=log, backend=a.backend)
    import torch.distributed as dist
    if dist.is_available() and dist.is_initialized():
        dist.destroy_process_group()
    return 0


if __name__ == "__main__":
    raise SystemExit(main())

"""Kernel-level view of one PPO update at the reference's batch size (README.md:23-53: batch 128,
10 epochs over 16 384 samples): run under rocprofv3 --kernel-trace --stats.
python tools/probes/gpu_update_small.py [iters]"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
import torch  # noqa: E402

from mujocoposelearning_amd.model import HUMANOID_XML, HsModel  # noqa: E402
from mujocoposelearning_amd.ppo import PPO  # noqa: E402
from mujocoposelearning_amd.train import env_config_from_kwargs  # noqa: E402
from mujocoposelearning_amd.vec_env import HumanoidVecEnv  # noqa: E402


def main(iters=3):
    cfg = env_config_from_kwargs({"reward_function": "stand", "frame_skip": 3}, HUMANOID_XML)
    env = HumanoidVecEnv(cfg, n_envs=128, model=HsModel(HUMANOID_XML), seed=0, precision="fp64")
    env.batch.configure(aux=False, ctrl=False)
    ppo = PPO(env, n_steps=128, seed=0, learning_rate=5e-5, batch_size=128, n_epochs=10, ent_coef=0.002,
              policy_kwargs={"activation_fn": "ReLU", "net_arch": {"pi": [256, 256], "vf": [256, 256]}})
    for it in range(iters):
        adv, ret = ppo.collect_rollouts()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        ppo.train(adv, ret)
        torch.cuda.synchronize()
        dt = time.perf_counter() - t0
        print(f"iter {it}: update {dt * 1e3:.1f} ms = {dt * 1e6 / (10 * 128):.1f} us per minibatch", flush=True)
    env.close()


if __name__ == "__main__":
    main(int(sys.argv[1]) if len(sys.argv) > 1 else 3)

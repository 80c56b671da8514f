"""The reference's own training config on the GPU path: config.py's PPO kwargs (n_envs 8,
n_steps 2048, batch 256, 20 epochs, MLP[64,64] ReLU, lr 3e-4, ent_coef 0) -- the configs[0] shape a
user of the reference starts from.  Per PPO iteration (16 384 env steps): rollout_s and train_s,
synchronized; fp64 env.
    python tools/probes/gpu_reference_config.py [iterations]"""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
import torch  # noqa: E402

from mujocoposelearning_amd import ppo as P  # noqa: E402
from mujocoposelearning_amd.model import HsModel  # noqa: E402
from mujocoposelearning_amd.vec_env import HumanoidVecEnv  # noqa: E402

XML = os.path.join(ROOT, "mujocoposelearning_amd", "assets", "humanoid.xml")


def main():
    iters = int(sys.argv[1]) if len(sys.argv) > 1 else 3
    env = HumanoidVecEnv({"model_path": XML, "duration": 10.0, "frame_skip": 3, "reward_config": {"type": "stand"}},
                         n_envs=8, model=HsModel(XML), seed=0, precision="fp64")
    ppo = P.PPO(env, n_steps=2048, batch_size=256, n_epochs=20, learning_rate=3e-4, gamma=0.99, gae_lambda=0.95,
                clip_range=0.2, ent_coef=0.0, seed=0,
                policy_kwargs={"net_arch": {"pi": [64, 64], "vf": [64, 64]}, "activation_fn": "ReLU"})
    rows = []
    for it in range(iters):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        adv, ret = ppo.collect_rollouts()
        torch.cuda.synchronize()
        t1 = time.perf_counter()
        ppo.train(adv, ret)
        torch.cuda.synchronize()
        t2 = time.perf_counter()
        rows.append({"it": it, "rollout_s": t1 - t0, "train_s": t2 - t1,
                     "env_steps_per_s": 2048 * 8 / (t2 - t0)})
        print(json.dumps(rows[-1]), flush=True)
    env.close()


if __name__ == "__main__":
    main()

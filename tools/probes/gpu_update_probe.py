"""PPO update-phase probe: one rollout, then `reps` train() calls (16 minibatches each) of the
bench train-leg config; prints ms per minibatch.  Run under rocprofv3 --kernel-trace --stats to
get the per-minibatch kernel mix.  python tools/probes/gpu_update_probe.py [reps]"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
import torch  # noqa: E402

from mujocoposelearning_amd.model import HsModel  # noqa: E402
from mujocoposelearning_amd.ppo import PPO  # noqa: E402
from mujocoposelearning_amd.vec_env import HumanoidVecEnv  # noqa: E402

XML = os.path.join(ROOT, "mujocoposelearning_amd", "assets", "humanoid.xml")


def main(reps=5):
    env = HumanoidVecEnv({"model_path": XML, "duration": 10.0, "reward_config": {"type": "stand"}, "frame_skip": 3},
                         n_envs=4096, model=HsModel(XML), seed=0)
    ppo = PPO(env, n_steps=32, batch_size=32768, n_epochs=4, seed=0,
              policy_kwargs={"activation_fn": "ReLU", "net_arch": {"pi": [256, 256], "vf": [256, 256]}})
    adv, ret = ppo.collect_rollouts()
    ppo.train(adv, ret)
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(reps):
        ppo.train(adv, ret)
    torch.cuda.synchronize()
    mb = reps * 4 * (32 * 4096 // 32768)
    print(f"update: {1e3 * (time.perf_counter() - t) / mb:.3f} ms per minibatch ({mb + 16} minibatches run)",
          flush=True)
    env.close()


if __name__ == "__main__":
    main(int(sys.argv[1]) if len(sys.argv) > 1 else 5)

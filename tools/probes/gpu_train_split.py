"""Where a bench.py train-leg iteration goes: PPO.learn with the bench's train config (4096 fp64
envs, 32 steps, batch 32768, 4 epochs, MLP[256,256] ReLU), per iteration the logger's rollout_s
(collect_rollouts + warning check) and train_s (the update), synchronized.
    python tools/probes/gpu_train_split.py [iterations] [nochain]
(nochain: the nets' backward module by module, ppo_ops.FUSED_CHAIN off)"""
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
    iters = int(sys.argv[1]) if len(sys.argv) > 1 else 6
    if "nochain" in sys.argv[2:]:
        from mujocoposelearning_amd import ppo_ops
        ppo_ops.FUSED_CHAIN = False
    n = 4096
    env = HumanoidVecEnv({"model_path": XML, "duration": 10.0, "frame_skip": 3, "reward_config": {"type": "stand"}},
                         n_envs=n, model=HsModel(XML), seed=0, precision="fp64")
    ppo = P.PPO(env, n_steps=32, batch_size=32768, n_epochs=4, learning_rate=3e-4, seed=0,
                policy_kwargs={"net_arch": {"pi": [256, 256], "vf": [256, 256]}, "activation_fn": "ReLU"})
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
        rows.append({"it": it, "rollout_ms": (t1 - t0) * 1e3, "train_ms": (t2 - t1) * 1e3})
        print(json.dumps(rows[-1]), flush=True)
    r = rows[2:] or rows
    print(json.dumps({"mean_rollout_ms": sum(x["rollout_ms"] for x in r) / len(r),
                      "mean_train_ms": sum(x["train_ms"] for x in r) / len(r)}), flush=True)
    env.close()


if __name__ == "__main__":
    main()

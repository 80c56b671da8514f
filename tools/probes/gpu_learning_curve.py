"""Learning-curve sanity of the on-device PPO (SB3 is not importable, so the trainer
is judged by the stand reward rising).  bench.py's train config: 4096 envs, n_steps 32,
batch 32768, 4 epochs, lr 3e-4, MLP[256,256] ReLU (batch and epochs overridable).
python tools/probes/gpu_learning_curve.py [iters] [stand|kneeling] [fp32|fp64] [seed] [batch] [epochs] [stagger] [lr]
stagger = 1: spread the envs' episode clocks over the episode after the first reset (env i starts
i/N into it, as bench.py's window and the reference's 8 envs x 2048 steps per rollout do); without it
every env resets together and a 32-step rollout sees one phase of the episode."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
import numpy as np  # noqa: E402
import torch  # noqa: E402

from mujocoposelearning_amd.model import HsModel  # noqa: E402
from mujocoposelearning_amd.ppo import PPO  # noqa: E402
from mujocoposelearning_amd.vec_env import HumanoidVecEnv  # noqa: E402

XML = os.path.join(ROOT, "mujocoposelearning_amd", "assets", "humanoid.xml")


def main(iters=400, reward="stand", precision="fp32", seed=0, batch=32768, epochs=4, stagger=0, lr=3e-4):
    env = HumanoidVecEnv({"model_path": XML, "duration": 10.0, "reward_config": {"type": reward}, "frame_skip": 3},
                         n_envs=4096, model=HsModel(XML), seed=seed, precision=precision)
    ppo = PPO(env, n_steps=32, batch_size=batch, n_epochs=epochs, learning_rate=lr, seed=seed,
              policy_kwargs={"activation_fn": "ReLU", "net_arch": {"pi": [256, 256], "vf": [256, 256]}})
    if stagger:
        b, n, ep = env.batch, env.num_envs, 667
        kk = np.floor(np.arange(n) * ep / n)
        b.t["time"].copy_(torch.as_tensor(kk * 3 * 0.005 + 0.005, dtype=b.dtype, device=b.t["time"].device))
        b.t["step_count"].copy_(torch.as_tensor(kk, dtype=torch.int32, device=b.t["time"].device))
    t0 = time.perf_counter()
    rows = []
    for it in range(1, iters + 1):
        adv, ret = ppo.collect_rollouts()
        r_step = float(ppo.buf["rew"].mean())
        h = float(ppo.buf["obs"][..., 0].mean())          # obs[0] = qpos[2], the torso height
        st = ppo.train(adv, ret)
        if it % max(1, iters // 20) == 0 or it == 1:
            ep = float(np.mean(ppo.ep_returns[-200:])) if ppo.ep_returns else float("nan")
            rows.append((it, ppo.num_timesteps, r_step, h, ep, st["value_loss"], time.perf_counter() - t0))
            print(f"iter {it:4d} steps {ppo.num_timesteps / 1e6:6.1f}M  mean step reward {r_step:.4f}  "
                  f"mean height {h:.3f}  ep return (last 200) {ep:8.2f}  vf loss {st['value_loss']:.4f}  "
                  f"log_std {float(ppo.policy.log_std.detach().mean()):.3f}  fused {ppo._fused_rollout_args() is not None}  "
                  f"{time.perf_counter() - t0:6.1f}s", flush=True)
    env.close()
    return rows


if __name__ == "__main__":
    if os.environ.get("HS_NOCHAIN") == "1":   # A/B: the nets' backward module by module
        from mujocoposelearning_amd import ppo_ops
        ppo_ops.FUSED_CHAIN = False
    main(int(sys.argv[1]) if len(sys.argv) > 1 else 400, sys.argv[2] if len(sys.argv) > 2 else "stand",
         sys.argv[3] if len(sys.argv) > 3 else "fp32", int(sys.argv[4]) if len(sys.argv) > 4 else 0,
         int(sys.argv[5]) if len(sys.argv) > 5 else 32768, int(sys.argv[6]) if len(sys.argv) > 6 else 4,
         int(sys.argv[7]) if len(sys.argv) > 7 else 0, float(sys.argv[8]) if len(sys.argv) > 8 else 3e-4)

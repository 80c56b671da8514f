"""Learning curve under the reference's own PPO hyperparameters (README.md:23-53): lr 5e-5,
n_steps 2048 x 8 envs = 16 384 samples per rollout, batch 128, 10 epochs, gamma 0.99, lambda 0.95,
clip 0.2, ent_coef 0.002, MLP[256,256] ReLU, 'stand', frame_skip 3, duration 10 s
(train_sb3.py:183-200), 20 M env steps.  The 16 384 samples per rollout are spread over more envs
(``--envs`` x ``--n-steps``, default 128 x 128) so a run fits one GPU call; pass ``--envs 8
--n-steps 2048`` for the literal layout.  fp64 env (the reference's arithmetic).

python tools/probes/gpu_learning_curve_ref.py --seed 0 [--envs 128 --n-steps 128 --steps 20e6]
Prints one progress line per ``--every`` iterations: env steps, SB3's ep_rew_mean over the last 100
episodes (every stand episode runs 667 steps: termination is time >= duration, custom_env.py), the
fraction of the rollout's steps with the torso above 1.0 m ("upright") and the mean torso height."""
import argparse
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
import numpy as np  # noqa: E402
import torch  # noqa: E402

from mujocoposelearning_amd.model import HUMANOID_XML, HsModel  # noqa: E402
from mujocoposelearning_amd.ppo import PPO  # noqa: E402
from mujocoposelearning_amd.train import env_config_from_kwargs  # noqa: E402
from mujocoposelearning_amd.vec_env import HumanoidVecEnv  # noqa: E402

PPO_KWARGS = dict(learning_rate=5e-5, batch_size=128, n_epochs=10, gamma=0.99, gae_lambda=0.95, clip_range=0.2,
                  ent_coef=0.002, policy_kwargs={"activation_fn": "ReLU", "net_arch": {"pi": [256, 256], "vf": [256, 256]}})
# the reference's config.py (README.md:154 points to it for "the hyperparams"): 5 M steps
CONFIGPY_KWARGS = dict(learning_rate=3e-4, batch_size=256, n_epochs=20, gamma=0.99, gae_lambda=0.95, clip_range=0.2,
                       ent_coef=0.0, policy_kwargs={"activation_fn": "ReLU", "net_arch": {"pi": [64, 64], "vf": [64, 64]}})


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--seed", type=int, default=0)
    ap.add_argument("--envs", type=int, default=128)
    ap.add_argument("--n-steps", type=int, default=128)
    ap.add_argument("--steps", type=float, default=20e6)
    ap.add_argument("--precision", default="fp64")
    ap.add_argument("--reward", default="stand")
    ap.add_argument("--every", type=int, default=20)
    ap.add_argument("--config", default="readme", choices=("readme", "configpy"))
    ap.add_argument("--ent-coef", type=float, default=None, help="override the config's ent_coef (diagnosis runs)")
    ap.add_argument("--load", default=None, help="resume from a PPO.save zip (weights, Adam state, timesteps)")
    ap.add_argument("--save", default=None, help="PPO.save zip written at the end (resume with --load)")
    ap.add_argument("--stagger", action="store_true",
                    help="spread the envs' episode clocks over the episode (env i starts i/N into it, as bench.py's "
                         "window): every rollout then holds every phase of an episode, as the reference's 8 envs x "
                         "2048 steps (3 whole episodes per rollout) do; without it all envs reset together and a "
                         "128-step rollout sees one fifth of the episode")
    a = ap.parse_args()
    cfg = env_config_from_kwargs({"reward_function": a.reward, "frame_skip": 3}, HUMANOID_XML)
    env = HumanoidVecEnv(cfg, n_envs=a.envs, model=HsModel(HUMANOID_XML), seed=a.seed, precision=a.precision)
    env.batch.configure(aux=False, ctrl=False)
    kw = dict(PPO_KWARGS if a.config == "readme" else CONFIGPY_KWARGS)
    if a.ent_coef is not None:
        kw["ent_coef"] = a.ent_coef
    ppo = PPO(env, n_steps=a.n_steps, seed=a.seed, **kw)
    if a.load:
        ppo.load(a.load)
    if a.stagger:        # after PPO's reset: env i's episode clock at i/N of the 667-step episode
        k = np.floor(np.arange(a.envs) * 667 / a.envs)
        env.batch.t["time"].copy_(torch.as_tensor(k * 0.015 + 0.005, dtype=env.batch.dtype, device=env.device))
        env.batch.t["step_count"].copy_(torch.as_tensor(k, dtype=torch.int32, device=env.device))
    t0 = time.perf_counter()
    it = 0
    t_roll = t_train = 0.0
    while ppo.num_timesteps < a.steps:
        t1 = time.perf_counter()
        adv, ret = ppo.collect_rollouts()
        h = ppo.buf["obs"][..., 0]                     # obs[0] = qpos[2], the torso height
        upright = float((h > 1.0).float().mean())
        hmean = float(h.mean())
        t2 = time.perf_counter()
        st = ppo.train(adv, ret)
        torch.cuda.synchronize()
        t3 = time.perf_counter()
        t_roll += t2 - t1
        t_train += t3 - t2
        it += 1
        if it % a.every == 0 or ppo.num_timesteps >= a.steps:
            ep = float(np.mean(ppo.ep_returns[-100:])) if ppo.ep_returns else float("nan")
            print(f"seed {a.seed} iter {it:5d} steps {ppo.num_timesteps / 1e6:7.3f}M ep_rew_mean {ep:8.2f} "
                  f"episodes {len(ppo.ep_returns):6d} upright {upright:.3f} height {hmean:.3f} "
                  f"vf_loss {st['value_loss']:.3f} log_std {float(ppo.policy.log_std.mean()):.3f} "
                  f"rollout {t_roll / it:.3f}s train {t_train / it:.3f}s per iter {time.perf_counter() - t0:7.1f}s",
                  flush=True)
    if a.save:
        ppo.save(a.save)
    env.close()


if __name__ == "__main__":
    torch.backends.cuda.matmul.allow_tf32 = False
    main()

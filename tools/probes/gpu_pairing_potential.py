"""How much would pairing envs by predicted cost save?  A pair wave costs about the max of its two
envs (the loops run for the slower one).  On the bench window (4096 fp64 envs, staggered episode
clocks), record each env's Newton iterations and contact count of every env step (aux columns; the
last substep's), and compare, with cost proxy 1 + 0.15 * iterations per step:
  static   sum over pairs (2p, 2p+1) of max(cost)
  sorted   pairs formed by sorting envs on the PREVIOUS step's cost, sum of max(this step's cost)
  ideal    sum of cost / 2 (no max-of-two loss)
    python tools/probes/gpu_pairing_potential.py"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
import numpy as np  # noqa: E402
import torch  # noqa: E402

from mujocoposelearning_amd.model import HUMANOID_XML, HsModel  # noqa: E402
from mujocoposelearning_amd.vec_env import HumanoidVecEnv  # noqa: E402


def main():
    n, steps, EP = 4096, 120, 667
    env = HumanoidVecEnv({"model_path": HUMANOID_XML, "duration": 10.0, "frame_skip": 3,
                          "reward_config": {"type": "stand"}}, n_envs=n, model=HsModel(HUMANOID_XML), seed=0,
                         precision="fp64")
    b = env.batch
    b.configure(aux=True, ctrl=False)
    kk = np.floor(np.arange(n) * EP / n)
    b.t["time"].copy_(torch.as_tensor(kk * 3 * 0.005 + 0.005, dtype=b.dtype, device="cuda"))
    b.t["step_count"].copy_(torch.as_tensor(kk, dtype=torch.int32, device="cuda"))
    g = torch.Generator(device="cuda").manual_seed(0)
    for _ in range(EP):   # one untimed episode: the window's mix
        env.step_tensors(torch.rand(n, 21, device="cuda", generator=g) * 2 - 1)
    its, con = [], []
    for _ in range(steps):
        env.step_tensors(torch.rand(n, 21, device="cuda", generator=g) * 2 - 1)
        ax = b.aux.double()
        its.append(ax[:, 37].cpu().numpy())
        con.append(ax[:, 35].cpu().numpy())
    its, con = np.array(its), np.array(con)
    cost = 1 + 0.15 * its
    static = sum(np.maximum(c[0::2], c[1::2]).sum() for c in cost)
    sorted_ = 0.0
    for t in range(1, steps):
        o = np.argsort(cost[t - 1])
        c = cost[t][o]
        sorted_ += np.maximum(c[0::2], c[1::2]).sum()
    sorted_ *= steps / (steps - 1)
    ideal = cost.sum() / 2
    corr = np.corrcoef(cost[:-1].ravel(), cost[1:].ravel())[0, 1]
    print(json.dumps({"steps": steps, "mean_iters": float(its.mean()), "mean_contacts": float(con.mean()),
                      "static_over_ideal": static / ideal, "sorted_over_ideal": sorted_ / ideal,
                      "step_to_step_corr": float(corr)}), flush=True)
    env.close()


if __name__ == "__main__":
    main()

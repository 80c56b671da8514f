"""Cost of the fused rollout's in-kernel policy: the same 4096-env fp64 batch state (staggered
clocks, one untimed episode) stepped 32 env steps (a) as one open-loop tape launch, (b) as one fused
rollout (hs_rollout: policy forward + sampling + bookkeeping per step), (c) per step with the policy
GEMM path (the per-step graph of collect_rollouts).  python tools/probes/gpu_rollout_cost.py"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
import numpy as np  # noqa: E402
import torch  # noqa: E402

from mujocoposelearning_amd import ppo as ppo_mod  # noqa: E402
from mujocoposelearning_amd.model import HUMANOID_XML, HsModel  # noqa: E402
from mujocoposelearning_amd.vec_env import HumanoidVecEnv  # noqa: E402

N, T, REPS = 4096, 32, 5


def make(model):
    env = HumanoidVecEnv({"model_path": HUMANOID_XML, "duration": 10.0, "reward_config": {"type": "stand"},
                          "frame_skip": 3}, n_envs=N, model=model, seed=0, precision="fp64")
    env.batch.configure(aux=False, ctrl=False)
    p = ppo_mod.PPO(env, n_steps=T, batch_size=32768, n_epochs=1, seed=0,
                    policy_kwargs={"net_arch": {"pi": [256, 256], "vf": [256, 256]}, "activation_fn": "ReLU"})
    k = np.floor(np.arange(N) * 667 / N)
    env.batch.t["time"].copy_(torch.as_tensor(k * 0.015 + 0.005, dtype=torch.float64, device="cuda"))
    env.batch.t["step_count"].copy_(torch.as_tensor(k, dtype=torch.int32, device="cuda"))
    return env, p


def timeit(fn):
    torch.cuda.synchronize()
    ts = []
    for _ in range(REPS):
        t0 = time.perf_counter()
        fn()
        torch.cuda.synchronize()
        ts.append(time.perf_counter() - t0)
    return np.median(ts) * 1e3


def main():
    model = HsModel(HUMANOID_XML)
    env, p = make(model)
    g = torch.Generator(device="cuda").manual_seed(1)
    tape = (torch.rand(667 + T, N, 21, device="cuda", generator=g) * 2 - 1)
    for k in range(667):                                      # one untimed episode: the staggered mix
        env.step_tensors(tape[k])
    p.obs.copy_(env.batch.obs.float())
    p.policy.pack_heads()
    ms_tape = timeit(lambda: env.batch.step_tape(tape[667:667 + T], outputs=False))
    ms_fused = timeit(p._rollout_fused)
    ms_collect_f = timeit(p.collect_rollouts)
    ppo_mod.FUSED_ROLLOUT = False
    p.collect_rollouts()                                      # graph capture
    ms_collect_s = timeit(p.collect_rollouts)
    ms_body = timeit(p._rollout_body)
    print(f"32 env steps of 4096 fp64 envs (ms): tape {ms_tape:.2f} ({ms_tape / T:.3f}/step); fused rollout "
          f"{ms_fused:.2f} ({ms_fused / T:.3f}/step); per-step rollout body (eager, no graph) {ms_body:.2f}; "
          f"collect_rollouts fused {ms_collect_f:.2f} / per-step graph {ms_collect_s:.2f}", flush=True)


if __name__ == "__main__":
    main()

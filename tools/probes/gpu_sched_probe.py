"""GPU probe (not a test): sim-only env steps/s of one batch under each step-kernel schedule
("single": one env per wave, "direct": one wave per env pair, "auto"), on bench.py's staggered
whole-episode window.  Default: configs[4]'s per-GPU shard (1024 envs, full-state obs) in fp64.

    python tools/probes/gpu_sched_probe.py [--envs 1024] [--precision fp64] [--full-state 1] [--steps 50]
"""
import argparse
import json
import math
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
XML = os.path.join(ROOT, "mujocoposelearning_amd", "assets", "humanoid.xml")
EPISODE = math.ceil(10.0 / 0.015 - 1e-9)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--envs", type=int, nargs="+", default=[1024])
    ap.add_argument("--precision", default="fp64")
    ap.add_argument("--full-state", type=int, default=1)
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--schedules", nargs="+", default=["single", "direct"])
    a = ap.parse_args()
    import torch
    from mujocoposelearning_amd.model import HsModel
    from mujocoposelearning_amd.vec_env import HumanoidVecEnv
    model = HsModel(XML)
    for n in a.envs:
        g = torch.Generator(device="cuda").manual_seed(1)
        tape = torch.rand(1024, n, 21, device="cuda", generator=g) * 2 - 1
        for sched in a.schedules:
            cfg = {"model_path": XML, "duration": 10.0, "reward_config": {"type": "stand"}, "frame_skip": 3,
                   "full_state_obs": bool(a.full_state)}
            e = HumanoidVecEnv(cfg, n_envs=n, precision=a.precision, seed=4000, model=model)
            e.batch.configure(aux=False, ctrl=False, schedule=sched)
            e.reset_tensors()
            t0 = np.floor(np.arange(n) * EPISODE / n) * 0.015 + 0.005
            e.batch.set_state(time=t0)
            for k in range(EPISODE + 10):
                e.step_tensors(tape[k % 1024])
            torch.cuda.synchronize()
            ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            t = time.perf_counter()
            ev0.record()
            for k in range(a.steps):
                e.step_tensors(tape[(EPISODE + 10 + k) % 1024])
            ev1.record()
            torch.cuda.synchronize()
            dt = time.perf_counter() - t
            print(json.dumps({"n_envs": n, "precision": a.precision, "full_state": bool(a.full_state),
                              "schedule": sched, "ran": e.batch.schedule_name(),
                              "env_steps_per_s": n * a.steps / dt, "ms_per_launch": ev0.elapsed_time(ev1) / a.steps,
                              "warnings": e.batch.warning.sum(0).tolist()}), flush=True)
            e.close()


if __name__ == "__main__":
    main()

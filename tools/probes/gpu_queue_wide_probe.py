"""Probe (not a test): tests/test_gpu_queue.py's queue-vs-direct scenario (fp64, 4096 envs, 16 lying
envs), repeated in one process; reports which run is inconsistent (obs[0:26] vs the committed qpos[2:])
and how runs differ."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
XML = os.path.join(ROOT, "mujocoposelearning_amd", "assets", "humanoid.xml")


def main():
    import torch
    from mujocoposelearning_amd.batch import HsBatch
    from mujocoposelearning_amd.model import HsModel
    from oracle.oracle import Oracle
    from test_gpu_contacts import lying_states
    model = HsModel(XML)
    n = 4096
    lying = np.stack(lying_states(Oracle(XML), 16, seed=11))
    idx = np.arange(16) * 255 + 7
    g = torch.Generator(device="cuda").manual_seed(5)
    acts = torch.rand(4, n, 21, device="cuda", generator=g) * 2 - 1
    runs = []
    sync = os.environ.get("PROBE_SYNC") == "1"
    for sched in ("auto", "direct", "direct", "auto", "auto", "direct"):
        b = HsBatch(model, n, precision="fp64", seed=3)
        b.configure(frame_skip=3, duration=10.0, reward_id=0, autoreset=1, max_steps=750, schedule=sched)
        b.reset()
        st = b.get_state()
        st["qpos"][idx] = lying
        st["qvel"][idx] = 0.0
        st["qacc_warmstart"][idx] = 0.0
        b.set_state(**st)
        b.step(acts[0])
        if sync:
            torch.cuda.synchronize()
        obs0, q0 = b.obs.clone(), b.qpos.clone()
        if sync:
            torch.cuda.synchronize()
        ocpu = b.obs.cpu().numpy()          # read again after the clone (host copy, synchronous)
        for k in range(1, 4):
            b.step(acts[k])
        torch.cuda.synchronize()
        o, q = obs0.cpu().numpy(), q0.cpu().numpy()
        incons = np.flatnonzero(np.abs(o[:, :26] - q[:, 2:]).max(1) > 0)
        if incons.size:
            again = np.abs(ocpu[incons, :26] - q[incons, 2:]).max(1)
            print(f"   re-read of obs after the clone: {int((again > 0).sum())} of {incons.size} still inconsistent", flush=True)
        runs.append((sched, o, q))
        print(f"{sched}: obs[0:26] != committed qpos[2:] for {incons.size} envs {incons[:12].tolist()}", flush=True)
        b.close()
    for i, (sched, o, q) in enumerate(runs[1:], 1):
        do = np.flatnonzero(np.abs(o - runs[0][1]).max(1) > 0)
        dq = np.flatnonzero(np.abs(q - runs[0][2]).max(1) > 0)
        print(f"run {i} ({sched}) vs run 0 (auto): obs differ {do.size}, qpos differ {dq.size}")


if __name__ == "__main__":
    main()

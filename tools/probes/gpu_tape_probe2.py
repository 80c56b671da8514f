"""Tape launch diagnosis: determinism (tape vs tape) and the first differing step / obs components
against the step loop, fp64, small batches.  python tools/probes/gpu_tape_probe2.py"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
import numpy as np  # noqa: E402
import torch  # noqa: E402

from mujocoposelearning_amd.batch import HsBatch  # noqa: E402
from mujocoposelearning_amd.model import HUMANOID_XML, HsModel  # noqa: E402


def run(model, n, acts, t0, mode, pre="auto"):
    b = HsBatch(model, n, precision="fp64", seed=3)
    b.configure(frame_skip=3, duration=10.0, reward_id=0, autoreset=1, max_steps=750, schedule=pre)
    b.reset()
    b.set_state(time=t0)
    b.step(acts[0])
    b.configure(schedule="auto")
    K = acts.shape[0] - 1
    if mode == "tape":
        obs = b.step_tape(acts[1:])[0].clone()
    elif mode == "tape_split":       # two tape launches of K/2
        o1 = b.step_tape(acts[1:1 + K // 2])[0].clone()
        o2 = b.step_tape(acts[1 + K // 2:])[0].clone()
        obs = torch.cat([o1, o2])
    else:
        o = []
        for k in range(K):
            b.step(acts[1 + k])
            o.append(b.obs.clone())
        obs = torch.stack(o)
    w = b.warning.sum(0).tolist()
    b.close()
    return obs, w


def cmp(name, a, b):
    d = (a - b).abs().amax(2)
    bad = torch.nonzero(d > 0)
    if bad.numel() == 0:
        print(f"{name}: bitwise equal", flush=True)
        return
    t = int(bad[0, 0])
    envs = torch.nonzero(d[t] > 0).flatten().tolist()
    e = envs[0]
    comp = torch.nonzero((a[t, e] - b[t, e]).abs() > 0).flatten().tolist()
    print(f"{name}: first diff step {t}, envs {envs[:8]}, env {e} components {comp[:12]} (of {a.shape[2]}), "
          f"max {float(d[t].max()):.3e}; prev-step max diff {float(d[t - 1].max()) if t else 0:.1e}", flush=True)


def main():
    model = HsModel(HUMANOID_XML)
    for n in (1024, 777):
        K = 40
        g = torch.Generator(device="cuda").manual_seed(21)
        acts = torch.rand(K + 1, n, 21, device="cuda", generator=g) * 2 - 1
        t0 = np.floor(np.arange(n) * 667 / n) * 0.015 + 0.005
        loop, wl = run(model, n, acts, t0, "loop")
        tape1, w1 = run(model, n, acts, t0, "tape")
        tape2, w2 = run(model, n, acts, t0, "tape")
        tape3, w3 = run(model, n, acts, t0, "tape", pre="direct")
        split, w4 = run(model, n, acts, t0, "tape_split")
        print(f"n {n}: warnings loop {wl} tape {w1} {w2} {w3} split {w4}", flush=True)
        cmp(f"n {n} tape vs tape", tape1, tape2)
        cmp(f"n {n} tape vs loop", tape1, loop)
        cmp(f"n {n} tape(pre-step paired) vs loop", tape3, loop)
        cmp(f"n {n} split tape vs loop", split, loop)


if __name__ == "__main__":
    main()

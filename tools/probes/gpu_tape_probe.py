"""Tape launch vs step loop: first differing (step, env) per case, and warnings (lost hand-offs show
as HS_WARN_BADQPOS).  python tools/probes/gpu_tape_probe.py"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
import numpy as np  # noqa: E402
import torch  # noqa: E402

from mujocoposelearning_amd.batch import HsBatch  # noqa: E402
from mujocoposelearning_amd.model import HUMANOID_XML, HsModel  # noqa: E402


def run(model, n, prec, acts, t0, tape, sched="auto"):
    b = HsBatch(model, n, precision=prec, seed=3)
    b.configure(frame_skip=3, duration=10.0, reward_id=0, autoreset=1, max_steps=750, schedule=sched)
    b.reset()
    b.set_state(time=t0)
    b.step(acts[0])
    K = acts.shape[0] - 1
    if tape:
        obs = b.step_tape(acts[1:])[0].clone()
    else:
        o = []
        for k in range(K):
            b.step(acts[1 + k])
            o.append(b.obs.clone())
        obs = torch.stack(o)
    w = b.warning.sum(0).tolist()
    st = b.step_count.clone()
    b.close()
    return obs, w, st


def main():
    model = HsModel(HUMANOID_XML)
    for n, prec, sched in [(777, "fp64", "auto"), (777, "fp64", "direct"), (778, "fp64", "auto"), (1024, "fp64", "auto"),
                           (2048, "fp64", "auto"), (777, "fp32", "auto")]:
        K = 40
        g = torch.Generator(device="cuda").manual_seed(21)
        acts = torch.rand(K + 1, n, 21, device="cuda", generator=g) * 2 - 1
        t0 = np.floor(np.arange(n) * 667 / n) * 0.015 + 0.005
        oa, wa, sa = run(model, n, prec, acts, t0, True, sched)
        ob, wb, sb = run(model, n, prec, acts, t0, False, sched)
        d = (oa.double() - ob.double()).abs().amax(2)        # [K, n]
        bad = torch.nonzero(d > 0)
        msg = f"n {n} {prec} {sched}: warnings tape {wa} loop {wb}; "
        if bad.numel() == 0:
            msg += "bitwise equal"
        else:
            first = bad[0].tolist()
            envs = torch.unique(bad[:, 1]).tolist()
            msg += (f"{len(envs)} envs differ (first step {first[0]} env {first[1]}; envs {envs[:12]}); "
                    f"step_count tape {sa[envs[:6]].tolist()} loop {sb[envs[:6]].tolist()}; t0 {t0[envs[:6]].round(3).tolist()}")
        print(msg, flush=True)


if __name__ == "__main__":
    main()

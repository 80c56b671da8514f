"""1000-substep parity report (SURVEY.md 8d "Parity run"): max |dqpos| / |dqvel| per checkpoint of
the GPU engine (fp64 and fp32) against the fp64 oracle on the same state and action tape, next to
the CHAOS ENVELOPE -- the oracle against itself with the initial qvel perturbed by 1e-15
(relative), i.e. what any two correct fp64 implementations that round differently do.

Run on the GPU box:  python tests/parity_report.py > profiles/parity_report.md
"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402

from mujocoposelearning_amd.batch import HsBatch  # noqa: E402
from mujocoposelearning_amd.model import HsModel  # noqa: E402
from oracle.oracle import Oracle  # noqa: E402

XML = os.path.join(ROOT, "mujocoposelearning_amd", "assets", "humanoid.xml")
NSUB, EVERY = 1000, 100


def initial(o, seed):
    rng = np.random.default_rng(seed)
    q = o.M["qpos0"].copy()
    q[2] = 1.282
    q[3:7] = [1, 0, 0, 0]
    q += rng.uniform(-0.01, 0.01, 28) * np.r_[1, 1, 0.1, 0, 0, 0, 0, np.ones(21)]
    return q, rng.uniform(-0.01, 0.01, 27), rng


def run_oracle(q, v, tape, perturb=0.0):
    o = Oracle(XML)
    o.qpos[:] = q
    o.qvel[:] = v * (1 + perturb)
    out = []
    for s in range(NSUB):
        o.step(tape[s].astype(np.float64), 1)
        if (s + 1) % EVERY == 0:
            out.append((o.qpos.copy(), o.qvel.copy()))
    return out


def run_gpu(model, prec, q, v, tape):
    b = HsBatch(model, 1, precision=prec)
    b.set_state(qpos=q, qvel=v, time=0.0, qacc_warmstart=0.0)
    c = torch.tensor(tape, device=b.device)
    out = []
    for s in range(NSUB):
        b.physics_step(c[s:s + 1], 1)
        if (s + 1) % EVERY == 0:
            st = b.get_state()
            out.append((st["qpos"][0].copy(), st["qvel"][0].copy()))
    return out


def fmt(a, b):
    return f"{np.abs(a[0] - b[0]).max():.1e} / {np.abs(a[1] - b[1]).max():.1e}"


def main():
    model = HsModel(XML)
    print("# 1000-substep parity report (GPU engine vs fp64 oracle, same state + action tape)\n")
    print("Cells: max |dqpos| / max |dqvel| after the given number of substeps (h = 5 ms).  "
          "'chaos envelope' = oracle vs oracle with qvel perturbed by 1e-15 (relative): the "
          "divergence any two correct fp64 implementations that round differently show.\n")
    for tape_name in ("zeros", "uniform"):
        for seed in (0, 1):
            o = Oracle(XML)
            q, v, rng = initial(o, seed)
            tape = (np.zeros((NSUB, 21)) if tape_name == "zeros" else rng.uniform(-1, 1, (NSUB, 21))).astype(np.float32)
            ref = run_oracle(q, v, tape)
            env = run_oracle(q, v, tape, perturb=1e-15)
            g64 = run_gpu(model, "fp64", q, v, tape)
            g32 = run_gpu(model, "fp32", q, v, tape)
            print(f"## tape = {tape_name}, seed {seed}\n")
            print("| substeps | chaos envelope (fp64 oracle, 1e-15 perturbation) | GPU fp64 | GPU fp32 |")
            print("|---|---|---|---|")
            for k in range(len(ref)):
                print(f"| {(k + 1) * EVERY} | {fmt(env[k], ref[k])} | {fmt(g64[k], ref[k])} | {fmt(g32[k], ref[k])} |")
            print()


if __name__ == "__main__":
    main()

"""Contact pile-up states for tests/test_gpu_contacts.py (our own data, made with the oracle).

Prone / supine / on-the-side humanoids pushed into the floor with their joints at random points or
at their range limits (limbs folded under the torso), searched for the most contacts: the worst
cases reach ~60 contacts / ~160 constraint rows (floor + body-body), close to the wide kernel tier
(64 / 256) -- far past anything a rollout produces (14 / 52 over 48 oracle episodes, hs_model.h).
Run: python tests/golden/make_pileup_states.py  ->  tests/golden/pileup_states.npz
"""
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)
XML = os.path.join(ROOT, "mujocoposelearning_amd", "assets", "humanoid.xml")


def _qaxis(axis, ang):
    axis = np.asarray(axis, float) / np.linalg.norm(axis)
    return np.r_[np.cos(ang / 2), np.sin(ang / 2) * axis]


def _qmul(a, b):
    return np.r_[a[0] * b[0] - a[1:] @ b[1:], a[0] * b[1:] + b[0] * a[1:] + np.cross(a[1:], b[1:])]


def search(n_keep=8, iters=30000, seed=0):
    from oracle.oracle import Oracle
    o = Oracle(XML)
    M = o.M
    lo, hi = M["jnt_range"][1:, 0], M["jnt_range"][1:, 1]
    rng = np.random.default_rng(seed)
    found = []
    for _ in range(iters):
        q = M["qpos0"].copy()
        q[3:7] = _qmul(_qaxis([0, 0, 1], rng.uniform(-np.pi, np.pi)),
                       _qmul(_qaxis([0, 1, 0], np.pi / 2 * rng.choice([-1, 1])), _qaxis([1, 0, 0], rng.uniform(-np.pi, np.pi))))
        mode = rng.integers(3)
        if mode == 0:
            q[7:] = np.clip(rng.uniform(0, 0.3) * rng.normal(size=21), lo, hi)
        elif mode == 1:
            q[7:] = np.where(rng.uniform(size=21) < 0.5, lo, hi)      # limbs folded to their limits
        else:
            q[7:] = rng.uniform(lo, hi)
        q[2] = rng.uniform(-0.05, 0.2)
        o.reset_data()
        o.qpos[:] = q
        o.forward()
        nbb = sum(1 for c in o.contacts() if 0 not in c["geom"])
        found.append((o.d.ncon, o.d.nefc, nbb, q))
    found.sort(key=lambda r: (r[0], r[1]), reverse=True)
    top = found[:n_keep]
    return np.stack([r[3] for r in top]), np.array([[r[0], r[1], r[2]] for r in top])


if __name__ == "__main__":
    qpos, counts = search()
    out = os.path.join(HERE, "pileup_states.npz")
    np.savez(out, qpos=qpos, counts=counts)
    print(f"wrote {out}: (ncon, nefc, body-body contacts) = {counts.tolist()}")

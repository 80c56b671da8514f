"""Analysis tool (not a test, not product): how much of the fp64 chunk-queue launch is lost to the
lockstep of the two envs of a wave, and how much of it a cost-sorted pairing could recover.

Runs the fp64 oracle (checker build) on N envs whose clocks are staggered over the episode as in
bench.py's window, then records per env and substep the Newton iteration count and the row count
over `--steps` consecutive env steps.  A wave runs every substep of its two envs in lockstep, so
its Newton work is sum over substeps of max(it_a, it_b) (and likewise for loops over rows).  We
compare the fixed pairing (2p, 2p+1) with pairings sorted by the previous step's per-env cost.

    python tools/pairing_stats.py [--envs 256] [--steps 12] [--procs 8]
"""
import argparse
import math
import os
import sys
from multiprocessing import Pool

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
XML = os.path.join(ROOT, "mujocoposelearning_amd", "assets", "humanoid.xml")
EPISODE = math.ceil(10.0 / 0.015 - 1e-9)


def run_env(args):
    i, n, steps, fs = args
    from oracle.env import OracleHumanoidEnv
    rng = np.random.default_rng(1000 + i)
    e = OracleHumanoidEnv({"model_path": XML, "duration": 10.0, "reward_config": {"type": "stand"},
                           "frame_skip": fs})
    e.reset(seed=i)
    pre = int(i * EPISODE / n)
    for _ in range(pre):
        e.step(rng.uniform(-1, 1, 21))
    it = np.zeros((steps, fs), np.int32)
    nefc = np.zeros((steps, fs), np.int32)
    for k in range(steps):
        a = rng.uniform(-1, 1, 21)
        for s in range(fs):
            e.sim.step(a, 1)
            it[k, s] = e.sim.d.solver_niter
            nefc[k, s] = e.sim.d.nefc
    return it, nefc


def lockstep_cost(it, nefc, order, w_it=1.0, w_row=0.0):
    """sum over waves of the lockstep cost of one step (it/nefc: [N, fs]) with envs paired as
    order[0::2], order[1::2]"""
    a, b = order[0::2], order[1::2]
    c = np.maximum(it[a], it[b]) * w_it + np.maximum(nefc[a], nefc[b]) * w_row
    return c.sum()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--envs", type=int, default=256)
    ap.add_argument("--steps", type=int, default=12)
    ap.add_argument("--procs", type=int, default=8)
    a = ap.parse_args()
    n, fs = a.envs, 3
    with Pool(a.procs) as p:
        res = p.map(run_env, [(i, n, a.steps, fs) for i in range(n)])
    it = np.stack([r[0] for r in res], 1)       # [steps, N, fs]
    nefc = np.stack([r[1] for r in res], 1)
    tot = it.sum(2)                              # [steps, N]
    c = [np.corrcoef(tot[k], tot[k + 1])[0, 1] for k in range(a.steps - 1)]
    print(f"per-env Newton iterations per env step: mean {tot.mean():.2f}, sd {tot.std():.2f}; "
          f"step-to-step corr {np.mean(c):.2f}")
    rows = nefc.sum(2)
    cr = [np.corrcoef(rows[k], rows[k + 1])[0, 1] for k in range(a.steps - 1)]
    print(f"per-env rows per env step: mean {rows.mean():.1f}; step-to-step corr {np.mean(cr):.2f}")
    for w_it, w_row, name in [(1, 0, "newton iterations"), (0, 1, "rows"), (1, 0.25, "iters + rows/4")]:
        fixed, prev_sorted, ideal, half = [], [], [], []
        for k in range(1, a.steps):
            ident = np.arange(n)
            fixed.append(lockstep_cost(it[k], nefc[k], ident, w_it, w_row))
            key = tot[k - 1] * w_it + rows[k - 1] * w_row
            prev_sorted.append(lockstep_cost(it[k], nefc[k], np.argsort(key, kind="stable"), w_it, w_row))
            keyc = tot[k] * w_it + rows[k] * w_row
            ideal.append(lockstep_cost(it[k], nefc[k], np.argsort(keyc, kind="stable"), w_it, w_row))
            half.append((it[k] * w_it + nefc[k] * w_row).sum() / 2)
        f = np.sum(fixed)
        print(f"[{name}] lockstep work, fixed pairs = 1: sorted by previous step {np.sum(prev_sorted) / f:.3f}, "
              f"sorted by this step (oracle) {np.sum(ideal) / f:.3f}, no lockstep loss {np.sum(half) / f:.3f}")


if __name__ == "__main__":
    main()

"""CPU probe (not a test): how many constraint rows change their active state between consecutive
Newton factorizations, per env pair, on the bench's staggered whole-episode mix -- the input to
the incremental-factor question (MuJoCo's Newton updates its Cholesky factor by
rank-1 updates / downdates for the rows that changed state instead of rebuilding it).

For each oracle substep it replays the kernel's Newton iteration (hs_kernels.hip Stepper::solve:
warm start, exact line search, done when no row changes state at alpha ~ 1 or the scaled gradient is
below tolerance) on the substep's own constraint data (efc_J / efc_D / efc_aref / qM / qacc_smooth,
which the oracle leaves in OrcData), and records, for iterations after the first, the number of
rows whose active flag differs from the set the previous factorization used.  Envs are paired as
on the GPU (a wave runs max over its two envs), and the result is printed as a histogram plus the
projected per-substep Hessian + factorization cost of both strategies from measured cycle counts.

    python tools/probes/newton_update_stats.py [--envs 64] [--steps 200] [--seed 0]
"""
import argparse
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
XML = os.path.join(ROOT, "mujocoposelearning_amd", "assets", "humanoid.xml")


def newton_changes(o, x0, tol, maxit=100):
    """Kernel-rule Newton from x0 on the oracle's current constraint data; returns the per-iteration
    changed-row counts (relative to the previous factorization's active set), one entry per
    factorization after the first."""
    nv, ne = o.M["nv"], o.d.nefc
    M = o.get("qM")
    a0 = o.arr("qacc_smooth", nv).copy() if hasattr(o.d, "qacc_smooth") else None
    J = np.ctypeslib.as_array(o.d.efc_J)[:ne, :nv].copy()
    D = np.ctypeslib.as_array(o.d.efc_D)[:ne].copy()
    ar = np.ctypeslib.as_array(o.d.efc_aref)[:ne].copy()
    scale = 1.0 / (o.M["stat_meaninertia"] * nv)
    x = x0.copy()
    fs = M @ a0
    jar = J @ x - ar
    prev = None
    changes = []
    for it in range(maxit):
        act = jar < 0
        g = M @ x - fs + J.T @ (np.where(act, D * jar, 0.0))
        if scale * scale * (g @ g) < tol * tol:
            break
        if prev is not None:
            changes.append(int(np.sum(act != prev)))
        prev = act.copy()
        H = M + (J[act].T * D[act]) @ J[act]
        s = -np.linalg.solve(H, g)
        Js = J @ s
        Ms = M @ s
        A0, B0 = s @ Ms, s @ (M @ x - fs)
        # exact minimiser along s (piecewise quadratic): breakpoint walk
        bp = np.sort([t for t in (-jar[Js != 0] / Js[Js != 0]) if t > 0])
        lo, alpha = 0.0, 0.0
        for k in range(len(bp) + 1):
            hi = bp[k] if k < len(bp) else np.inf
            mid = 0.5 * (lo + hi) if k < len(bp) else lo + 1.0
            a = (jar + mid * Js) < 0
            A = A0 + np.sum(D[a] * Js[a] ** 2)
            B = B0 + np.sum(D[a] * jar[a] * Js[a])
            root = -B / A
            if root <= hi:
                alpha = max(root, lo)
                break
            lo = hi
            alpha = lo
        x = x + alpha * s
        nj = jar + alpha * Js
        changed = np.any((nj < 0) != act)
        jar = nj
        if not changed and abs(alpha - 1) < 1e-3:
            break
    return changes


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--envs", type=int, default=64)
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--seed", type=int, default=0)
    ap.add_argument("--chol", type=float, default=13.5e3, help="cycles per full factorization (r3l timing)")
    ap.add_argument("--hess", type=float, default=9.2e3, help="cycles per Hessian build (r3l timing)")
    ap.add_argument("--r1", type=float, default=None, help="cycles per rank-1 update (GPU probe)")
    a = ap.parse_args()
    from oracle.oracle import Oracle
    rng = np.random.default_rng(a.seed)
    o = Oracle(XML)
    tol = float(o.M["opt_tolerance"])
    nv = o.M["nv"]
    episode = 667
    per_env = []      # per env: list over substeps of change lists
    for e in range(a.envs):
        o.reset_data()
        q = o.qpos
        q[:] = o.M["qpos0"]
        q[2] = 1.282
        q[7:] += rng.uniform(-0.01, 0.01, nv - 6)
        # staggered: skip ahead a random part of an episode so fallen states are represented
        warm = int(rng.integers(0, episode - a.steps))
        for _ in range(warm):
            o.step(rng.uniform(-1, 1, 21), 3)
        subs = []
        for _ in range(a.steps):
            act = rng.uniform(-1, 1, 21)
            for _s in range(3):
                ws = o.arr("qacc_warmstart", nv).copy()
                o.step(act, 1)
                subs.append(newton_changes(o, ws, tol))
        per_env.append(subs)
    # pair envs (2k, 2k+1): per substep, the wave runs max(iterations); per iteration max(changes)
    full, inc, hist = [], [], {}
    for k in range(0, a.envs - 1, 2):
        for c0, c1 in zip(per_env[k], per_env[k + 1]):
            nf = max(len(c0), len(c1)) + (1 if (c0 or c1) else 0)   # factorizations of the wave
            n = max(len(c0), len(c1))
            ch = [max(c0[i] if i < len(c0) else 0, c1[i] if i < len(c1) else 0) for i in range(n)]
            for c in ch:
                hist[c] = hist.get(c, 0) + 1
            full.append(nf)
            inc.append(ch)
    nsub = len(full)
    tot_fact = sum(full)
    later = [c for ch in inc for c in ch]
    out = {"pairs": a.envs // 2, "substeps": nsub, "factorizations_per_substep": tot_fact / nsub,
           "later_factorizations_per_substep": len(later) / nsub,
           "changed_rows_hist": dict(sorted(hist.items())),
           "changed_rows_mean": float(np.mean(later)) if later else 0.0,
           "changed_rows_p50": float(np.percentile(later, 50)) if later else 0.0,
           "changed_rows_p90": float(np.percentile(later, 90)) if later else 0.0}
    if a.r1:
        cost_full = tot_fact * (a.chol + a.hess) / nsub
        cost_inc = (tot_fact - len(later)) * (a.chol + a.hess) / nsub + sum(later) * a.r1 / nsub
        out.update({"cycles_full_per_substep": cost_full, "cycles_incremental_per_substep": cost_inc})
    print(json.dumps(out))


if __name__ == "__main__":
    main()

"""Global fit of the unrecorded controls of the reference's MuJoCo rollout, on the GPU.

For each key interval of tests/golden/humanoid_trajectory.xml (25 substeps: 5 env steps of
frame_skip 5, each with one constant control vector in [-1, 1]; oracle/trajfit.py has the setup),
a CMA-ES over the 105 controls evaluates POP candidate tapes per generation as POP envs of one fp64
HsBatch (every env starts from the key; 5 physics_step launches of 5 substeps), then a box-clipped
Gauss-Newton polish with finite-difference Jacobians (106 envs per Jacobian).  The objective is
the miss of the next key in half-quanta of its 6-decimal printing (5e-7).  The best controls are
re-evaluated by the fp64 oracle (CPU), which is what the report quotes.

Model variants that are XML edits run the same way: ``armature_zero`` (every joint armature 0) and
``friction_07`` (floor friction 0.7 = the min-mixed floor-vs-body friction).  ``--synthetic``
replaces each recorded end key by the oracle's own end state from known controls (rounded to 6
decimals): the fit must recover it, which shows the search reaches the basin.

python tools/probes/gpu_trajfit.py [--intervals 3,10,...] [--variants truth,armature_zero] [--pop 4096]
Prints markdown; per-interval progress to stderr.
"""
import argparse
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
import torch  # noqa: E402

from mujocoposelearning_amd.batch import HsBatch  # noqa: E402
from mujocoposelearning_amd.model import HUMANOID_XML, HsModel  # noqa: E402
from oracle import trajfit as T  # noqa: E402

KEYS = os.path.join(ROOT, "tests", "golden", "humanoid_trajectory.xml")
K, NU, FS = T.STEPS_PER_KEY, 21, T.FRAME_SKIP


class GpuShooter:
    """POP control tapes from one start state, 25 substeps, fp64 GPU engine."""

    def __init__(self, model, pop):
        self.b = HsBatch(model, pop, precision="fp64")
        self.b.configure(aux=False)
        self.pop = pop

    def final(self, q0, v0, X):
        """X [n, 105] float32 (n <= pop) -> end states [n, 55] (fp64, device)."""
        b, n = self.b, X.shape[0]
        b.t["qpos"].copy_(torch.as_tensor(q0, dtype=torch.float64, device=b.device).expand(self.pop, -1))
        b.t["qvel"].copy_(torch.as_tensor(v0, dtype=torch.float64, device=b.device).expand(self.pop, -1))
        b.t["qacc_warmstart"].zero_()
        b.t["time"].zero_()
        Xf = torch.zeros(self.pop, K * NU, dtype=torch.float32, device=b.device)
        Xf[:n] = X
        for k in range(K):
            b.physics_step(Xf[:, k * NU:(k + 1) * NU].contiguous(), FS)
        return torch.cat([b.t["qpos"][:n], b.t["qvel"][:n]], 1)


def cma_fit(shoot, q0, v0, s1, pop, gens, seed, sigma0=0.5, log=None):
    d = K * NU
    r = np.random.default_rng(seed)
    m = np.zeros(d)
    sigma = sigma0
    C = np.eye(d)
    ps = np.zeros(d)
    pc = np.zeros(d)
    mu = pop // 2
    w = np.log(mu + 0.5) - np.log(np.arange(1, mu + 1))
    w /= w.sum()
    mueff = 1 / np.sum(w ** 2)
    cs = (mueff + 2) / (d + mueff + 5)
    ds = 1 + 2 * max(0, np.sqrt((mueff - 1) / (d + 1)) - 1) + cs
    cc = (4 + mueff / d) / (d + 4 + 2 * mueff / d)
    c1 = 2 / ((d + 1.3) ** 2 + mueff)
    cmu = min(1 - c1, 2 * (mueff - 2 + 1 / mueff) / ((d + 2) ** 2 + mueff))
    chiN = np.sqrt(d) * (1 - 1 / (4 * d) + 1 / (21 * d * d))
    tgt = torch.as_tensor(s1, dtype=torch.float64)
    best = (np.inf, None)
    for g in range(gens):
        ev, B = np.linalg.eigh(C)
        D = np.sqrt(np.maximum(ev, 1e-30))
        z = r.standard_normal((pop, d))
        X = np.clip(m + sigma * (z @ (B * D).T), -1, 1).astype(np.float32)
        S = shoot.final(q0, v0, torch.as_tensor(X, device=shoot.b.device))
        F = (((S - tgt.to(S.device)) / T.QUANT) ** 2).sum(1).cpu().numpy()
        F = np.where(np.isfinite(F), F, np.inf)
        idx = np.argsort(F)
        if F[idx[0]] < best[0]:
            best = (float(F[idx[0]]), X[idx[0]].astype(np.float64))
        sel = (X[idx[:mu]].astype(np.float64) - m) / sigma
        yw = sel.T @ w
        m = np.clip(m + sigma * yw, -1, 1)    # keep the mean in the box (clipped samples otherwise let sigma run away)
        invsqrt = (B / D) @ B.T
        ps = (1 - cs) * ps + np.sqrt(cs * (2 - cs) * mueff) * invsqrt @ yw
        hs = np.linalg.norm(ps) / np.sqrt(1 - (1 - cs) ** (2 * (g + 1))) < (1.4 + 2 / (d + 1)) * chiN
        pc = (1 - cc) * pc + hs * np.sqrt(cc * (2 - cc) * mueff) * yw
        C = (1 - c1 - cmu) * C + c1 * np.outer(pc, pc) + cmu * (sel.T * w) @ sel
        C = 0.5 * (C + C.T)
        sigma *= np.exp((cs / ds) * (np.linalg.norm(ps) / chiN - 1))
        if log and g % 50 == 0:
            log(f"    gen {g} best rms {np.sqrt(best[0] / 55):.3e} sigma {sigma:.2e}")
        if np.sqrt(best[0] / 55) < 1.0 or sigma < 1e-7:
            break
    return best[1], np.sqrt(best[0] / 55), g + 1


def polish(shoot, q0, v0, s1, x, iters=40, h=2e-4):
    """Box-clipped Gauss-Newton with Levenberg damping; FD Jacobian from 1 + 105 envs per iteration
    (float32 controls: h is far above their rounding)."""
    dev = shoot.b.device
    tgt = torch.as_tensor(s1, dtype=torch.float64, device=dev)
    lam = 1e-6
    x = np.clip(x, -1, 1)

    def evalx(X):
        S = shoot.final(q0, v0, torch.as_tensor(X.astype(np.float32), device=dev))
        return ((S - tgt) / T.QUANT).double().cpu().numpy()
    r0 = evalx(x[None])[0]
    f0 = float(r0 @ r0)
    for _ in range(iters):
        steps = np.where(x + h <= 1, h, -h)
        P = np.repeat(x[None], K * NU, 0) + np.diag(steps)
        R = evalx(np.vstack([x[None], P]))
        J = (R[1:] - R[0]).T / steps
        r0 = R[0]
        JTJ, JTr = J.T @ J, J.T @ r0
        improved = False
        for _t in range(8):
            dx = -np.linalg.solve(JTJ + lam * (np.diag(np.diag(JTJ)) + 1e-9 * np.eye(len(x))), JTr)
            xn = np.clip(x + dx, -1, 1)
            rn = evalx(xn[None])[0]
            fn = float(rn @ rn)
            if np.isfinite(fn) and fn < f0:
                x, f0 = xn, fn
                lam = max(lam / 10, 1e-12)
                improved = True
                break
            lam *= 10
        if not improved or np.sqrt(f0 / 55) < 0.5:
            break
    return x, np.sqrt(f0 / 55)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--intervals", default="")
    ap.add_argument("--n", type=int, default=24, help="contact-rich intervals to fit when --intervals is empty")
    ap.add_argument("--variants", default="truth,armature_zero,friction_07")
    ap.add_argument("--pop", type=int, default=4096)
    ap.add_argument("--gens", type=int, default=400)
    ap.add_argument("--synthetic", action="store_true")
    ap.add_argument("--seed", type=int, default=0)
    a = ap.parse_args()
    keys = T.load_keys(KEYS)
    Mtruth = T.make_model(HUMANOID_XML)
    if a.intervals:
        ivs = [int(x) for x in a.intervals.split(",")]
    else:   # contact-rich: >= 2 contacts at the start key (oracle), spread over the rollout
        rich = [i for i in range(len(keys) - 1) if T._ncon(Mtruth, *keys[i]) >= 2]
        ivs = [rich[j] for j in np.linspace(0, len(rich) - 1, a.n).round().astype(int)]
    log = lambda m: print(m, file=sys.stderr, flush=True)   # noqa: E731
    rows = []
    rng = np.random.default_rng(123)
    for var in a.variants.split(","):
        xml = T.variant_xml(var)
        model = HsModel(xml)
        M = T.make_model(xml)
        shoot = GpuShooter(model, a.pop)
        for i in ivs:
            (q0, v0), (q1, v1) = keys[i], keys[i + 1]
            u_true = None
            if a.synthetic:    # the oracle's own end state from known controls, printed like the keys
                u_true = np.clip(rng.normal(0, 0.7, (K, NU)), -1, 1).astype(np.float32).astype(np.float64)
                s = T.IntervalFit(M, q0, v0, q0, v0).final_state(u_true)
                q1, v1 = np.round(s[:28], 6), np.round(s[28:], 6)
            s1 = np.r_[q1, v1]
            t0 = time.time()
            x, rms_cma, gens = cma_fit(shoot, q0, v0, s1, a.pop, a.gens, a.seed + i,
                                       log=lambda m: log(f"{var} {i}: {m}"))
            x, rms_pol = polish(shoot, q0, v0, s1, x)
            xr = x.astype(np.float32).astype(np.float64)
            res = T.IntervalFit(M, q0, v0, q1, v1).residual(xr)     # the oracle's verdict
            rms_orc = float(np.sqrt(np.mean(res ** 2)))
            worst = int(np.argmax(np.abs(res)))
            err = float(np.abs(xr - u_true.ravel()).max()) if u_true is not None else float("nan")
            rows.append((var, i, T._ncon(M, q0, v0), rms_cma, gens, rms_pol, rms_orc, float(np.abs(res).max()), worst,
                         int(np.sum(np.abs(xr) > 1 - 1e-6)), err))
            log(f"{var} interval {i}: cma {rms_cma:.3e} ({gens} gens) polish {rms_pol:.3e} oracle {rms_orc:.3e} "
                f"ctrl err {err:.2e} {time.time() - t0:.1f}s")
        shoot.b.close()
    print("| variant | interval | contacts at start | CMA-ES rms | generations | polished rms (GPU) | oracle rms | "
          "oracle max | worst component | controls at the box | max control error (synthetic) |")
    print("|---|---|---|---|---|---|---|---|---|---|---|")
    for r in rows:
        print(f"| {r[0]} | {r[1]} | {r[2]} | {r[3]:.3e} | {r[4]} | {r[5]:.3e} | {r[6]:.3e} | {r[7]:.3e} | {r[8]} | "
              f"{r[9]} | {r[10]:.2e} |")


if __name__ == "__main__":
    main()

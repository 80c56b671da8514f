"""Evidence for DESIGN.md 5 / profiles/parity_report.md: can the reference's recorded MuJoCo rollout
(tests/golden/humanoid_trajectory.xml, 25 substeps and 5 unknown control vectors between keys) pin
the physics by fitting the controls?  CPU only (oracle/trajfit.py).  Prints markdown.

    python tools/probes/trajfit_report.py > gpurun_out/trajfit.md
"""
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)

from scipy.optimize import least_squares  # noqa: E402

from oracle import trajfit as T  # noqa: E402
from oracle.oracle import Oracle  # noqa: E402
from mujocoposelearning_amd.model import HUMANOID_XML  # noqa: E402

KEYS = os.path.join(ROOT, "tests", "golden", "humanoid_trajectory.xml")
INTERVALS = (3, 10, 35, 56, 90, 112)


def main():
    keys = T.load_keys(KEYS)
    M = T.make_model(HUMANOID_XML)
    rng = np.random.default_rng(0)
    print("### Control fit on the recorded rollout (oracle/trajfit.py)\n")
    print("Residual in units of the printing half-quantum (5e-7); a correct model and a global fit would reach ~1.\n")
    print("| interval | contacts at start | recorded keys: rms / max | synthetic (oracle's own data, known controls): rms / max / max ctrl error |")
    print("|---|---|---|---|")
    for i in INTERVALS:
        (q0, v0), (q1, v1) = keys[i], keys[i + 1]
        t0 = time.time()
        real = T.IntervalFit(M, q0, v0, q1, v1).fit(max_nfev=60)
        u_true = np.clip(rng.normal(0, 0.7, (5, 21)), -1, 1)
        s = T.IntervalFit(M, q0, v0, q0, v0).final_state(u_true)
        syn = T.IntervalFit(M, q0, v0, np.round(s[:28], 6), np.round(s[28:], 6)).fit(max_nfev=60)
        err = np.abs(syn["x"] - u_true.ravel()).max()
        print(f"| {i} | {T._ncon(M, q0, v0)} | {real['rms']:.2e} / {real['maxabs']:.2e} | "
              f"{syn['rms']:.2e} / {syn['maxabs']:.2e} / {err:.2f} |", flush=True)
        print(f"interval {i}: {time.time() - t0:.1f} s", file=sys.stderr)

    print("\n### Basin of the fit: one env step (5 substeps, 21 controls, 55 outputs, unique solution)\n")
    o = Oracle(M=M)

    def seg(st, u, n):
        o.reset_data()
        o.qpos[:] = st[:28]
        o.qvel[:] = st[28:]
        o.step(u, n)
        return np.r_[o.qpos, o.qvel]
    st = np.r_[keys[56][0], keys[56][1]]
    u_true = np.clip(np.random.default_rng(0).normal(0, 0.7, 21), -1, 1)
    print("| substeps | start | rms | max ctrl error |")
    print("|---|---|---|---|")
    for n in (1, 5):
        tgt = seg(st, u_true, n)
        f = lambda u: (seg(st, u, n) - tgt) / T.QUANT  # noqa: E731
        starts = [("0", np.zeros(21))] + [(f"truth + N(0, {d})", np.clip(u_true + rng.normal(0, d, 21), -1, 1))
                                          for d in (0.01, 0.03, 0.3)]
        for name, x0 in starts:
            r = least_squares(f, x0, bounds=(-1, 1), method="trf", max_nfev=200, ftol=1e-15, xtol=1e-15, gtol=1e-15)
            print(f"| {n} | {name} | {np.sqrt(np.mean(r.fun ** 2)):.2e} | {np.abs(r.x - u_true).max():.2e} |",
                  flush=True)

    print("\n### Size of each known-wrong variant's effect over one interval (same start key, same tape)\n")
    print("| interval | " + " | ".join(T.VARIANTS[1:]) + " |")
    print("|---|" + "---|" * (len(T.VARIANTS) - 1))
    for i in INTERVALS:
        (q0, v0), _ = keys[i], keys[i + 1]
        u = np.clip(rng.normal(0, 0.7, (5, 21)), -1, 1)
        base = T.IntervalFit(M, q0, v0, q0, v0).final_state(u)
        cells = []
        for var in T.VARIANTS[1:]:
            sv = T.IntervalFit(T.make_model(HUMANOID_XML, var), q0, v0, q0, v0, variant=var).final_state(u)
            T.set_variant(0)
            cells.append(f"{np.abs(sv - base).max():.1e}")
        print(f"| {i} | " + " | ".join(cells) + " |", flush=True)


if __name__ == "__main__":
    main()

"""ORACLE (test infrastructure only): fit the unrecorded controls of the reference's MuJoCo rollout.

The reference's ``trajectories/humanoid_trajectory.xml`` (fixture ``tests/golden/humanoid_trajectory.xml``)
holds rollout states that real MuJoCo 3.2.5 produced, written by
``generate_trajectories.py:46-61``: one key every ``step_interval`` = 5 env steps, each env step
``frame_skip`` = 5 substeps (``custom_env.py:28`` default; ``custom_env.py:158-160`` sets
``data.ctrl[:] = action`` before every ``mj_step``), so consecutive keys are 25 ``mj_step`` apart
with 5 unknown constant control vectors in between, each clipped to the action box [-1, 1]
(SB3 ``predict`` clips to the Box action space; the motors' ctrlrange is [-1, 1] too).  qpos / qvel
are printed with 6 decimals.

For one interval, :class:`IntervalFit` finds the 5 x nu controls in [-1, 1] that bring the
oracle's state from key i as close as possible to key i + 1, with the miss measured in units of
the printing quantum (5e-7), by a box-constrained trust-region least-squares fit (scipy ``trf``)
with forward-difference Jacobians (a control of env step k only affects the substeps from 5k on,
so each Jacobian column re-simulates from the saved state at that boundary).

``variant`` switches known-WRONG physics in the oracle (``orc_variant`` bits, hsim_oracle.c) or in
the model, to show the fit has power: a correct restatement reaches the printing floor on intervals
where the wrong ones cannot.  Never used by the product.
"""
from __future__ import annotations

import ctypes as C
import os
import xml.etree.ElementTree as ET

import numpy as np

from .oracle import Oracle, OrcData, lib
from .model import compile_mjcf

QUANT = 5e-7                  # half of the 6-decimal printing quantum
STEPS_PER_KEY = 5             # generate_trajectories.py:6 step_interval
FRAME_SKIP = 5                # custom_env.py:28 default (generate_trajectories.py:12-17 passes none)

# oracle physics variants (bits of orc_variant in hsim_oracle.c) and model edits
VARIANT_BITS = {"pyramid_R_unscaled": 1, "no_implicit_damping": 2, "friction_min_mix": 4, "mujoco_tolerance_stop": 8}
MODEL_VARIANTS = ("armature_zero",)
VARIANTS = ("truth",) + tuple(VARIANT_BITS) + MODEL_VARIANTS


def load_keys(path):
    """(qpos, qvel) of the rollout keys (the keys after ``initial_pose``; the first rollout key
    repeats initial_pose: generate_trajectories.py:36-40 then :48-57 at step 0)."""
    keys = [k for k in ET.parse(path).getroot().iter("key") if k.get("qpos") and k.get("qvel")]
    i0 = keys.index(next(k for k in keys if k.get("name") == "initial_pose"))
    out = []
    for k in keys[i0 + 1:]:
        out.append((np.array([float(x) for x in k.get("qpos").split()]),
                    np.array([float(x) for x in k.get("qvel").split()])))
    return out


def set_variant(bits):
    L = lib()
    C.c_int.in_dll(L, "orc_variant").value = int(bits)


def make_model(xml_path, variant="truth"):
    M = compile_mjcf(xml_path)
    if variant == "armature_zero":
        M["dof_armature"] = np.zeros_like(np.asarray(M["dof_armature"], float))
    return M


def variant_xml(name, xml_path=None):
    """A model file for the XML-edit variants (the GPU fit, tools/probes/gpu_trajfit.py, runs them
    through both compilers): ``armature_zero`` sets every joint armature to 0, ``friction_07`` the
    floor friction to 0.7 (what min-mixing the floor's 1 with the bodies' 0.7 would give)."""
    import re
    import tempfile
    if xml_path is None:
        from mujocoposelearning_amd.model import HUMANOID_XML as xml_path
    src = open(xml_path).read()
    if name == "truth":
        return xml_path
    if name == "armature_zero":
        src, n = re.subn(r'armature="[^"]*"', 'armature="0"', src)
        assert n > 0
    elif name == "friction_07":
        # the floor geom's friction 1 -> 0.7: max(0.7, body 0.7) = 0.7, as a min-mixing rule would give
        src, n = re.subn(r'(<geom[^>]*name="floor"[^>]*?)friction="[^"]*"', r'\1friction="0.7 0.005 0.0001"', src)
        if n == 0:
            src, n = re.subn(r'(<geom[^>]*name="floor")', r'\1 friction="0.7 0.005 0.0001"', src)
        assert n > 0
    else:
        raise ValueError(name)
    d = tempfile.mkdtemp()
    p = os.path.join(d, f"humanoid_{name}.xml")
    open(p, "w").write(src)
    return p


class IntervalFit:
    """Controls of one key interval: u[k, :] for env step k = 0..4 of the interval."""

    def __init__(self, M, q0, v0, q1, v1, variant="truth", steps=STEPS_PER_KEY, frame_skip=FRAME_SKIP):
        self.o = Oracle(M=M)
        self.variant_bits = VARIANT_BITS.get(variant, 0)
        self.q0, self.v0, self.q1, self.v1 = (np.asarray(x, float) for x in (q0, v0, q1, v1))
        self.K, self.fs = steps, frame_skip
        self.nu = M["nu"]
        self.nq, self.nv = M["nq"], M["nv"]
        self._snap = [OrcData() for _ in range(self.K + 1)]
        self.nsim = 0

    def _copy(self, dst, src):
        C.memmove(C.addressof(dst), C.addressof(src), C.sizeof(OrcData))

    def _start(self):
        o = self.o
        o.reset_data()
        o.qpos[:] = self.q0
        o.qvel[:] = self.v0

    def _run(self, u, save=False, k0=0):
        """Simulate env steps k0..K-1 from the current oracle state; save boundary snapshots."""
        set_variant(self.variant_bits)
        o = self.o
        for k in range(k0, self.K):
            if save:
                self._copy(self._snap[k], o.d)
            o.step(u[k], self.fs)
            self.nsim += self.fs
        return np.r_[o.qpos, o.qvel]

    def final_state(self, u):
        self._start()
        return self._run(np.asarray(u, float).reshape(self.K, self.nu))

    def residual(self, x):
        s = self.final_state(x)
        return (s - np.r_[self.q1, self.v1]) / QUANT

    def jacobian(self, x, eps=1e-6):
        u = np.asarray(x, float).reshape(self.K, self.nu)
        self._start()
        base = self._run(u, save=True)
        J = np.empty((base.size, u.size))
        for k in range(self.K):
            for j in range(self.nu):
                up = u.copy()
                h = eps if u[k, j] + eps <= 1.0 else -eps
                up[k, j] += h
                self._copy(self.o.d, self._snap[k])
                J[:, k * self.nu + j] = (self._run(up, k0=k) - base) / (h * QUANT)
        return J

    def fit(self, x0=None, max_nfev=60, ftol=1e-10, xtol=1e-10, gtol=1e-10):
        from scipy.optimize import least_squares
        x0 = np.zeros(self.K * self.nu) if x0 is None else np.clip(np.asarray(x0, float).ravel(), -1, 1)
        r = least_squares(self.residual, x0, jac=self.jacobian, bounds=(-1.0, 1.0), method="trf",
                          x_scale=1.0, max_nfev=max_nfev, ftol=ftol, xtol=xtol, gtol=gtol)
        res = self.residual(r.x)
        return dict(x=r.x, res=res, rms=float(np.sqrt(np.mean(res ** 2))), maxabs=float(np.abs(res).max()),
                    nfev=int(r.nfev), status=int(r.status), active=int(np.sum(np.abs(r.x) > 1 - 1e-9)))


def fit_interval(args):
    """Process-pool entry: (xml_path, keys_path, i, variant, jitter_seed, max_nfev) -> dict."""
    xml_path, keys_path, i, variant, jitter_seed, max_nfev = args
    keys = load_keys(keys_path)
    M = make_model(xml_path, variant)
    (q0, v0), (q1, v1) = keys[i], keys[i + 1]
    if jitter_seed is not None:            # the start key moved inside its printing quantum
        rng = np.random.default_rng(jitter_seed)
        q0 = q0 + rng.uniform(-QUANT, QUANT, q0.size)
        v0 = v0 + rng.uniform(-QUANT, QUANT, v0.size)
    f = IntervalFit(M, q0, v0, q1, v1, variant=variant)
    out = f.fit(max_nfev=max_nfev)
    out.update(i=i, variant=variant, jitter=jitter_seed, ncon0=_ncon(M, q0, v0), nsim=f.nsim)
    return out


def _ncon(M, q, v):
    o = Oracle(M=M)
    o.reset_data()
    o.qpos[:] = q
    o.qvel[:] = v
    o.forward()
    return int(o.d.ncon)


def run_many(jobs, workers=None):
    workers = workers or min(8, os.cpu_count() or 1)
    if workers <= 1:
        return [fit_interval(j) for j in jobs]
    import multiprocessing as mp
    with mp.get_context("fork").Pool(workers) as pool:
        return pool.map(fit_interval, jobs, chunksize=1)

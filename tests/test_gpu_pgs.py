"""The <option solver="PGS"> kernel instance against the oracle's PGS (oracle/hsim_oracle.c
solve_pgs, mj_solPGS semantics) and against the engine's own Newton solve.

The reference's humanoid.xml runs MuJoCo's default Newton solver, so PGS is an opt-in engine mode
(BASELINE.json's north star names a PGS contact solve).  Tolerances, fp64 kernel:
  * PGS vs oracle PGS, one substep, sweeps run to convergence: |d qacc| <= 1e-7 scale
  * PGS vs the engine's Newton on the same states (both converged): |d qacc| <= 1e-6 scale
fp32 kernel (MuJoCo's default 100 sweeps / 1e-8): |d qacc| <= 2e-3 scale against the fp64 oracle (the
Newton fp32 bound)."""
import re

import numpy as np
import pytest

from conftest import XML

pytestmark = pytest.mark.gpu


def _pgs_xml(tmp_path, iterations, tolerance):
    src = re.sub(r"<option[^>]*/>", f'<option timestep="0.005" solver="PGS" iterations="{iterations}" '
                 f'tolerance="{tolerance}"/>', open(XML).read(), count=1)
    p = tmp_path / f"pgs_{iterations}_{tolerance}.xml"
    p.write_text(src)
    return str(p)


def _contact_states(M, n, seed, deep=False):
    """Keyframes pushed into the floor; ``deep``: every other round 3 cm deeper (prone / supine then
    have ~118 constraint rows, past the PGS instance's LDS row cache of 56 / 64)."""
    rng = np.random.default_rng(seed)
    keys = list(M["keyframes"].values())
    out = []
    for i in range(n):
        q = keys[i % len(keys)].copy()
        q[2] -= 0.002 * (1 + i // len(keys)) + (0.03 if deep and (i // len(keys)) % 2 == 1 else 0.0)
        q[7:] += rng.uniform(-0.05, 0.05, 21)
        out.append((q, rng.normal(0, 0.5, 27), rng.uniform(-1, 1, 21).astype(np.float32)))
    return out


def _gpu_one_substep(model, states, prec):
    import torch
    from mujocoposelearning_amd.batch import HsBatch
    b = HsBatch(model, len(states), precision=prec)
    b.set_state(qpos=np.stack([s[0] for s in states]), qvel=np.stack([s[1] for s in states]), time=0.0,
                qacc_warmstart=0.0)
    b.physics_step(torch.tensor(np.stack([s[2] for s in states]), device=b.device), 1)
    st = b.get_state()
    aux = b.aux.double().cpu().numpy()
    b.close() if hasattr(b, "close") else None
    return st, aux


def _oracle_one_substep(o, q, v, c):
    o.reset_data()
    o.qpos[:] = q
    o.qvel[:] = v
    o.step(c.astype(np.float64), 1)
    return o.qpos.copy(), o.qvel.copy(), o.get("qacc"), o.d.nefc, o.d.solver_niter


@pytest.mark.parametrize("prec", ["fp64", "fp32"])
def test_pgs_kernel_matches_oracle_pgs(tmp_path, prec):
    from mujocoposelearning_amd.model import HsModel
    from oracle.oracle import Oracle
    # fp64: sweeps to convergence; fp32: MuJoCo's defaults (100 sweeps, tolerance 1e-8).  Run far past
    # them, fp32 rounding noise drives the forces along the pyramid's null directions (the 4 edge
    # rows of a contact span 3 dimensions; only the tiny R regularises that direction) until their
    # cancellation in J'f costs the qacc its accuracy -- fp32 PGS is a MuJoCo-defaults mode
    xml = _pgs_xml(tmp_path, 3000, 1e-20) if prec == "fp64" else _pgs_xml(tmp_path, 100, 1e-8)
    m, o = HsModel(xml), Oracle(xml)
    assert m.field("opt_solver")[0] == 1 and o.m.solver == 1
    states = _contact_states(o.M, 24, seed=11, deep=prec == "fp64")
    st, aux = _gpu_one_substep(m, states, prec)
    rows = 0
    for i, (q, v, c) in enumerate(states):
        rq, rv, ra, nefc, nit = _oracle_one_substep(o, q, v, c)
        rows += nefc
        assert int(aux[i, 36]) == nefc, i
        scale = 1 + np.abs(ra).max()
        if prec == "fp64":
            assert np.abs(aux[i, :27] - ra).max() <= 1e-7 * scale, (i, np.abs(aux[i, :27] - ra).max(), scale)
            assert np.abs(st["qvel"][i] - rv).max() <= 1e-9 * scale, i
            assert np.abs(st["qpos"][i] - rq).max() <= 1e-11, i
        else:
            assert np.abs(aux[i, :27] - ra).max() <= 2e-3 * scale, (i, np.abs(aux[i, :27] - ra).max(), scale)
            assert np.abs(st["qvel"][i] - rv).max() <= 1e-5 * scale, i
    assert rows > 24 * 10       # contact-rich states
    # fp64: rows past the LDS row cache (u_r rebuilt per use) are exercised too
    assert int(aux[:, 36].max()) > (64 if prec == "fp64" else 32)


def test_pgs_kernel_converges_to_newton_kernel(tmp_path):
    """Same states through the engine's Newton instance and its PGS instance (fp64): the primal
    and dual solves of the same problem agree (SURVEY.md section 4.4 on the GPU)."""
    from mujocoposelearning_amd.model import HsModel
    mp, mn = HsModel(_pgs_xml(tmp_path, 5000, 1e-24)), HsModel(XML)
    from oracle.oracle import Oracle
    states = _contact_states(Oracle(XML).M, 16, seed=5)
    _, ap = _gpu_one_substep(mp, states, "fp64")
    _, an = _gpu_one_substep(mn, states, "fp64")
    for i in range(len(states)):
        scale = 1 + np.abs(an[i, :27]).max()
        assert np.abs(ap[i, :27] - an[i, :27]).max() <= 1e-6 * scale, (i, np.abs(ap[i, :27] - an[i, :27]).max())
        assert int(ap[i, 36]) == int(an[i, 36])


def test_pgs_default_tolerance_env_rollout(tmp_path):
    """An env batch on the PGS model (MuJoCo's default iterations 100 / tolerance 1e-8) steps a
    U(-1,1) tape for 60 env steps in fp32 with finite outputs, and its sweep counts stop early on
    the tolerance rule."""
    import torch
    from mujocoposelearning_amd.model import HsModel
    from mujocoposelearning_amd.vec_env import HumanoidVecEnv
    xml = _pgs_xml(tmp_path, 100, 1e-8)
    env = HumanoidVecEnv({"model_path": xml, "duration": 10.0, "reward_config": {"type": "stand"}, "frame_skip": 3},
                         n_envs=256, model=HsModel(xml), seed=0)
    env.reset_tensors()
    g = torch.Generator(device="cuda").manual_seed(0)
    for _ in range(60):
        obs, rew, term, trunc = env.step_tensors(torch.rand(256, 21, device="cuda", generator=g) * 2 - 1)
    torch.cuda.synchronize()
    assert torch.isfinite(obs).all() and torch.isfinite(rew).all()
    w = env.batch.warning.sum(0).tolist()
    print("warnings [badqpos, badqvel, badqacc, overflow]:", w)
    # Newton mode has none; PGS at 100 sweeps leaves a few hard states unconverged, which
    # mj_checkAcc resets (measured: 1 in 46k substeps here, 6 in 614k at 4096 envs)
    assert w[0] == 0 and w[1] == 0 and w[2] + w[3] <= 4, w
    it = env.batch.aux[:, 37].float()
    assert float(it.mean()) < 100 and float(it.max()) <= 100
    env.close()


def test_pgs_fp64_trajectory_matches_oracle(tmp_path):
    """50 substeps of the PGS model from a standing pose with floor contacts and a U(-1,1) tape:
    the fp64 kernel tracks the oracle's PGS (sweeps run to convergence in both)."""
    import torch
    from mujocoposelearning_amd.batch import HsBatch
    from mujocoposelearning_amd.model import HsModel
    from oracle.oracle import Oracle
    xml = _pgs_xml(tmp_path, 2000, 1e-20)
    m, o = HsModel(xml), Oracle(xml)
    rng = np.random.default_rng(8)
    q = o.M["qpos0"].copy()
    q[2] = 1.25                      # feet slightly in the floor
    v = rng.uniform(-0.05, 0.05, 27)
    b = HsBatch(m, 1, precision="fp64")
    b.set_state(qpos=q, qvel=v, time=0.0, qacc_warmstart=0.0)
    o.reset_data()
    o.qpos[:] = q
    o.qvel[:] = v
    ctrl = rng.uniform(-1, 1, (50, 21)).astype(np.float32)
    c = torch.tensor(ctrl, device=b.device)
    for s in range(50):
        b.physics_step(c[s:s + 1], 1)
        o.step(ctrl[s].astype(np.float64), 1)
    st = b.get_state()
    assert int(b.aux[0, 36]) > 0               # contact rows active at the end
    assert np.abs(st["qpos"][0] - o.qpos).max() < 1e-8
    assert np.abs(st["qvel"][0] - o.qvel).max() < 1e-6

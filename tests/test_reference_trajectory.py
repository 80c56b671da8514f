"""Physics checked against the reference's recorded MuJoCo 3.2.5 rollout (beyond initial_pose).

Fixture: tests/golden/humanoid_trajectory.xml = the reference's trajectories/humanoid_trajectory.xml,
written by generate_trajectories.py:6-72: a stochastic `walk` policy in HumanoidEnv with the
default frame_skip 5 (custom_env.py:28), one <key> every step_interval = 5 env steps, i.e. 25
mj_step substeps = 0.125 s apart (the keys' `time` attribute is step * timestep, a mislabel), qpos
and qvel printed with 6 decimals.  The 25 actions in between are not recorded.

1. **No contact-free interval exists** (the free-flight momentum identities cannot be used):
   28 of the 150 rollout keys have no contact and 5 consecutive key pairs are contact-free at both
   ends, but every one of those pairs received a large upward external impulse in between
   (J_z = 12..64 N s against a 6-decimal uncertainty of ~1e-3), and the oracle started from the
   first key of each pair makes floor contact within the interval on 79 of 80 random action tapes.
2. **Friction-cone identity over all 149 intervals.**  Only gravity and floor contacts act on the
   humanoid from outside (actuators, springs, dampers, joint / tendon limits and body-body
   contacts are internal), so the external impulse over an interval is
       J = P(t + 0.125) - P(t) - M g 0.125,
   where P is the total linear momentum computed by OUR model (masses, COM kinematics: P is the
   linear part of sum_b cinert_b * cvel_b) from MuJoCo's recorded (qpos, qvel).  Every floor
   contact force lies in the pyramidal friction cone around +z with the mixed friction
   mu = max(1, 0.7) = 1 (humanoid.xml:40,105), whose cross-section is inside the circle of radius
   mu, and a sum of such forces stays in that cone: J_z >= 0 and |J_xy| <= mu J_z.  The recorded
   data satisfy it on all 149 intervals with max |J_xy| / J_z = 0.849, which also excludes the
   alternative mixing rule min(1, 0.7) = 0.7 (MuJoCo takes the max; the oracle and the kernel do).
   Parity remains unpinned beyond these inequalities and tests/test_reference_pin.py.
"""
import os
import xml.etree.ElementTree as ET

import numpy as np
import pytest

from conftest import GOLDEN, XML

SUBSTEPS_PER_KEY = 5 * 5          # step_interval 5 env steps x frame_skip 5 (generate_trajectories.py:6,16-17,46)
QUANT = 2e-3                      # bound on |dJ| from the 6-decimal printing (27 qvel x 5e-7 x ~40 kg m)


@pytest.fixture(scope="module")
def rollout():
    from oracle.oracle import Oracle
    keys = [k for k in ET.parse(os.path.join(GOLDEN, "humanoid_trajectory.xml")).getroot().iter("key")
            if k.get("qpos") and k.get("qvel")]
    keys = keys[keys.index(next(k for k in keys if k.get("name") == "initial_pose")) + 1:]   # the rollout keys
    o = Oracle(XML)
    out = []
    for k in keys:
        q = np.array([float(x) for x in k.get("qpos").split()])
        v = np.array([float(x) for x in k.get("qvel").split()])
        o.reset_data()
        o.qpos[:] = q
        o.qvel[:] = v
        o.forward()
        out.append(dict(q=q, v=v, P=spatial_momentum(o)[3:], ncon=o.d.ncon))
    return o, out


def spatial_momentum(o):
    """sum_b cinert_b * cvel_b: [angular momentum about the root subtree COM, linear momentum]."""
    h = np.zeros(6)
    for i, x in zip(o.get("cinert")[1:], o.get("cvel")[1:]):
        h += [i[0] * x[0] + i[3] * x[1] + i[4] * x[2] - i[8] * x[4] + i[7] * x[5],
              i[3] * x[0] + i[1] * x[1] + i[5] * x[2] + i[8] * x[3] - i[6] * x[5],
              i[4] * x[0] + i[5] * x[1] + i[2] * x[2] - i[7] * x[3] + i[6] * x[4],
              i[8] * x[1] - i[7] * x[2] + i[9] * x[3], i[6] * x[2] - i[8] * x[0] + i[9] * x[4],
              i[7] * x[0] - i[6] * x[1] + i[9] * x[5]]
    return h


def impulses(o, rows):
    M = float(np.sum(o.M["body_mass"]))
    g = np.asarray(o.M["opt_gravity"], float)
    dt = SUBSTEPS_PER_KEY * float(o.M["opt_timestep"])
    return np.array([b["P"] - a["P"] - M * g * dt for a, b in zip(rows, rows[1:])])


def test_momentum_is_linear_momentum(rollout):
    """sanity of the momentum helper: the linear part equals M * d(com)/dt by finite differences"""
    o, _ = rollout
    rng = np.random.default_rng(0)
    q = o.M["qpos0"].copy()
    q[7:] += rng.uniform(-0.3, 0.3, 21)
    v = rng.normal(0, 1, 27)
    o.reset_data()
    o.qpos[:] = q
    o.qvel[:] = v
    o.forward()
    P = spatial_momentum(o)[3:]
    c0 = o.get("subtree_com")[0]
    eps = 1e-7
    # move the configuration by eps along v (translations add, hinges add, quaternion via exp)
    qn = q.copy()
    qn[:3] += eps * v[:3]
    qn[7:] += eps * v[6:]
    w = v[3:6] * eps / 2
    dq = np.r_[1.0, w] / np.linalg.norm(np.r_[1.0, w])
    a = q[3:7]
    qn[3:7] = [a[0] * dq[0] - a[1:] @ dq[1:], *(a[0] * dq[1:] + dq[0] * a[1:] + np.cross(a[1:], dq[1:]))]
    o.reset_data()
    o.qpos[:] = qn
    o.forward()
    c1 = o.get("subtree_com")[0]
    M = float(np.sum(o.M["body_mass"]))
    np.testing.assert_allclose(P, M * (c1 - c0) / eps, rtol=1e-5, atol=1e-5)


def test_no_contact_free_interval_qualifies(rollout):
    o, rows = rollout
    assert len(rows) == 150
    free = [i for i, r in enumerate(rows) if r["ncon"] == 0]
    pairs = [i for i in range(len(rows) - 1) if rows[i]["ncon"] == 0 and rows[i + 1]["ncon"] == 0]
    assert len(free) == 28 and len(pairs) == 5
    J = impulses(o, rows)
    # every contact-free-at-both-ends pair received an upward external impulse far above the
    # printing precision: contact happened in between
    assert np.all(J[pairs, 2] > 10.0), J[pairs]
    # and the oracle, started from the pair's first key, touches the floor within the interval on
    # (nearly) every random action tape of 5 env steps x 5 substeps
    rng = np.random.default_rng(0)
    touched = 0
    for i in pairs:
        for _ in range(16):
            o.reset_data()
            o.qpos[:] = rows[i]["q"]
            o.qvel[:] = rows[i]["v"]
            hit = False
            for _e in range(5):
                act = rng.uniform(-1, 1, 21)
                for _s in range(5):
                    o.step(act, 1)
                    hit = hit or o.d.ncon > 0
            touched += hit
    assert touched >= 75, touched


def test_external_impulse_inside_the_friction_cone_on_every_interval(rollout):
    o, rows = rollout
    J = impulses(o, rows)
    assert J.shape == (149, 3)
    assert np.all(J[:, 2] > -QUANT), J[:, 2].min()               # the floor only pushes
    ratio = np.hypot(J[:, 0], J[:, 1]) / np.maximum(J[:, 2], 1e-12)
    # the model's floor friction (max-mixed): 1.0
    o.reset_data()
    o.qpos[:] = rows[np.argmax(np.array([r["ncon"] for r in rows]))]["q"]
    o.forward()
    mus = {c["friction"][0] for c in o.contacts() if 0 in c["geom"]}
    assert mus == {1.0}
    assert np.all(np.hypot(J[:, 0], J[:, 1]) <= 1.0 * J[:, 2] + QUANT), ratio.max()
    # the data need mu >= 0.849: a min-mixed friction (0.7) is excluded by MuJoCo's own output
    assert 0.84 < ratio.max() < 0.86
    assert ratio.max() > 0.7 + 0.1


def test_control_fit_machinery_recovers_one_substep_controls():
    """oracle/trajfit.py's least-squares fit (used to try to pin the physics against the recorded
    rollout): on one substep the map from controls to the next state is smooth, and the
    fit recovers synthetic controls from zero exactly.  (Over an interval's 25 substeps the map is
    multi-modal and the fit does not recover even the oracle's own synthetic data:
    profiles/reference_trajectory_fit_r4.md.)"""
    from oracle import trajfit as T
    keys = T.load_keys(os.path.join(GOLDEN, "humanoid_trajectory.xml"))
    assert len(keys) == 150
    M = T.make_model(XML)
    (q0, v0), _ = keys[56], keys[57]
    u = np.clip(np.random.default_rng(0).normal(0, 0.7, 21), -1, 1)
    f = T.IntervalFit(M, q0, v0, q0, v0, steps=1, frame_skip=1)
    s = f.final_state(u)
    fit = T.IntervalFit(M, q0, v0, s[:28], s[28:], steps=1, frame_skip=1).fit(max_nfev=40)
    assert fit["rms"] < 1e-3 and np.abs(fit["x"] - u).max() < 1e-6


def test_wrong_physics_variants_change_an_interval():
    """The known-wrong variants the fit was meant to reject (oracle orc_variant bits and model edits)
    are live: each moves the state after one 25-substep interval by far more than the printing
    quantum, on the same start key and control tape; the tolerance-stop check changes nothing."""
    from oracle import trajfit as T
    keys = T.load_keys(os.path.join(GOLDEN, "humanoid_trajectory.xml"))
    (q0, v0), _ = keys[56], keys[57]
    u = np.clip(np.random.default_rng(1).normal(0, 0.7, (5, 21)), -1, 1)
    base = T.IntervalFit(T.make_model(XML), q0, v0, q0, v0).final_state(u)
    try:
        for var in T.VARIANTS[1:]:
            s = T.IntervalFit(T.make_model(XML, var), q0, v0, q0, v0, variant=var).final_state(u)
            d = np.abs(s - base).max()
            if var == "mujoco_tolerance_stop":
                assert d == 0.0
            else:
                assert d > 1e3 * T.QUANT, (var, d)
    finally:
        T.set_variant(0)


def test_gpu_fit_variant_models_compile_with_both_compilers():
    """The XML-edit variants of the GPU fit (tools/probes/gpu_trajfit.py): armature 0 everywhere /
    floor friction 0.7, as the product's MJCF compiler and the oracle's both read them."""
    from oracle import trajfit as T
    from oracle.model import compile_mjcf
    from mujocoposelearning_amd.model import HsModel
    for var, check in (("armature_zero", lambda M: np.all(np.asarray(M["dof_armature"]) == 0)),
                       ("friction_07", lambda M: abs(M["geom_friction"][0][0] - 0.7) < 1e-12)):
        p = T.variant_xml(var, XML)
        assert check(compile_mjcf(p)), var
        m = HsModel(p)
        assert check({"dof_armature": m.field("dof_armature"), "geom_friction": m.field("geom_friction")}), var

"""Physics invariants that pin the fp64 oracle restatement of mj_step (no MuJoCo available here:
SURVEY.md section 4 item 4).  Each check uses an independent path (energies, finite differences,
analytic geometry, KKT conditions) rather than re-running the same code."""
import ctypes as C

import numpy as np
import pytest

from conftest import XML


@pytest.fixture()
def orc():
    from oracle.oracle import Oracle
    return Oracle(XML)


def _random_state(o, seed, scale=0.3):
    rng = np.random.default_rng(seed)
    q = o.M["qpos0"].copy()
    q[7:] += rng.uniform(-scale, scale, 21)
    quat = np.array([1.0, *rng.normal(0, 0.2, 3)])
    q[3:7] = quat / np.linalg.norm(quat)
    q[2] += 1.0   # airborne: no contacts
    return q, rng.normal(0, 1.0, 27)


def _kinetic_energy(o):
    """0.5 sum_b cvel_b' I_b cvel_b from the com-frame spatial inertias (independent of qM)."""
    cinert, cvel = o.get("cinert"), o.get("cvel")
    ke = 0.0
    for b in range(1, o.M["nbody"]):
        i, v = cinert[b], cvel[b]
        I = np.array([[i[0], i[3], i[4]], [i[3], i[1], i[5]], [i[4], i[5], i[2]]])
        m, c = i[9], i[6:9]
        w, lin = v[:3], v[3:]
        # spatial inertia about origin with first moment c = m * com_offset
        ke += 0.5 * (w @ I @ w + m * lin @ lin + 2 * lin @ np.cross(w, c))
    return ke


def _potential(o):
    g = np.array(o.m.gravity)     # the (possibly modified) model actually simulated
    return -sum(o.M["body_mass"][b] * g @ o.get("xipos")[b] for b in range(1, o.M["nbody"]))


@pytest.mark.parametrize("seed", [0, 1, 2])
def test_mass_matrix_matches_kinetic_energy(orc, seed):
    q, v = _random_state(orc, seed)
    orc.qpos[:] = q
    orc.qvel[:] = v
    orc.forward()
    M = orc.get("qM")
    assert np.allclose(M, M.T)
    assert np.all(np.linalg.eigvalsh(M) > 0)
    arm = orc.M["dof_armature"]
    ke_tree = _kinetic_energy(orc)
    assert 0.5 * v @ (M - np.diag(arm)) @ v == pytest.approx(ke_tree, rel=1e-10)


def test_gravity_bias_is_potential_gradient(orc):
    q, _ = _random_state(orc, 3)
    orc.qpos[:] = q
    orc.qvel[:] = 0
    orc.forward()
    bias = orc.get("qfrc_bias")
    eps = 1e-6
    for dof in range(6, 27):           # hinge dofs: qvel == d qpos / dt
        qa = 7 + dof - 6
        vals = []
        for s in (+1, -1):
            orc.qpos[:] = q
            orc.qpos[qa] += s * eps
            orc.forward()
            vals.append(_potential(orc))
        dV = (vals[0] - vals[1]) / (2 * eps)
        assert bias[dof] == pytest.approx(dV, rel=1e-6, abs=1e-7)


def _strip_model(o, gravity=True):
    m = o.m
    m.npair = 0
    for j in range(o.M["njnt"]):
        m.jnt_limited[j] = 0
        m.jnt_stiffness[j] = 0
    for t in range(o.M["ntendon"]):
        m.tendon_limited[t] = 0
    for d in range(o.M["nv"]):
        m.dof_damping[d] = 0
    if not gravity:
        for k in range(3):
            m.gravity[k] = 0


def _total_energy(o):
    """tree kinetic energy + armature kinetic energy + gravitational potential."""
    return _kinetic_energy(o) + 0.5 * np.sum(o.M["dof_armature"] * o.qvel ** 2) + _potential(o)


def test_zero_gravity_energy_error_is_first_order_in_h():
    """Euler on a configuration-dependent M is not exactly energy-conserving; its energy error
    over a fixed horizon must shrink linearly with the timestep (integrator consistency)."""
    from oracle.oracle import Oracle
    drift = []
    for h in (0.005, 0.0025, 0.00125):
        o = Oracle(XML)
        _strip_model(o, gravity=False)
        o.m.timestep = h
        q, v = _random_state(o, 4)
        o.qpos[:] = q
        o.qvel[:] = 0.3 * v
        o.forward()
        e0 = _total_energy(o)
        for _ in range(int(round(1.5 / h))):
            o.step(None, 1)
        o.forward()
        drift.append(abs(_total_energy(o) - e0) / e0)
    assert drift[0] < 1e-2
    assert 1.6 < drift[0] / drift[1] < 2.5 and 1.6 < drift[1] / drift[2] < 2.5


def test_free_fall_energy_bias_is_symplectic_euler(orc):
    """Under constant gravity semi-implicit Euler loses exactly 0.5*M*g^2*h^2 per step."""
    _strip_model(orc)
    q, v = _random_state(orc, 4)
    orc.qpos[:] = q
    orc.qvel[:] = 0.3 * v
    orc.forward()
    e0 = _total_energy(orc)
    n = 200
    for _ in range(n):
        orc.step(None, 1)
    orc.forward()
    h, g, mt = orc.M["opt_timestep"], 9.81, orc.M["body_subtreemass"][0]
    expect = -n * 0.5 * mt * g * g * h * h
    assert (_total_energy(orc) - e0) == pytest.approx(expect, rel=0.05)


def test_zero_gravity_momentum_error_is_first_order_in_h():
    """Linear momentum of a free articulated body is conserved by the continuous dynamics; the
    Euler discretisation must conserve it up to an O(h) error over a fixed horizon."""
    from oracle.oracle import Oracle

    def momentum(o):
        o.forward()
        p = np.zeros(3)
        for b in range(1, o.M["nbody"]):
            i, vel = o.get("cinert")[b], o.get("cvel")[b]
            p += i[9] * vel[3:] - np.cross(i[6:9], vel[:3])
        return p
    err = []
    for h in (0.005, 0.0025, 0.00125):
        o = Oracle(XML)
        _strip_model(o, gravity=False)
        o.m.timestep = h
        q, v = _random_state(o, 5)
        o.qpos[:] = q
        o.qvel[:] = v
        p0 = momentum(o)
        for _ in range(int(round(0.5 / h))):
            o.step(None, 1)
        err.append(np.abs(momentum(o) - p0).max() / np.abs(p0).max())
    assert err[0] < 5e-2
    assert 1.5 < err[0] / err[1] < 2.6 and 1.5 < err[1] / err[2] < 2.6


@pytest.mark.parametrize("key", ["squat", "prone", "supine", "stand_on_left_leg"])
def test_contact_geometry_analytic(orc, key):
    q = orc.M["keyframes"][key].copy()
    q[2] -= 0.01   # push slightly into the floor so contacts exist
    orc.qpos[:] = q
    orc.forward()
    cons = orc.contacts()
    gx, gm = orc.get("geom_xpos"), orc.get("geom_xmat").reshape(-1, 3, 3)
    found = 0
    for c in cons:
        g1, g2 = c["geom"]
        if orc.M["geom_type"][g1] != 0:
            continue
        found += 1
        r = orc.M["geom_size"][g2][0]
        if orc.M["geom_type"][g2] == 2:
            expect = [gx[g2][2] - r]
        else:
            ax = gm[g2][:, 2] * orc.M["geom_size"][g2][1]
            expect = [gx[g2][2] + ax[2] - r, gx[g2][2] - ax[2] - r]
        assert min(abs(c["dist"] - e) for e in expect) < 1e-12
        assert np.allclose(c["frame"][:3], [0, 0, 1])
        assert abs(c["frame"][:3] @ c["frame"][3:6]) < 1e-12 and abs(np.linalg.norm(c["frame"][3:6]) - 1) < 1e-12
    # every capsule/sphere end below the floor must have produced a contact
    expect_n = 0
    for a, b in orc.M["collision_pairs"]:
        if orc.M["geom_type"][a] != 0:
            continue
        r = orc.M["geom_size"][b][0]
        if orc.M["geom_type"][b] == 2:
            expect_n += int(gx[b][2] - r <= 0)
        else:
            ax = gm[b][:, 2] * orc.M["geom_size"][b][1]
            expect_n += int(gx[b][2] + ax[2] - r <= 0) + int(gx[b][2] - ax[2] - r <= 0)
    assert found == expect_n and found > 0


@pytest.mark.parametrize("key", ["squat", "prone", "supine"])
def test_newton_solution_satisfies_kkt(orc, key):
    q = orc.M["keyframes"][key].copy()
    q[2] -= 0.005
    orc.qpos[:] = q
    orc.qvel[:] = np.random.default_rng(1).normal(0, 0.5, 27)
    orc.forward()
    d = orc.d
    ne, nv = d.nefc, orc.M["nv"]
    assert ne > 0
    J = np.ctypeslib.as_array(d.efc_J)[:ne, :nv]
    aref = np.ctypeslib.as_array(d.efc_aref)[:ne]
    D = np.ctypeslib.as_array(d.efc_D)[:ne]
    qacc, qs, M = orc.get("qacc"), orc.get("qacc_smooth"), orc.get("qM")
    jar = J @ qacc - aref
    f = np.where(jar < 0, -D * jar, 0.0)
    assert np.allclose(M @ (qacc - qs), J.T @ f, rtol=1e-9, atol=1e-8 * np.abs(J.T @ f).max())
    assert np.allclose(np.ctypeslib.as_array(d.efc_force)[:ne], f, rtol=1e-9, atol=1e-9)
    # dual check: the optimum of the primal is unique -- perturbing qacc raises the cost
    def cost(x):
        j = J @ x - aref
        return 0.5 * (x - qs) @ M @ (x - qs) + 0.5 * np.sum(D * np.minimum(j, 0) ** 2)
    c0 = cost(qacc)
    rng = np.random.default_rng(2)
    for _ in range(20):
        assert cost(qacc + 1e-4 * rng.normal(size=nv)) >= c0


def test_joint_limit_rows_and_impedance(orc):
    q = orc.M["qpos0"].copy()
    q[2] += 1.0
    j = orc.M["jnt_name"].index("knee_right")
    qa = orc.M["jnt_qposadr"][j]
    q[qa] = orc.M["jnt_range"][j][0] - 0.005    # 5 mrad past the lower limit
    orc.qpos[:] = q
    orc.forward()
    d = orc.d
    rows = [r for r in range(d.nefc) if d.efc_type[r] == 3]
    assert len(rows) == 1 and d.efc_id[rows[0]] == j
    r = rows[0]
    J = np.ctypeslib.as_array(d.efc_J)[r, :27]
    assert J[orc.M["jnt_dofadr"][j]] == 1.0 and np.count_nonzero(J) == 1
    assert d.efc_pos[r] == pytest.approx(-0.005)
    # solimplimit "0 .99 .01" with midpoint .5, power 2: x = .5 -> y = .5 -> imp = d0 + .5 (dmax - d0)
    d0, dmax = 1e-4, 0.99
    assert d.efc_KBIP[r][2] == pytest.approx(d0 + 0.5 * (dmax - d0))


def test_bad_state_autoreset(orc):
    orc.qpos[:] = orc.M["qpos0"]
    orc.qpos[10] = np.nan
    orc.step(None, 1)
    assert orc.d.warning_badqpos == 1
    assert orc.time == pytest.approx(0.005)
    assert np.all(np.isfinite(orc.qpos))


def test_oracle_struct_layout_matches_c():
    from oracle import oracle as O
    L = O.lib()
    assert L.orc_sizeof_model() == C.sizeof(O.OrcModel)
    assert L.orc_sizeof_data() == C.sizeof(O.OrcData)


# ---------------------------------------------------------------- full-state option (cfrc_ext, subtree_linvel)
def _chain_masks(o):
    """dof j moves body b iff j is on b's chain (body_dofadr..dofnum of b and its ancestors)."""
    nb, nv = o.M["nbody"], o.M["nv"]
    parent, adr, num = o.M["body_parentid"], o.M["body_dofadr"], o.M["body_dofnum"]
    on = np.zeros((nb, nv), bool)
    for b in range(1, nb):
        a = b
        while a > 0:
            on[b, adr[a]:adr[a] + num[a]] = True
            a = parent[a]
    return on


@pytest.mark.parametrize("key", ["squat", "prone", "supine"])
def test_cfrc_ext_generalized_force_equals_contact_rows(orc, key):
    """Power identity: sum_b cdof_j . cfrc_ext[b] over the bodies dof j moves == (J_c' f)_j, the
    contact part of qfrc_constraint from the efc Jacobian path (an independent computation)."""
    q = orc.M["keyframes"][key].copy()
    q[2] -= 0.005
    orc.qpos[:] = q
    orc.qvel[:] = np.random.default_rng(3).normal(0, 0.5, 27)
    orc.forward()
    orc.contact_forces()
    d, nv = orc.d, orc.M["nv"]
    ne = d.nefc
    J = np.ctypeslib.as_array(d.efc_J)[:ne, :nv]
    f = np.ctypeslib.as_array(d.efc_force)[:ne]
    typ = np.ctypeslib.as_array(d.efc_type)[:ne]
    contact = typ >= 5
    assert contact.any() and np.abs(f[contact]).max() > 1.0
    expect = J[contact].T @ f[contact]
    cf, cdof, on = orc.get("cfrc_ext"), orc.get("cdof"), _chain_masks(orc)
    got = np.array([sum(cdof[j] @ cf[b] for b in range(1, orc.M["nbody"]) if on[b, j]) for j in range(nv)])
    assert np.allclose(got, expect, rtol=1e-9, atol=1e-9 * np.abs(expect).max())


def test_cfrc_ext_resultant_and_static_equilibrium(orc):
    """Lying still on the floor: the floor's resultant force carries the weight and the com
    velocity vanishes."""
    q = orc.M["keyframes"]["prone"].copy()
    orc.qpos[:] = q
    for _ in range(2000):
        orc.step(None, 1, full=True)
    cf = orc.get("cfrc_ext")
    total = cf[1:, 3:].sum(0)
    mg = orc.M["body_subtreemass"][0] * 9.81
    assert abs(total[2] - mg) < 0.02 * mg and np.abs(total[:2]).max() < 0.02 * mg
    assert np.linalg.norm(orc.get("subtree_linvel")[0]) < 1e-2


def test_subtree_linvel_is_momentum_over_mass():
    """subtree_linvel[0] * M == sum_b (m_b lin_b - (m_b d_b) x ang_b) from cinert/cvel, and with no
    gravity/contacts it stays constant (momentum conservation) over the Euler steps."""
    from oracle.oracle import Oracle
    o = Oracle(XML)
    _strip_model(o, gravity=False)
    q, v = _random_state(o, 9)
    o.qpos[:] = q
    o.qvel[:] = v
    o.forward()
    o.contact_forces()
    p = np.zeros(3)
    for b in range(1, o.M["nbody"]):
        i, vel = o.get("cinert")[b], o.get("cvel")[b]
        p += i[9] * vel[3:] - np.cross(i[6:9], vel[:3])
    M = o.M["body_subtreemass"][0]
    lv0 = o.get("subtree_linvel")[0].copy()
    assert np.allclose(lv0 * M, p, rtol=1e-12, atol=1e-12)
    for _ in range(20):
        o.step(None, 1, full=True)
    # conserved up to semi-implicit Euler's O(h) momentum error (pinned separately above)
    assert np.allclose(o.get("subtree_linvel")[0], lv0, rtol=1e-2, atol=1e-2 * np.abs(lv0).max())


def test_full_flag_off_keeps_reference_zeros(orc):
    orc.qpos[:] = orc.M["keyframes"]["prone"]
    for _ in range(50):
        orc.step(None, 1)
    assert not orc.get("cfrc_ext").any() and not orc.get("subtree_linvel").any()


def _pgs_vs_newton_state(key, seed):
    from oracle.oracle import Oracle, pack_model
    out = []
    for solver in (0, 1):
        o = Oracle(XML)
        o.M = dict(o.M, opt_solver=solver, opt_iterations=20000 if solver else 100, opt_tolerance=1e-30)
        o.m = pack_model(o.M)
        o.reset_data()
        q = o.M["keyframes"][key].copy()
        q[2] -= 0.005
        o.qpos[:] = q
        o.qvel[:] = np.random.default_rng(seed).normal(0, 0.5, 27)
        o.forward()
        ne = o.d.nefc
        out.append((o.arr("efc_force", ne).copy(), o.get("qacc"), o.d.solver_niter, ne))
    return out


@pytest.mark.parametrize("key,seed", [("squat", 1), ("prone", 2), ("supine", 3), ("stand_on_left_leg", 4)])
def test_pgs_and_newton_converge_to_same_forces(key, seed):
    """the primal Newton solver (MuJoCo default, what the reference runs) and
    the dual PGS solver (<option solver="PGS">) solve the same convex problem, so at convergence
    they give the same constraint forces and accelerations -- an independent check of the Newton
    solve that does not reuse its active-set logic."""
    (fn, an, itn, ne), (fp, ap, itp, ne2) = _pgs_vs_newton_state(key, seed)
    assert ne == ne2 and ne > 0 and itp > 10
    scale = max(1.0, np.abs(fn).max())
    # measured: <= 2.4e-12 absolute on forces up to 1.2e3 (Newton 2-5 iterations, PGS 150-20000 sweeps)
    assert np.abs(fp - fn).max() < 1e-9 * scale, np.abs(fp - fn).max()
    assert np.abs(ap - an).max() < 1e-9 * max(1.0, np.abs(an).max())


def test_pgs_stopping_rule_and_option_parsing(tmp_path):
    """<option solver="PGS" iterations tolerance> reaches the oracle; the default tolerance stops
    PGS early (MuJoCo's improvement * scale < tolerance rule), and unknown solvers are rejected."""
    from oracle.model import compile_mjcf
    from oracle.oracle import Oracle
    src = open(XML).read()
    x = tmp_path / "pgs.xml"
    x.write_text(src.replace('<option timestep="0.005"/>', '<option timestep="0.005" solver="PGS" iterations="50"/>'))
    o = Oracle(str(x))
    assert o.m.solver == 1 and o.m.iterations == 50
    q = o.M["keyframes"]["prone"].copy()
    q[2] -= 0.005
    o.qpos[:] = q
    o.forward()
    assert 0 < o.d.solver_niter <= 50 and o.d.nefc > 0
    bad = tmp_path / "cg.xml"
    bad.write_text(src.replace('<option timestep="0.005"/>', '<option timestep="0.005" solver="CG"/>'))
    with pytest.raises(ValueError, match="solver"):
        compile_mjcf(str(bad))


def test_newton_tolerance_stop_gives_the_exact_trajectory():
    """MuJoCo's Newton also stops when scale*improvement or scale*|grad| falls below opt.tolerance
    (1e-8); the oracle (and the kernel) stop at the exact active set.  With the exact line search the
    tolerance rule never fires first: the oracle run with it (orc_variant bit 8) is bitwise the same
    over 300 substeps of random torques with contacts.  (MuJoCo's inexact line search is bit 32:
    test_mujoco_inexact_line_search_agrees_to_round_off.)"""
    from oracle import trajfit as T
    from oracle.oracle import Oracle
    M = T.make_model(XML)
    a, b = Oracle(M=M), Oracle(M=M)
    rng = np.random.default_rng(0)
    noise = rng.uniform(-0.01, 0.01, 27)
    for o in (a, b):
        o.reset_data()
        o.qpos[2] = 1.282
        o.qvel[:] = noise
    try:
        for n in range(300):
            if n % 3 == 0:
                u = rng.uniform(-1, 1, 21)
            T.set_variant(0)
            a.step(u, 1)
            T.set_variant(8)
            b.step(u, 1)
            assert np.array_equal(a.qpos, b.qpos) and np.array_equal(a.qvel, b.qvel), n
    finally:
        T.set_variant(0)
    assert a.d.ncon > 0 or np.abs(a.qpos[2]) < 1.0      # it reached the floor


def test_mujoco_inexact_line_search_agrees_to_round_off():
    """MuJoCo 3.2.5's own Newton iteration (orc_variant 8|32: its Newton-bracketing line search with
    ls_tolerance 0.01 and its opt.tolerance stop, restated in hsim_oracle.c line_search_mujoco)
    against the restatement's exact line search + exact-active-set stop, which the kernel runs.
    From the same mjData at every substep of a random-torque tape with contacts the qacc agree to
    round-off, and the zero-tape trajectories stay far inside the north star's 1e-4 qpos bar
    (profiles/mujoco_linesearch_r5.md has seeds 0-4 over 1000 substeps: <= 3.1e-11)."""
    from oracle.oracle import Oracle
    a, b = Oracle(XML), Oracle(XML)
    rng = np.random.default_rng(0)
    q = a.M["qpos0"].copy()
    q[2], q[3:7] = 1.282, [1, 0, 0, 0]
    q += rng.uniform(-0.01, 0.01, 28) * np.r_[1, 1, 0.1, 0, 0, 0, 0, np.ones(21)]
    v = rng.uniform(-0.01, 0.01, 27)
    var = C.c_int.in_dll(a.lib, "orc_variant")
    evals = C.c_long.in_dll(a.lib, "orc_stat_ls_evals")
    e0 = evals.value
    a.qpos[:], a.qvel[:] = q, v
    worst, ncon = 0.0, 0
    try:
        for n in range(150):
            u = rng.uniform(-1, 1, 21)
            C.memmove(C.byref(b.d), C.byref(a.d), C.sizeof(a.d))
            var.value = 8 | 32
            b.step(u, 1)
            var.value = 0
            a.step(u, 1)
            qa = a.get("qacc")
            worst = max(worst, np.abs(b.get("qacc") - qa).max() / max(1.0, np.abs(qa).max()))
            ncon = max(ncon, a.d.ncon)
        assert ncon > 0 and evals.value > e0          # contacts were active, and bit 32 ran
        assert worst < 1e-12, worst
        za, zb = Oracle(XML), Oracle(XML)
        for o in (za, zb):
            o.qpos[:], o.qvel[:] = q, v
        dq = 0.0
        for n in range(300):
            var.value = 8 | 32
            zb.step(None, 1)
            var.value = 0
            za.step(None, 1)
            dq = max(dq, np.abs(za.qpos - zb.qpos).max())
        assert dq < 1e-9, dq
    finally:
        var.value = 0


def test_fp32_state_storage_alone_breaks_the_1e4_bound_through_contact_flips():
    """Why the fp32 engine cannot hold the north star's < 1e-4 over 1000 substeps:
    the fp64 oracle with NOTHING but its state rounded to fp32 after every substep (exact arithmetic
    otherwise) already drifts to ~2e-4 by smooth amplification of that rounding, and then a resting
    contact at distance ~0 (a capsule end-point at -1.7e-6) is in one run's contact set and not the
    other's: from that substep on the runs differ by > 1e-3.  Zero tape, the initial state of
    tools/probes/parity_report.py seed 1 (first flip at substep 375)."""
    from oracle.oracle import Oracle
    _oracle = lambda: Oracle(XML)  # noqa: E731
    o = _oracle()
    rng = np.random.default_rng(1)
    q = o.M["qpos0"].copy()
    q[2], q[3:7] = 1.282, [1, 0, 0, 0]
    q += rng.uniform(-0.01, 0.01, 28) * np.r_[1, 1, 0.1, 0, 0, 0, 0, np.ones(21)]
    v = rng.uniform(-0.01, 0.01, 27)
    a, b = _oracle(), _oracle()
    a.qpos[:], a.qvel[:] = q, v
    b.qpos[:], b.qvel[:] = q.astype(np.float32), v.astype(np.float32)
    first_flip, before, worst = None, 0.0, 0.0
    for s in range(1000):
        a.step(np.zeros(21), 1)
        b.step(np.zeros(21), 1)
        b.qpos[:] = b.qpos.astype(np.float32)
        b.qvel[:] = b.qvel.astype(np.float32)
        d = float(np.abs(a.qpos - b.qpos).max())
        if first_flip is None and (a.d.ncon, a.d.nefc) != (b.d.ncon, b.d.nefc):
            first_flip = s
        if first_flip is None:
            before = max(before, d)
        worst = max(worst, d)
    assert first_flip is not None
    assert before < 1e-3           # fp32-storage round-off, amplified smoothly, until the flip
    assert worst > 1e-3 and worst > 10 * before      # ... and a jump past the north star's bound


def test_precision_emulation_build_mask0_is_the_oracle_bitwise():
    """oracle/precision.py (the restatement with chosen stages rounded to fp32) with no stage
    selected steps bitwise like the plain build, so its per-stage results isolate rounding."""
    from oracle import precision as P
    from oracle.oracle import Oracle
    a, b = Oracle(XML), P.PrecOracle(XML)
    rng = np.random.default_rng(2)
    v = rng.uniform(-0.5, 0.5, 27)
    for o in (a, b):
        o.qpos[2] = 1.25
        o.qvel[:] = v
    P.set_mask(0)
    for _ in range(60):
        u = rng.uniform(-1, 1, 21)
        a.step(u, 1)
        b.step(u, 1)
    assert np.array_equal(a.qpos, b.qpos) and np.array_equal(a.qvel, b.qvel)
    P.set_mask(P.ALL)
    b.step(u, 1)
    a.step(u, 1)
    P.set_mask(0)
    d = np.abs(a.qvel - b.qvel).max()
    assert 0 < d < 1e-2 * (1 + np.abs(a.qvel).max())       # fp32 arithmetic: close, not equal


def test_mixed_precision_newton_gate_fails():
    """The round-5 CPU gate for an fp32 Hessian / Cholesky / triangular-solve Newton under fp64
    state, gradient and line search (tools/probes/mixed_newton_gate.py, profiles/mixed_newton_r5.md):
    the fp32 factor with the exact-active-set stop leaves the zero tape above 1e-6 (contact flips),
    and as a preconditioner it needs more than one extra Newton iteration per substep to reach the
    kernel's 1e-13 stop.  So the kernel keeps its fp64 solve."""
    import mixed_newton_gate as G
    from oracle import precision as P
    o = P.PrecOracle(XML)
    HC = P.mask_of(["solver_hessian", "solver_cholesky"])
    q, v, rng = G.initial(o.M, 4)
    zero = np.zeros((G.NSUB, 21), np.float32)
    ref, it0, _ = G.run(o, q, v, zero, (0, 0))
    norefine, it1, _ = G.run(o, q, v, zero, (HC, 0))
    refine, it2, nf2 = G.run(o, q, v, zero, (HC, 16, 1e-13))
    assert np.abs(norefine - ref).max() > 1e-6
    assert np.abs(refine - ref).max() < 1e-8
    assert abs(it1 - it0) < 0.1 and abs(nf2 - it0) < 0.1      # same factorizations as the exact solve
    assert it2 - it0 > 1.0                                    # ... plus more than one refinement each

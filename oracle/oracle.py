"""ORACLE (test infrastructure only): ctypes binding of the fp64 C restatement of mj_step.

Only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline`` leg may
import this module.  It never backs the product path.
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess

import numpy as np

from .model import compile_mjcf

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "build", "libhsim_oracle.so")
# a prebuilt variant to load instead (tests/test_sanitizers.py: the ASan/UBSan build of the same C)
LIB_OVERRIDE = os.environ.get("HSIM_ORACLE_LIB")

OMAXB, OMAXJ, OMAXV, OMAXQ, OMAXG, OMAXT, OMAXW, OMAXU = 32, 32, 40, 48, 32, 8, 32, 32
OMAXCON, OMAXEFC, OMAXPAIR = 160, 640, 512

D, I = C.c_double, C.c_int


def _a(t, *dims):
    for n in reversed(dims):
        t = t * n
    return t


class OrcModel(C.Structure):
    _fields_ = [
        ("nq", I), ("nv", I), ("nu", I), ("nbody", I), ("njnt", I), ("ngeom", I), ("ntendon", I), ("npair", I),
        ("timestep", D), ("gravity", _a(D, 3)), ("impratio", D), ("tolerance", D), ("meaninertia", D),
        ("iterations", I), ("solver", I),
        ("body_parentid", _a(I, OMAXB)), ("body_rootid", _a(I, OMAXB)), ("body_weldid", _a(I, OMAXB)),
        ("body_jntnum", _a(I, OMAXB)), ("body_jntadr", _a(I, OMAXB)), ("body_dofnum", _a(I, OMAXB)),
        ("body_dofadr", _a(I, OMAXB)),
        ("body_pos", _a(D, OMAXB, 3)), ("body_quat", _a(D, OMAXB, 4)), ("body_ipos", _a(D, OMAXB, 3)),
        ("body_inertia_full", _a(D, OMAXB, 9)),
        ("body_mass", _a(D, OMAXB)), ("body_subtreemass", _a(D, OMAXB)), ("body_invweight0", _a(D, OMAXB, 2)),
        ("jnt_type", _a(I, OMAXJ)), ("jnt_qposadr", _a(I, OMAXJ)), ("jnt_dofadr", _a(I, OMAXJ)),
        ("jnt_bodyid", _a(I, OMAXJ)), ("jnt_limited", _a(I, OMAXJ)),
        ("jnt_pos", _a(D, OMAXJ, 3)), ("jnt_axis", _a(D, OMAXJ, 3)), ("jnt_range", _a(D, OMAXJ, 2)),
        ("jnt_stiffness", _a(D, OMAXJ)),
        ("jnt_solref", _a(D, OMAXJ, 2)), ("jnt_solimp", _a(D, OMAXJ, 5)), ("jnt_margin", _a(D, OMAXJ)),
        ("dof_bodyid", _a(I, OMAXV)), ("dof_jntid", _a(I, OMAXV)), ("dof_parentid", _a(I, OMAXV)),
        ("dof_armature", _a(D, OMAXV)), ("dof_damping", _a(D, OMAXV)), ("dof_invweight0", _a(D, OMAXV)),
        ("qpos0", _a(D, OMAXQ)), ("qpos_spring", _a(D, OMAXQ)),
        ("geom_type", _a(I, OMAXG)), ("geom_bodyid", _a(I, OMAXG)), ("geom_condim", _a(I, OMAXG)),
        ("geom_priority", _a(I, OMAXG)),
        ("geom_size", _a(D, OMAXG, 3)), ("geom_pos", _a(D, OMAXG, 3)), ("geom_quat", _a(D, OMAXG, 4)),
        ("geom_friction", _a(D, OMAXG, 3)),
        ("geom_solref", _a(D, OMAXG, 2)), ("geom_solimp", _a(D, OMAXG, 5)), ("geom_margin", _a(D, OMAXG)),
        ("geom_gap", _a(D, OMAXG)),
        ("geom_solmix", _a(D, OMAXG)), ("geom_rbound", _a(D, OMAXG)),
        ("tendon_adr", _a(I, OMAXT)), ("tendon_num", _a(I, OMAXT)), ("tendon_limited", _a(I, OMAXT)),
        ("tendon_range", _a(D, OMAXT, 2)), ("tendon_solref", _a(D, OMAXT, 2)), ("tendon_solimp", _a(D, OMAXT, 5)),
        ("tendon_margin", _a(D, OMAXT)), ("tendon_invweight0", _a(D, OMAXT)),
        ("wrap_jnt", _a(I, OMAXW)), ("wrap_coef", _a(D, OMAXW)),
        ("actuator_trnid", _a(I, OMAXU)), ("actuator_ctrllimited", _a(I, OMAXU)),
        ("actuator_gear", _a(D, OMAXU)), ("actuator_ctrlrange", _a(D, OMAXU, 2)),
        ("pair_geom", _a(I, OMAXPAIR, 2)),
    ]


class OrcContact(C.Structure):
    _fields_ = [("pos", _a(D, 3)), ("frame", _a(D, 9)), ("dist", D), ("includemargin", D),
                ("friction", _a(D, 5)), ("solref", _a(D, 2)), ("solimp", _a(D, 5)),
                ("geom", _a(I, 2)), ("dim", I), ("efc_address", I)]


class OrcData(C.Structure):
    _fields_ = [
        ("time", D),
        ("qpos", _a(D, OMAXQ)), ("qvel", _a(D, OMAXV)), ("ctrl", _a(D, OMAXU)), ("qacc_warmstart", _a(D, OMAXV)),
        ("qacc", _a(D, OMAXV)), ("qacc_smooth", _a(D, OMAXV)),
        ("xpos", _a(D, OMAXB, 3)), ("xquat", _a(D, OMAXB, 4)), ("xmat", _a(D, OMAXB, 9)),
        ("xipos", _a(D, OMAXB, 3)), ("ximat", _a(D, OMAXB, 9)),
        ("xanchor", _a(D, OMAXJ, 3)), ("xaxis", _a(D, OMAXJ, 3)), ("geom_xpos", _a(D, OMAXG, 3)),
        ("geom_xmat", _a(D, OMAXG, 9)),
        ("subtree_com", _a(D, OMAXB, 3)), ("cinert", _a(D, OMAXB, 10)), ("cdof", _a(D, OMAXV, 6)),
        ("cvel", _a(D, OMAXB, 6)), ("cdof_dot", _a(D, OMAXV, 6)),
        ("crb", _a(D, OMAXB, 10)),
        ("qM", _a(D, OMAXV, OMAXV)),
        ("ten_length", _a(D, OMAXT)), ("ten_J", _a(D, OMAXT, OMAXV)),
        ("actuator_force", _a(D, OMAXU)),
        ("qfrc_bias", _a(D, OMAXV)), ("qfrc_passive", _a(D, OMAXV)), ("qfrc_actuator", _a(D, OMAXV)),
        ("qfrc_smooth", _a(D, OMAXV)),
        ("qfrc_constraint", _a(D, OMAXV)),
        ("cfrc_ext", _a(D, OMAXB, 6)), ("subtree_linvel", _a(D, OMAXB, 3)),
        ("ncon", I),
        ("contact", OrcContact * OMAXCON),
        ("nefc", I),
        ("efc_type", _a(I, OMAXEFC)), ("efc_id", _a(I, OMAXEFC)),
        ("efc_J", _a(D, OMAXEFC, OMAXV)),
        ("efc_pos", _a(D, OMAXEFC)), ("efc_margin", _a(D, OMAXEFC)), ("efc_vel", _a(D, OMAXEFC)),
        ("efc_aref", _a(D, OMAXEFC)),
        ("efc_R", _a(D, OMAXEFC)), ("efc_D", _a(D, OMAXEFC)), ("efc_diagApprox", _a(D, OMAXEFC)),
        ("efc_KBIP", _a(D, OMAXEFC, 4)),
        ("efc_force", _a(D, OMAXEFC)),
        ("solver_niter", I),
        ("warning_badqpos", I), ("warning_badqvel", I), ("warning_badqacc", I), ("warning_overflow", I),
    ]


def build(force=False):
    """Compile the C restatement with gcc into oracle/build/ (checker build, not product)."""
    if LIB_OVERRIDE:
        return LIB_OVERRIDE
    src = os.path.join(HERE, "hsim_oracle.c")
    if force or not os.path.exists(LIB_PATH) or os.path.getmtime(LIB_PATH) < os.path.getmtime(src):
        os.makedirs(os.path.dirname(LIB_PATH), exist_ok=True)
        tmp = f"{LIB_PATH}.{os.getpid()}.tmp"     # atomic: parallel test workers may build at once
        subprocess.check_call(["gcc", "-O2", "-fPIC", "-shared", "-std=c11", "-o", tmp, src, "-lm"])
        os.replace(tmp, LIB_PATH)
    return LIB_PATH


_LIB = None


def lib():
    global _LIB
    if _LIB is None:
        _LIB = C.CDLL(build())
        for fn in ("orc_reset_data", "orc_forward", "orc_step"):
            getattr(_LIB, fn).argtypes = [C.c_void_p, C.c_void_p]
            getattr(_LIB, fn).restype = None
        _LIB.orc_step_n.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p, C.c_int]
        _LIB.orc_step_n.restype = None
        _LIB.orc_step_n_full.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p, C.c_int, C.c_int]
        _LIB.orc_step_n_full.restype = None
        _LIB.orc_contact_forces.argtypes = [C.c_void_p, C.c_void_p]
        _LIB.orc_contact_forces.restype = None
        assert _LIB.orc_sizeof_model() == C.sizeof(OrcModel), "OrcModel layout mismatch"
        assert _LIB.orc_sizeof_data() == C.sizeof(OrcData), "OrcData layout mismatch"
    return _LIB


def _fill(dst, arr):
    a = np.asarray(arr)
    view = np.ctypeslib.as_array(dst)
    if a.ndim == 1 and view.ndim == 2:
        a = a.reshape(-1, view.shape[1])
    view[tuple(slice(0, n) for n in a.shape)] = a


def pack_model(M):
    om = OrcModel()
    for k in ("nq", "nv", "nu", "nbody", "njnt", "ngeom", "ntendon"):
        setattr(om, k, int(M[k]))
    om.npair = len(M["collision_pairs"])
    om.timestep = M["opt_timestep"]
    _fill(om.gravity, M["opt_gravity"])
    om.impratio = M["opt_impratio"]
    om.tolerance = M["opt_tolerance"]
    om.meaninertia = M["stat_meaninertia"]
    om.iterations = M["opt_iterations"]
    om.solver = M.get("opt_solver", 0)
    for k in ("body_parentid", "body_rootid", "body_weldid", "body_jntnum", "body_jntadr", "body_dofnum",
              "body_dofadr", "body_pos", "body_quat", "body_ipos", "body_mass", "body_subtreemass",
              "body_invweight0", "jnt_type", "jnt_qposadr", "jnt_dofadr", "jnt_bodyid", "jnt_limited",
              "jnt_pos", "jnt_axis", "jnt_range", "jnt_stiffness", "jnt_solref", "jnt_solimp", "jnt_margin",
              "dof_bodyid", "dof_jntid", "dof_parentid", "dof_armature", "dof_damping", "dof_invweight0",
              "qpos0", "qpos_spring", "geom_type", "geom_bodyid", "geom_condim", "geom_priority", "geom_size",
              "geom_pos", "geom_quat", "geom_friction", "geom_solref", "geom_solimp", "geom_margin", "geom_gap",
              "geom_solmix", "geom_rbound", "tendon_adr", "tendon_num", "tendon_limited", "tendon_range",
              "tendon_solref", "tendon_solimp", "tendon_margin", "tendon_invweight0", "wrap_jnt", "wrap_coef",
              "actuator_trnid", "actuator_ctrllimited", "actuator_gear", "actuator_ctrlrange"):
        if len(np.asarray(M[k]).ravel()):
            _fill(getattr(om, k), M[k])
    _fill(om.body_inertia_full, np.asarray(M["body_inertia_full"]).reshape(M["nbody"], 9))
    _fill(om.pair_geom, M["collision_pairs"])
    return om


class Oracle:
    """One fp64 CPU humanoid instance (an MjModel/MjData pair restated)."""

    def __init__(self, model_path=None, M=None):
        self.M = M if M is not None else compile_mjcf(model_path)
        self.m = pack_model(self.M)
        self.d = OrcData()
        self.lib = lib()
        self.reset_data()

    # views
    def arr(self, name, n=None):
        a = np.ctypeslib.as_array(getattr(self.d, name))
        return a if n is None else a[:n]

    @property
    def qpos(self):
        return self.arr("qpos", self.M["nq"])

    @property
    def qvel(self):
        return self.arr("qvel", self.M["nv"])

    @property
    def ctrl(self):
        return self.arr("ctrl", self.M["nu"])

    @property
    def time(self):
        return self.d.time

    def reset_data(self):
        self.lib.orc_reset_data(C.byref(self.m), C.byref(self.d))

    def forward(self):
        self.lib.orc_forward(C.byref(self.m), C.byref(self.d))

    def step(self, ctrl=None, nsub=1, full=False):
        """nsub x mj_step; full=True also computes cfrc_ext / subtree_linvel after mj_forward
        (hsim's full_state option; zeros otherwise, as in the reference)."""
        c = np.zeros(self.M["nu"]) if ctrl is None else np.ascontiguousarray(ctrl, dtype=np.float64)
        self.lib.orc_step_n_full(C.byref(self.m), C.byref(self.d), c.ctypes.data, int(nsub), int(bool(full)))

    def contact_forces(self):
        """cfrc_ext / subtree_linvel of the current (forward) state."""
        self.lib.orc_contact_forces(C.byref(self.m), C.byref(self.d))

    def get(self, name):
        nb, nv, nj, ng = self.M["nbody"], self.M["nv"], self.M["njnt"], self.M["ngeom"]
        sizes = {"xpos": nb, "xquat": nb, "xmat": nb, "xipos": nb, "subtree_com": nb, "cinert": nb, "cvel": nb,
                 "cdof": nv, "cdof_dot": nv, "qacc": nv, "qacc_smooth": nv, "qfrc_bias": nv, "qfrc_passive": nv,
                 "qfrc_actuator": nv, "qfrc_smooth": nv, "qfrc_constraint": nv, "xanchor": nj, "xaxis": nj,
                 "geom_xpos": ng, "geom_xmat": ng, "cfrc_ext": nb, "subtree_linvel": nb, "crb": nb,
                 "ten_length": self.M["ntendon"]}
        if name == "qM":
            return np.ctypeslib.as_array(self.d.qM)[:nv, :nv].copy()
        return self.arr(name)[:sizes[name]].copy()

    def contacts(self):
        out = []
        for i in range(self.d.ncon):
            c = self.d.contact[i]
            out.append(dict(pos=np.array(c.pos), frame=np.array(c.frame), dist=c.dist, geom=(c.geom[0], c.geom[1]),
                            dim=c.dim, friction=np.array(c.friction), solref=np.array(c.solref),
                            solimp=np.array(c.solimp), efc_address=c.efc_address))
        return out

"""ORACLE (test infrastructure only) -- independent MJCF compiler for the humanoid.xml subset.

This file is part of the *checker*, never the product: only ``tests/``,
``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline`` leg may import it.

It restates what MuJoCo 3.2.5's compiler (``mj_loadXML`` -> ``mjCModel::Compile`` ->
``mj_setConst``) produces for the constructs used by the reference model
``XML/humanoid.xml`` (the file ``custom_env.py:53`` loads via ``MjModel.from_xml_path``):

* ``<default>`` classes with nesting, ``childclass`` / ``class`` resolution
  (humanoid.xml:35-102, childclass at :110);
* bodies with ``pos`` (:110-181), hinge joints with ``pos/axis/range`` in degrees
  (compiler default ``angle="degree"``), ``<freejoint>`` (:111; stiffness/damping/armature
  forced to 0 by the MJCF shortcut);
* capsule (``fromto``), sphere and plane geoms; ``inertiafromgeom`` with density 1000
  and the exact capsule / sphere inertia formulas; body principal inertia;
* fixed tendons (:191-200), motor actuators with gear (:202-224), contact excludes
  (:186-189), keyframes (:226-266);
* ``mj_setConst`` quantities: ``body_invweight0``, ``dof_invweight0``,
  ``tendon_invweight0``, ``stat.meaninertia`` (computed at ``qpos0``).

MuJoCo itself is not importable in this container so the compiled
values are "parity unpinned" against real MuJoCo; they are pinned instead by analytic
mass / inertia formulas in ``tests/test_model.py`` and cross-checked against the
product's independent C++ compiler.
"""
from __future__ import annotations

import math
import xml.etree.ElementTree as ET

import numpy as np

MINVAL = 1e-15
# geom types (mjtGeom ordering: plane=0, hfield=1, sphere=2, capsule=3, ...)
GEOM_PLANE, GEOM_SPHERE, GEOM_CAPSULE = 0, 2, 3
JNT_FREE, JNT_HINGE = 0, 3

# MuJoCo built-in defaults (mjs default element values)
GEOM_DEFAULTS = dict(type="sphere", condim=3, contype=1, conaffinity=1, friction=(1.0, 0.005, 0.0001),
                     solref=(0.02, 1.0), solimp=(0.9, 0.95, 0.001, 0.5, 2.0), margin=0.0, gap=0.0,
                     solmix=1.0, priority=0, density=1000.0, size=(0.0, 0.0, 0.0))
JOINT_DEFAULTS = dict(type="hinge", pos=(0.0, 0.0, 0.0), axis=(0.0, 0.0, 1.0), range=(0.0, 0.0),
                      limited="auto", damping=0.0, stiffness=0.0, armature=0.0, springref=0.0,
                      solreflimit=(0.02, 1.0), solimplimit=(0.9, 0.95, 0.001, 0.5, 2.0), margin=0.0)
MOTOR_DEFAULTS = dict(gear=(1.0, 0, 0, 0, 0, 0), ctrlrange=(0.0, 0.0), ctrllimited="auto")
TENDON_DEFAULTS = dict(range=(0.0, 0.0), limited="auto", solreflimit=(0.02, 1.0),
                       solimplimit=(0.9, 0.95, 0.001, 0.5, 2.0), margin=0.0)


def _floats(s):
    return tuple(float(x) for x in s.split())


# ----------------------------------------------------------------------------- quaternion helpers
def quat_mul(a, b):
    w1, x1, y1, z1 = a
    w2, x2, y2, z2 = b
    return np.array([w1 * w2 - x1 * x2 - y1 * y2 - z1 * z2,
                     w1 * x2 + x1 * w2 + y1 * z2 - z1 * y2,
                     w1 * y2 - x1 * z2 + y1 * w2 + z1 * x2,
                     w1 * z2 + x1 * y2 - y1 * x2 + z1 * w2])


def quat2mat(q):
    w, x, y, z = q
    return np.array([[1 - 2 * (y * y + z * z), 2 * (x * y - w * z), 2 * (x * z + w * y)],
                     [2 * (x * y + w * z), 1 - 2 * (x * x + z * z), 2 * (y * z - w * x)],
                     [2 * (x * z - w * y), 2 * (y * z + w * x), 1 - 2 * (x * x + y * y)]])


def quat_z2vec(vec):
    """mju_quatZ2Vec: minimal rotation taking +z to ``vec``."""
    q = np.array([1.0, 0.0, 0.0, 0.0])
    v = np.asarray(vec, float)
    n = np.linalg.norm(v)
    if n < MINVAL:
        return q
    v = v / n
    axis = np.cross([0.0, 0.0, 1.0], v)
    a = np.linalg.norm(axis)
    if abs(a) < MINVAL:
        if v[2] < 0:
            return np.array([0.0, 1.0, 0.0, 0.0])
        return q
    axis = axis / a
    ang = math.atan2(a, v[2])
    return np.array([math.cos(ang / 2), *(axis * math.sin(ang / 2))])


def mat2quat(R):
    """Rotation matrix -> unit quaternion (w >= 0)."""
    t = np.trace(R)
    if t > 0:
        s = math.sqrt(t + 1.0) * 2
        q = [0.25 * s, (R[2, 1] - R[1, 2]) / s, (R[0, 2] - R[2, 0]) / s, (R[1, 0] - R[0, 1]) / s]
    elif R[0, 0] > R[1, 1] and R[0, 0] > R[2, 2]:
        s = math.sqrt(1.0 + R[0, 0] - R[1, 1] - R[2, 2]) * 2
        q = [(R[2, 1] - R[1, 2]) / s, 0.25 * s, (R[0, 1] + R[1, 0]) / s, (R[0, 2] + R[2, 0]) / s]
    elif R[1, 1] > R[2, 2]:
        s = math.sqrt(1.0 + R[1, 1] - R[0, 0] - R[2, 2]) * 2
        q = [(R[0, 2] - R[2, 0]) / s, (R[0, 1] + R[1, 0]) / s, 0.25 * s, (R[1, 2] + R[2, 1]) / s]
    else:
        s = math.sqrt(1.0 + R[2, 2] - R[0, 0] - R[1, 1]) * 2
        q = [(R[1, 0] - R[0, 1]) / s, (R[0, 2] + R[2, 0]) / s, (R[1, 2] + R[2, 1]) / s, 0.25 * s]
    q = np.array(q)
    q /= np.linalg.norm(q)
    return q if q[0] >= 0 else -q


# ----------------------------------------------------------------------------- geom mass properties
def geom_mass_inertia(gtype, size, density):
    """Exact solid mass / principal inertia (geom frame) -- MuJoCo mjCGeom::SetInertia."""
    if gtype == GEOM_SPHERE:
        r = size[0]
        m = density * 4.0 / 3.0 * math.pi * r ** 3
        i = 0.4 * m * r * r
        return m, np.array([i, i, i])
    if gtype == GEOM_CAPSULE:
        r, h = size[0], 2.0 * size[1]
        ms = density * 4.0 / 3.0 * math.pi * r ** 3
        mc = density * math.pi * r * r * h
        ixx = mc * (3 * r * r + h * h) / 12.0 + ms * (0.4 * r * r + h * h / 4.0 + 3.0 * h * r / 8.0)
        izz = mc * r * r / 2.0 + ms * 0.4 * r * r
        return ms + mc, np.array([ixx, ixx, izz])
    return 0.0, np.zeros(3)


class _Defaults:
    """One MJCF default class: per-element attribute dictionaries, inherited from parent."""

    def __init__(self, parent=None):
        self.attrs = {k: dict(v) for k, v in parent.attrs.items()} if parent else \
            {"geom": {}, "joint": {}, "motor": {}, "tendon": {}}


def compile_mjcf(path):
    """Compile humanoid.xml (subset) into a dict of numpy arrays with MuJoCo field names."""
    root = ET.parse(path).getroot()
    classes = {}

    def parse_default(el, parent):
        d = _Defaults(parent)
        for child in el:
            if child.tag in ("geom", "joint", "motor", "tendon"):
                d.attrs[child.tag].update(child.attrib)
        classes[el.get("class", "main")] = d
        for child in el:
            if child.tag == "default":
                parse_default(child, d)

    top = root.find("default")
    if top is not None:
        parse_default(top, None)
    else:
        classes["main"] = _Defaults()

    def resolve(tag, el, cls):
        base = {"geom": GEOM_DEFAULTS, "joint": JOINT_DEFAULTS, "motor": MOTOR_DEFAULTS,
                "tendon": TENDON_DEFAULTS}[tag]
        out = dict(base)
        c = el.get("class", cls)
        for k, v in classes[c].attrs[tag].items():
            out[k] = v
        for k, v in el.attrib.items():
            out[k] = v
        return out

    opt = root.find("option")
    o = opt.attrib if opt is not None else {}
    timestep = float(o.get("timestep", 0.002))
    gravity = np.array([float(x) for x in o.get("gravity", "0 0 -9.81").split()])
    iterations = int(float(o.get("iterations", 100)))
    tolerance = float(o.get("tolerance", 1e-8))
    solvers = {"Newton": 0, "PGS": 1}
    if o.get("solver", "Newton") not in solvers:
        raise ValueError("only solver='Newton' (MuJoCo default) or 'PGS' is supported")
    solver = solvers[o.get("solver", "Newton")]
    # options that change the dynamics beyond what the restatement covers are rejected, not ignored
    if o.get("integrator", "Euler") != "Euler":
        raise ValueError("only integrator='Euler' is supported")
    if o.get("cone", "pyramidal") != "pyramidal":
        raise ValueError("only cone='pyramidal' is supported")
    if float(o.get("impratio", 1)) != 1:
        raise ValueError("only impratio=1 is supported")
    if float(o.get("noslip_iterations", 0)) != 0:
        raise ValueError("noslip solver not supported")
    if float(o.get("density", 0)) != 0 or float(o.get("viscosity", 0)) != 0:
        raise ValueError("fluid forces not supported")
    if opt is not None:
        for f in opt.findall("flag"):
            for a in f.attrib:
                if a != "energy":
                    raise ValueError(f"<option><flag {a}> not supported")

    bodies = [dict(name="world", parent=-1, pos=np.zeros(3), quat=np.array([1.0, 0, 0, 0]))]
    joints, geoms = [], []

    def vec(a, n, default):
        return np.array(_floats(a), float) if isinstance(a, str) else np.array(default if a is None else a, float)

    def add_geom(el, body_id, cls):
        a = resolve("geom", el, cls)
        gtype = {"plane": GEOM_PLANE, "sphere": GEOM_SPHERE, "capsule": GEOM_CAPSULE}[a["type"]]
        size = np.zeros(3)
        s = _floats(a["size"]) if isinstance(a["size"], str) else a["size"]
        size[:len(s)] = s
        pos = np.zeros(3)
        quat = np.array([1.0, 0, 0, 0])
        if "fromto" in a:
            ft = np.array(_floats(a["fromto"]))
            p0, p1 = ft[:3], ft[3:]
            pos = 0.5 * (p0 + p1)
            quat = quat_z2vec(p1 - p0)
            size[1] = 0.5 * np.linalg.norm(p1 - p0)
        else:
            if "pos" in a:
                pos = np.array(_floats(a["pos"]))
            if "zaxis" in a:
                quat = quat_z2vec(np.array(_floats(a["zaxis"])))
        fr = _floats(a["friction"]) if isinstance(a["friction"], str) else a["friction"]
        fr = list(fr) + list(GEOM_DEFAULTS["friction"][len(fr):])
        sr = _floats(a["solref"]) if isinstance(a["solref"], str) else a["solref"]
        si = _floats(a["solimp"]) if isinstance(a["solimp"], str) else a["solimp"]
        si = list(si) + list(GEOM_DEFAULTS["solimp"][len(si):])
        geoms.append(dict(name=el.get("name", ""), type=gtype, body=body_id, size=size, pos=pos, quat=quat,
                          condim=int(a["condim"]), contype=int(a["contype"]), conaffinity=int(a["conaffinity"]),
                          friction=np.array(fr), solref=np.array(sr), solimp=np.array(si),
                          margin=float(a["margin"]), gap=float(a["gap"]), solmix=float(a["solmix"]),
                          priority=int(a["priority"]), density=float(a["density"])))

    def add_joint(el, body_id, cls, free=False):
        if free:
            joints.append(dict(name=el.get("name", ""), type=JNT_FREE, body=body_id, pos=np.zeros(3),
                               axis=np.array([0.0, 0, 1]), range=np.zeros(2), limited=0, damping=0.0,
                               stiffness=0.0, armature=0.0, springref=0.0, solref=np.array([0.02, 1.0]),
                               solimp=np.array(JOINT_DEFAULTS["solimplimit"]), margin=0.0))
            return
        a = resolve("joint", el, cls)
        assert a["type"] == "hinge", a["type"]
        axis = vec(a["axis"], 3, None)
        axis = axis / np.linalg.norm(axis)
        rng = np.radians(vec(a["range"], 2, None))
        lim = a["limited"]
        limited = int(lim == "true" or (lim == "auto" and rng[0] < rng[1]))
        si = list(_floats(a["solimplimit"]) if isinstance(a["solimplimit"], str) else a["solimplimit"])
        si += list(JOINT_DEFAULTS["solimplimit"][len(si):])
        sr = _floats(a["solreflimit"]) if isinstance(a["solreflimit"], str) else a["solreflimit"]
        joints.append(dict(name=el.get("name", ""), type=JNT_HINGE, body=body_id, pos=vec(a["pos"], 3, None),
                           axis=axis, range=rng, limited=limited, damping=float(a["damping"]),
                           stiffness=float(a["stiffness"]), armature=float(a["armature"]),
                           springref=math.radians(float(a["springref"])), solref=np.array(sr),
                           solimp=np.array(si), margin=float(a["margin"])))

    def walk(el, parent_id, cls):
        for child in el:
            if child.tag == "geom":
                add_geom(child, parent_id, cls)
        for child in el:
            if child.tag == "body":
                bid = len(bodies)
                pos = np.array(_floats(child.get("pos", "0 0 0")))
                quat = np.array(_floats(child.get("quat", "1 0 0 0")))
                quat = quat / np.linalg.norm(quat)
                bodies.append(dict(name=child.get("name", ""), parent=parent_id, pos=pos, quat=quat))
                ccls = child.get("childclass", cls)
                for j in child:
                    if j.tag == "freejoint":
                        add_joint(j, bid, ccls, free=True)
                    elif j.tag == "joint":
                        add_joint(j, bid, ccls)
                walk(child, bid, ccls)

    walk(root.find("worldbody"), 0, "main")

    # MuJoCo orders bodies depth-first in XML order (already), joints by body, geoms by body.
    # Our walk adds a body's geoms before descending, so geoms are grouped by body in order.
    nbody, njnt, ngeom = len(bodies), len(joints), len(geoms)
    M = {}
    M["opt_timestep"] = timestep
    M["opt_gravity"] = gravity
    M["opt_impratio"] = 1.0
    M["opt_tolerance"] = tolerance
    M["opt_iterations"] = iterations
    M["opt_solver"] = solver
    M["opt_ls_iterations"] = 50
    M["nbody"], M["njnt"], M["ngeom"] = nbody, njnt, ngeom
    M["body_name"] = [b["name"] for b in bodies]
    M["body_parentid"] = np.array([b["parent"] for b in bodies], np.int32)
    M["body_pos"] = np.array([b["pos"] for b in bodies])
    M["body_quat"] = np.array([b["quat"] for b in bodies])

    # joints / dofs / qpos addresses
    jnt_qposadr, jnt_dofadr, dof_jnt = [], [], []
    nq = nv = 0
    for j in joints:
        jnt_qposadr.append(nq)
        jnt_dofadr.append(nv)
        if j["type"] == JNT_FREE:
            nq += 7
            dof_jnt += [len(jnt_dofadr) - 1] * 6
            nv += 6
        else:
            nq += 1
            dof_jnt.append(len(jnt_dofadr) - 1)
            nv += 1
    M["nq"], M["nv"] = nq, nv
    M["jnt_name"] = [j["name"] for j in joints]
    M["jnt_type"] = np.array([j["type"] for j in joints], np.int32)
    M["jnt_bodyid"] = np.array([j["body"] for j in joints], np.int32)
    M["jnt_qposadr"] = np.array(jnt_qposadr, np.int32)
    M["jnt_dofadr"] = np.array(jnt_dofadr, np.int32)
    M["jnt_pos"] = np.array([j["pos"] for j in joints])
    M["jnt_axis"] = np.array([j["axis"] for j in joints])
    M["jnt_range"] = np.array([j["range"] for j in joints])
    M["jnt_limited"] = np.array([j["limited"] for j in joints], np.int32)
    M["jnt_stiffness"] = np.array([j["stiffness"] for j in joints])
    M["jnt_solref"] = np.array([j["solref"] for j in joints])
    M["jnt_solimp"] = np.array([j["solimp"] for j in joints])
    M["jnt_margin"] = np.array([j["margin"] for j in joints])
    M["dof_jntid"] = np.array(dof_jnt, np.int32)
    M["dof_bodyid"] = M["jnt_bodyid"][M["dof_jntid"]]
    M["dof_armature"] = np.array([joints[j]["armature"] for j in dof_jnt])
    M["dof_damping"] = np.array([joints[j]["damping"] for j in dof_jnt])

    body_jntadr = np.full(nbody, -1, np.int32)
    body_jntnum = np.zeros(nbody, np.int32)
    body_dofadr = np.full(nbody, -1, np.int32)
    body_dofnum = np.zeros(nbody, np.int32)
    for ji, j in enumerate(joints):
        b = j["body"]
        if body_jntadr[b] < 0:
            body_jntadr[b] = ji
        body_jntnum[b] += 1
    for d, b in enumerate(M["dof_bodyid"]):
        if body_dofadr[b] < 0:
            body_dofadr[b] = d
        body_dofnum[b] += 1
    M["body_jntadr"], M["body_jntnum"] = body_jntadr, body_jntnum
    M["body_dofadr"], M["body_dofnum"] = body_dofadr, body_dofnum
    par = M["body_parentid"]
    weld = np.zeros(nbody, np.int32)
    root_ = np.zeros(nbody, np.int32)
    for b in range(1, nbody):
        weld[b] = b if body_jntnum[b] > 0 else weld[par[b]]
        root_[b] = b if par[b] == 0 else root_[par[b]]
    M["body_weldid"], M["body_rootid"] = weld, root_
    # dof_parentid
    dof_parent = np.full(nv, -1, np.int32)
    last_dof = np.full(nbody, -1, np.int32)   # last dof in chain ending at body
    for b in range(1, nbody):
        prev = last_dof[par[b]]
        for k in range(body_dofnum[b]):
            d = body_dofadr[b] + k
            dof_parent[d] = prev
            prev = d
        last_dof[b] = prev
    M["dof_parentid"] = dof_parent

    # qpos0 / qpos_spring
    qpos0 = np.zeros(nq)
    qspring = np.zeros(nq)
    for ji, j in enumerate(joints):
        a = jnt_qposadr[ji]
        if j["type"] == JNT_FREE:
            qpos0[a:a + 3] = bodies[j["body"]]["pos"]
            qpos0[a + 3:a + 7] = bodies[j["body"]]["quat"]
            qspring[a:a + 7] = qpos0[a:a + 7]
        else:
            qspring[a] = j["springref"]
    M["qpos0"], M["qpos_spring"] = qpos0, qspring

    # geoms
    M["geom_name"] = [g["name"] for g in geoms]
    for k in ("type", "body", "condim", "contype", "conaffinity", "priority"):
        M["geom_" + ("bodyid" if k == "body" else k)] = np.array([g[k] for g in geoms], np.int32)
    for k in ("size", "pos", "quat", "friction", "solref", "solimp"):
        M["geom_" + k] = np.array([g[k] for g in geoms])
    for k in ("margin", "gap", "solmix"):
        M["geom_" + k] = np.array([g[k] for g in geoms])
    rb = []
    for g in geoms:
        rb.append(0.0 if g["type"] == GEOM_PLANE else (g["size"][0] if g["type"] == GEOM_SPHERE else g["size"][0] + g["size"][1]))
    M["geom_rbound"] = np.array(rb)

    # body mass properties from geoms (inertiafromgeom)
    body_mass = np.zeros(nbody)
    body_ipos = np.zeros((nbody, 3))
    body_iquat = np.tile([1.0, 0, 0, 0], (nbody, 1))
    body_inertia = np.zeros((nbody, 3))
    body_ifull = np.zeros((nbody, 3, 3))
    for b in range(1, nbody):
        gs = [g for g in geoms if g["body"] == b]
        ms, Is = [], []
        for g in gs:
            m, I = geom_mass_inertia(g["type"], g["size"], g["density"])
            ms.append(m)
            Is.append(I)
        mtot = sum(ms)
        com = sum(m * g["pos"] for m, g in zip(ms, gs)) / mtot
        Ifull = np.zeros((3, 3))
        for m, I, g in zip(ms, Is, gs):
            R = quat2mat(g["quat"])
            d = g["pos"] - com
            Ifull += R @ np.diag(I) @ R.T + m * (d @ d * np.eye(3) - np.outer(d, d))
        w, V = np.linalg.eigh(Ifull)
        order = np.argsort(-w)
        w, V = w[order], V[:, order]
        if np.linalg.det(V) < 0:
            V[:, 2] = -V[:, 2]
        body_mass[b], body_ipos[b], body_inertia[b], body_iquat[b] = mtot, com, w, mat2quat(V)
        body_ifull[b] = Ifull
    M["body_mass"], M["body_ipos"], M["body_iquat"], M["body_inertia"] = body_mass, body_ipos, body_iquat, body_inertia
    M["body_inertia_full"] = body_ifull
    sub = body_mass.copy()
    for b in range(nbody - 1, 0, -1):
        sub[par[b]] += sub[b]
    M["body_subtreemass"] = sub

    # tendons (fixed)
    ten_adr, ten_num, wrap_jnt, wrap_coef, trng, tlim, tsr, tsi, tmg = [], [], [], [], [], [], [], [], []
    jname = {j["name"]: i for i, j in enumerate(joints)}
    ten_root = root.find("tendon")
    if ten_root is not None:
        for t in ten_root:
            assert t.tag == "fixed"
            a = resolve("tendon", t, "main")
            ten_adr.append(len(wrap_jnt))
            n = 0
            for w in t:
                wrap_jnt.append(jname[w.get("joint")])
                wrap_coef.append(float(w.get("coef", 1.0)))
                n += 1
            ten_num.append(n)
            r = _floats(a["range"]) if isinstance(a["range"], str) else a["range"]
            trng.append(r)
            lim = a["limited"]
            tlim.append(int(lim == "true" or (lim == "auto" and r[0] < r[1])))
            sr = _floats(a["solreflimit"]) if isinstance(a["solreflimit"], str) else a["solreflimit"]
            si = list(_floats(a["solimplimit"]) if isinstance(a["solimplimit"], str) else a["solimplimit"])
            si += list(TENDON_DEFAULTS["solimplimit"][len(si):])
            tsr.append(sr)
            tsi.append(si)
            tmg.append(float(a["margin"]))
    M["ntendon"] = len(ten_adr)
    M["tendon_adr"], M["tendon_num"] = np.array(ten_adr, np.int32), np.array(ten_num, np.int32)
    M["wrap_jnt"], M["wrap_coef"] = np.array(wrap_jnt, np.int32), np.array(wrap_coef)
    M["tendon_range"], M["tendon_limited"] = np.array(trng, float).reshape(-1, 2), np.array(tlim, np.int32)
    M["tendon_solref"], M["tendon_solimp"] = np.array(tsr, float).reshape(-1, 2), np.array(tsi, float).reshape(-1, 5)
    M["tendon_margin"] = np.array(tmg)

    # actuators (motor, joint transmission)
    act_root = root.find("actuator")
    trn, gear, crange, climited = [], [], [], []
    for a_el in act_root:
        assert a_el.tag == "motor"
        a = resolve("motor", a_el, "main")
        trn.append(jname[a_el.get("joint")])
        g = _floats(a["gear"]) if isinstance(a["gear"], str) else a["gear"]
        gear.append(g[0])
        cr = _floats(a["ctrlrange"]) if isinstance(a["ctrlrange"], str) else a["ctrlrange"]
        crange.append(cr)
        lim = a["ctrllimited"]
        climited.append(int(lim == "true" or (lim == "auto" and cr[0] < cr[1])))
    M["nu"] = len(trn)
    M["actuator_trnid"] = np.array(trn, np.int32)
    M["actuator_gear"] = np.array(gear)
    M["actuator_ctrlrange"] = np.array(crange)
    M["actuator_ctrllimited"] = np.array(climited, np.int32)

    # contact excludes (body-pair signatures)
    bname = {b["name"]: i for i, b in enumerate(bodies)}
    excl = []
    con_root = root.find("contact")
    if con_root is not None:
        for e in con_root:
            if e.tag == "exclude":
                b1, b2 = bname[e.get("body1")], bname[e.get("body2")]
                excl.append((min(b1, b2), max(b1, b2)))
    M["exclude"] = excl

    # keyframes
    keys = {}
    kroot = root.find("keyframe")
    if kroot is not None:
        for k in kroot:
            q = np.array(_floats(k.get("qpos")))
            keys[k.get("name")] = q
    M["keyframes"] = keys
    M["collision_pairs"] = collision_pairs(M)
    set_const(M)
    return M


def collision_pairs(M):
    """Static candidate geom pairs after MuJoCo's static filters, in MuJoCo's processing order.

    Filters (mj_collision / filterBodyPair): contype/conaffinity bits, same weld body,
    parent-child weld filter (world exempt), <exclude> body pairs.  Order: body pair
    (b1 < b2) ascending, then geoms of b1 x geoms of b2 in index order.
    """
    ng = M["ngeom"]
    gb = M["geom_bodyid"]
    weld = M["body_weldid"]
    par = M["body_parentid"]
    excl = set(M["exclude"])
    pairs = []
    for g1 in range(ng):
        for g2 in range(g1 + 1, ng):
            b1, b2 = int(gb[g1]), int(gb[g2])
            if not ((M["geom_contype"][g1] & M["geom_conaffinity"][g2]) or
                    (M["geom_contype"][g2] & M["geom_conaffinity"][g1])):
                continue
            w1, w2 = int(weld[b1]), int(weld[b2])
            if w1 == w2:
                continue
            wp1, wp2 = int(weld[par[w1]]) if w1 else 0, int(weld[par[w2]]) if w2 else 0
            if w1 != 0 and w2 != 0 and (w1 == wp2 or w2 == wp1):
                continue
            if (min(b1, b2), max(b1, b2)) in excl:
                continue
            lo, hi = (g1, g2) if b1 <= b2 else (g2, g1)
            pairs.append((min(b1, b2), max(b1, b2), lo, hi))
    pairs.sort()
    return np.array([(p[2], p[3]) for p in pairs], np.int32).reshape(-1, 2)


# ----------------------------------------------------------------------------- mj_setConst
def _kin_crb_qpos0(M):
    """Kinematics + com + cdof + CRB at qpos0 (numpy, fp64) for mj_setConst quantities."""
    nb, nv = M["nbody"], M["nv"]
    par = M["body_parentid"]
    q = M["qpos0"]
    xpos = np.zeros((nb, 3))
    xquat = np.zeros((nb, 4))
    xquat[0] = [1, 0, 0, 0]
    xanchor = np.zeros((M["njnt"], 3))
    xaxis = np.zeros((M["njnt"], 3))
    for b in range(1, nb):
        ja, jn = M["body_jntadr"][b], M["body_jntnum"][b]
        if jn == 1 and M["jnt_type"][ja] == JNT_FREE:
            qa = M["jnt_qposadr"][ja]
            p = q[qa:qa + 3].copy()
            qt = q[qa + 3:qa + 7] / np.linalg.norm(q[qa + 3:qa + 7])
            xanchor[ja] = p
            xaxis[ja] = M["jnt_axis"][ja]
        else:
            p = quat2mat(xquat[par[b]]) @ M["body_pos"][b] + xpos[par[b]]
            qt = quat_mul(xquat[par[b]], M["body_quat"][b])
            for j in range(ja, ja + jn):
                R = quat2mat(qt)
                xaxis[j] = R @ M["jnt_axis"][j]
                xanchor[j] = R @ M["jnt_pos"][j] + p
                ang = q[M["jnt_qposadr"][j]] - M["qpos0"][M["jnt_qposadr"][j]]
                ql = np.array([math.cos(ang / 2), *(M["jnt_axis"][j] * math.sin(ang / 2))])
                qt = quat_mul(qt, ql)
                p = xanchor[j] - quat2mat(qt) @ M["jnt_pos"][j]
        xquat[b] = qt / np.linalg.norm(qt)
        xpos[b] = p
    xmat = np.array([quat2mat(x) for x in xquat])
    xipos = np.array([xpos[b] + xmat[b] @ M["body_ipos"][b] for b in range(nb)])
    mass = M["body_mass"]
    sub = np.zeros((nb, 3))
    for b in range(nb):
        sub[b] = mass[b] * xipos[b]
    for b in range(nb - 1, 0, -1):
        sub[par[b]] += sub[b]
    subcom = np.array([sub[b] / M["body_subtreemass"][b] if M["body_subtreemass"][b] > MINVAL else xipos[b]
                       for b in range(nb)])
    cdof = np.zeros((nv, 6))
    for j in range(M["njnt"]):
        b = M["jnt_bodyid"][j]
        da = M["jnt_dofadr"][j]
        off = subcom[M["body_rootid"][b]] - xanchor[j]
        if M["jnt_type"][j] == JNT_FREE:
            for i in range(3):
                cdof[da + i, 3 + i] = 1.0
            for i in range(3):
                ax = xmat[b][:, i]
                cdof[da + 3 + i] = np.concatenate([ax, np.cross(ax, off)])
        else:
            ax = xaxis[j]
            cdof[da] = np.concatenate([ax, np.cross(ax, off)])
    # spatial inertia matrices about subtree com (6x6, motion=(w,v))
    I6 = np.zeros((nb, 6, 6))
    for b in range(1, nb):
        d = xipos[b] - subcom[M["body_rootid"][b]]
        R = xmat[b]
        Ic = R @ M["body_inertia_full"][b] @ R.T + mass[b] * (d @ d * np.eye(3) - np.outer(d, d))
        cx = np.array([[0, -d[2], d[1]], [d[2], 0, -d[0]], [-d[1], d[0], 0]])
        I6[b, :3, :3] = Ic
        I6[b, :3, 3:] = mass[b] * cx
        I6[b, 3:, :3] = -mass[b] * cx
        I6[b, 3:, 3:] = mass[b] * np.eye(3)
    crb = I6.copy()
    for b in range(nb - 1, 0, -1):
        if par[b] > 0:
            crb[par[b]] += crb[b]
    Mq = np.zeros((nv, nv))
    for i in range(nv):
        buf = crb[M["dof_bodyid"][i]] @ cdof[i]
        j = i
        while j >= 0:
            Mq[i, j] = Mq[j, i] = cdof[j] @ buf
            j = M["dof_parentid"][j]
        Mq[i, i] += M["dof_armature"][i]
    return xipos, subcom, cdof, Mq


def _body_chain(M, b):
    dofs = []
    while b > 0:
        for k in range(M["body_dofnum"][b] - 1, -1, -1):
            dofs.append(M["body_dofadr"][b] + k)
        b = M["body_parentid"][b]
    return dofs


def set_const(M):
    xipos, subcom, cdof, Mq = _kin_crb_qpos0(M)
    nv, nb = M["nv"], M["nbody"]
    Minv = np.linalg.inv(Mq)
    biw = np.zeros((nb, 2))
    for b in range(1, nb):
        jp = np.zeros((3, nv))
        jr = np.zeros((3, nv))
        off = xipos[b] - subcom[M["body_rootid"][b]]
        for d in _body_chain(M, b):
            jr[:, d] = cdof[d, :3]
            jp[:, d] = cdof[d, 3:] + np.cross(cdof[d, :3], off)
        biw[b, 0] = max(MINVAL, np.trace(jp @ Minv @ jp.T) / 3)
        biw[b, 1] = max(MINVAL, np.trace(jr @ Minv @ jr.T) / 3)
    M["body_invweight0"] = biw
    diw = np.zeros(nv)
    for j in range(M["njnt"]):
        da = M["jnt_dofadr"][j]
        if M["jnt_type"][j] == JNT_FREE:
            diw[da:da + 3] = np.trace(Minv[da:da + 3, da:da + 3]) / 3
            diw[da + 3:da + 6] = np.trace(Minv[da + 3:da + 6, da + 3:da + 6]) / 3
        else:
            diw[da] = Minv[da, da]
    M["dof_invweight0"] = diw
    tiw = np.zeros(M["ntendon"])
    for t in range(M["ntendon"]):
        J = np.zeros(nv)
        for w in range(M["tendon_adr"][t], M["tendon_adr"][t] + M["tendon_num"][t]):
            J[M["jnt_dofadr"][M["wrap_jnt"][w]]] += M["wrap_coef"][w]
        tiw[t] = J @ Minv @ J
    M["tendon_invweight0"] = tiw
    M["stat_meaninertia"] = np.trace(Mq) / nv
    M["qM0"] = Mq

"""Stage-by-stage GPU-vs-oracle comparison of one mj_step (debug helper; run on the GPU box).

usage: python tests/gpu_stage_check.py [fp64|fp32] [keyframe|noise] [nsteps]
Prints max-abs errors per pipeline stage for env 0 (xpos, cinert, cdof, M, cvel, cdof_dot,
qfrc_smooth, contacts, qacc, qpos/qvel after the step).
"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from mujocoposelearning_amd.batch import HsBatch  # noqa: E402
from mujocoposelearning_amd.model import HsModel  # noqa: E402
from oracle.oracle import Oracle  # noqa: E402

XML = os.path.join(ROOT, "tests", "golden", "humanoid.xml")


def main():
    prec = sys.argv[1] if len(sys.argv) > 1 else "fp64"
    init = sys.argv[2] if len(sys.argv) > 2 else "noise"
    nsteps = int(sys.argv[3]) if len(sys.argv) > 3 else 1
    model = HsModel(XML)
    o = Oracle(XML)
    rng = np.random.default_rng(0)
    qpos = o.M["qpos0"].copy()
    if init == "noise":
        qpos += rng.uniform(-0.01, 0.01, 28) * np.r_[1, 1, 0.1, 0, 0, 0, 0, np.ones(21)]
    else:
        qpos = o.M["keyframes"][init].copy()
    qvel = rng.uniform(-0.01, 0.01, 27)
    ctrl = rng.uniform(-1, 1, 21)
    b = HsBatch(model, 2, precision=prec)
    b.set_state(qpos=qpos, qvel=qvel, time=0.0, qacc_warmstart=0.0)
    b.set_debug(True)
    o.qpos[:] = qpos
    o.qvel[:] = qvel
    import torch
    c = torch.tensor(np.tile(ctrl, (2, 1)), dtype=torch.float32, device=b.device)
    for s in range(nsteps):
        b.physics_step(c, nsub=1)
        o.step(ctrl.astype(np.float32).astype(np.float64), 1)
    b.synchronize()
    dbg = b.get_debug()
    st = b.get_state()
    nb, nv = 17, 27
    def rep(name, gpu, ref):
        gpu, ref = np.asarray(gpu, float), np.asarray(ref, float)
        err = np.abs(gpu - ref).max() if gpu.size else 0.0
        print(f"{name:14s} maxerr {err:.3e}  (ref scale {np.abs(ref).max():.3e})")
    rep("xpos", dbg[0:nb * 3].reshape(nb, 3), o.get("xpos"))
    rep("xquat", dbg[100:100 + nb * 4].reshape(nb, 4), o.get("xquat"))
    rep("geom_xpos", dbg[4000:4000 + 60].reshape(20, 3), o.get("geom_xpos"))
    rep("xipos", dbg[4200:4200 + nb * 3].reshape(nb, 3)[1:], o.get("xipos")[1:])
    rep("com", dbg[2500:2503], o.get("subtree_com")[0])
    rep("cinert", dbg[200:200 + nb * 10].reshape(nb, 10), o.get("cinert"))
    rep("cdof", dbg[500:500 + nv * 6].reshape(nv, 6), o.get("cdof"))
    M = dbg[700:700 + 32 * 32].reshape(32, 32)[:nv, :nv]
    rep("qM", M, o.get("qM"))
    rep("cvel", dbg[1800:1800 + nb * 6].reshape(nb, 6), o.get("cvel"))
    rep("cdof_dot", dbg[2000:2000 + nv * 6].reshape(nv, 6), o.get("cdof_dot"))
    rep("qfrc_act", dbg[2280:2280 + nv], o.get("qfrc_actuator"))
    rep("qfrc_smooth", dbg[2320:2320 + nv], o.get("qfrc_smooth"))
    ncon, nefc, niter, nlim = dbg[2503], dbg[2504], dbg[2505], dbg[2506]
    print(f"ncon gpu {ncon:.0f} ref {o.d.ncon}   nefc gpu {nefc:.0f} ref {o.d.nefc}   newton iters gpu {niter:.0f} "
          f"ref {o.d.solver_niter}  nlim {nlim:.0f}")
    cons = o.contacts()
    for k in range(min(int(ncon), len(cons))):
        g = dbg[2600 + 11 * k: 2600 + 11 * k + 11]
        r = cons[k]
        print(f"  con{k}: pos err {np.abs(g[0:3] - r['pos']).max():.2e} n err {np.abs(g[3:6] - r['frame'][:3]).max():.2e}"
              f" t1 err {np.abs(g[6:9] - r['frame'][3:6]).max():.2e} dist {g[9]:.5f}/{r['dist']:.5f}")
    for r in range(min(int(nefc), o.d.nefc)):
        g = dbg[3200 + 6 * r: 3200 + 6 * r + 6]
        if r < 40:
            print(f"  row{r}: kind {g[0]:.0f} id {g[1]:.0f} D {g[2]:.4e}/{o.d.efc_D[r]:.4e} aref {g[3]:.5e}/{o.d.efc_aref[r]:.5e}"
                  f" f {g[4]:.5e}/{o.d.efc_force[r]:.5e}")
    rep("qfrc_con", dbg[2360:2360 + nv], o.get("qfrc_constraint"))
    rep("qacc", dbg[2400:2400 + nv], o.get("qacc"))
    rep("qpos(after)", st["qpos"][0], o.qpos)
    rep("qvel(after)", st["qvel"][0], o.qvel)
    rep("time", st["time"][0], o.time)
    print("env1 == env0:", np.abs(st["qpos"][1] - st["qpos"][0]).max())


if __name__ == "__main__":
    main()
